// Fused multi-tensor TF-Adam + bf16 weight repack on gfx950.
//
// ONE launch walks the flat fp32 master buffer (all 46 variables, laid out in
// backward-ready order) and per element:
//   m = b1 m + (1-b1) g ;  v = b2 v + (1-b2) g^2 ;  w -= lr_t m / (sqrt(v) + eps)
// (TF-1.x semantics, `test_dist.py:246`, SURVEY.md §2.5: eps on the
// UNcorrected sqrt(v), lr_t = lr sqrt(1-b2^t)/(1-b1^t) computed on the host),
// then writes the updated weight, rounded to bf16, into the compute layouts
// the conv kernels read:
//   conv  kernel HWIO [T][Ci][Co] -> fwd  [Co][T*Ci_pad, padded to Kpad = 64k]
//                                 -> dgrad [Ci][T*Co padded] with the taps flipped
//   tconv kernel [T][Co][Ci]      -> fwd  [(T, Co)][Ci padded]  (GEMM rows (tap, co))
//                                 -> dgrad [Ci][T*Co padded]
// With do_adam = 0 the kernel only repacks (initialisation / checkpoint load).
#include "common.h"
#include "conv_params.h"

namespace unet {


namespace {

constexpr int MAX_SEG = 128;

__global__ void __launch_bounds__(256) adam_pack_kernel(float* __restrict__ w, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v, int n_total,
                                                        const PackSeg* __restrict__ segs, int nseg, float lr_t,
                                                        float b1, float b2, float eps, float gscale, int do_adam,
                                                        const float* __restrict__ dev_scalars,
                                                        h16* __restrict__ arena) {
  // HIP-graph replay: the per-step lr_t / gradient scale come from device memory
  if (dev_scalars) {
    lr_t = dev_scalars[0];
    gscale = dev_scalars[1];
  }
  __shared__ PackSeg S[MAX_SEG];
  for (int i = threadIdx.x; i < nseg; i += blockDim.x) S[i] = segs[i];
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_total; i += gridDim.x * blockDim.x) {
    float wi = w[i];
    if (do_adam) {
      const float gi = g[i] * gscale;
      const float mi = b1 * m[i] + (1.f - b1) * gi;
      const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
      m[i] = mi;
      v[i] = vi;
      wi -= lr_t * mi / (sqrtf(vi) + eps);
      w[i] = wi;
    }
    // locate the segment (segments sorted by offset)
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (S[mid].off <= i) lo = mid; else hi = mid - 1;
    }
    const PackSeg& sg = S[lo];
    const int e = i - sg.off;
    if (sg.kind == 0 || e >= sg.n) continue;
    const h16 wb = (h16)wi;
    if (sg.kind == 1) {
      const int co = e % sg.Co;
      const int r = e / sg.Co;
      const int ci = r % sg.Ci;
      const int t = r / sg.Ci;
      if (sg.fwd_off >= 0) arena[sg.fwd_off + (long long)co * sg.rowstride + t * sg.Ci_pad + ci] = wb;
      if (sg.dg_off >= 0) arena[sg.dg_off + (long long)ci * sg.dg_rowstride + (sg.T - 1 - t) * sg.Co + co] = wb;
    } else {
      const int ci = e % sg.Ci;
      const int r = e / sg.Ci;
      const int co = r % sg.Co;
      const int t = r / sg.Co;
      if (sg.fwd_off >= 0) arena[sg.fwd_off + ((long long)t * sg.Co + co) * sg.rowstride + ci] = wb;
      if (sg.dg_off >= 0) arena[sg.dg_off + (long long)ci * sg.dg_rowstride + t * sg.Co + co] = wb;
    }
  }
}

}  // namespace

const char* adam_check(int nseg) {
  if (nseg > MAX_SEG) return "adam: too many segments";
  return nullptr;
}

hipError_t adam_pack_launch(float* w, const float* g, float* m, float* v, int n_total, const void* segs, int nseg,
                            float lr_t, float b1, float b2, float eps, float gscale, int do_adam,
                            const float* dev_scalars, void* arena, hipStream_t s) {
  int grid = (n_total + 255) / 256;
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(adam_pack_kernel, dim3(grid), dim3(256), 0, s, w, g, m, v, n_total, (const PackSeg*)segs, nseg,
                     lr_t, b1, b2, eps, gscale, do_adam, dev_scalars, (h16*)arena);
  return hipGetLastError();
}

}  // namespace unet
