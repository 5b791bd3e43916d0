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
// Every master element belongs to exactly one segment (kind 0 for biases and
// variables without compute copies), so the tiles cover the whole buffer once.
#include "common.h"
#include "conv_params.h"

namespace unet {


namespace {

constexpr int MAX_SEG = 128;
constexpr int TB = 32;          // transpose tile edge (conv / tconv kernel segments)

// Work unit of the launch: a kind-0 segment (biases) is cut into 1024-element runs; a
// kernel segment [T][R][C] (C fastest in the master) into (tap, 32 x 32) tiles.
__device__ __forceinline__ int seg_tiles(const PackSeg& sg) {
  if (sg.kind == 0) return (sg.n + 1023) / 1024;
  const int R = sg.kind == 1 ? sg.Ci : sg.Co, C = sg.kind == 1 ? sg.Co : sg.Ci;
  return sg.T * ((R + TB - 1) / TB) * ((C + TB - 1) / TB);
}

__device__ __forceinline__ void adam1(float& w, float g, float& m, float& v, float lr_t, float b1, float b2,
                                      float eps) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  w -= lr_t * m / (sqrtf(v) + eps);
}

// The 16-bit compute copies are transposes of each other: for a conv kernel (HWIO,
// [T][Ci][Co]) the dgrad copy [Ci][T*Co] is contiguous along Co like the master, the
// forward copy [Co][T*Ci] along Ci; for a tconv kernel ([T][Co][Ci]) the forward copy
// runs along Ci and the dgrad copy along Co.  A tile updates 32 x 32 master elements
// with coalesced 16-byte accesses, stores the copy that runs along the master's
// fastest axis directly and the other one through an LDS transpose -- every 16-bit
// store is a contiguous 8-byte run (the element-wise version scattered 2-byte stores
// with a row stride of up to 9 KB, 2x the ideal time).
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
  __shared__ int first[MAX_SEG + 1];          // exclusive prefix of work units per segment
  __shared__ h16 tr[TB][TB + 2];              // transpose tile [c][r]
  const int tid = threadIdx.x;
  for (int i = tid; i < nseg; i += blockDim.x) S[i] = segs[i];
  __syncthreads();
  if (tid == 0) {
    int acc = 0;
    for (int i = 0; i < nseg; ++i) {
      first[i] = acc;
      acc += seg_tiles(S[i]);
    }
    first[nseg] = acc;
  }
  __syncthreads();
  const int total = first[nseg];
  for (int u = blockIdx.x; u < total; u += gridDim.x) {
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (first[mid] <= u) lo = mid; else hi = mid - 1;
    }
    const PackSeg sg = S[lo];
    const int k = u - first[lo];
    if (sg.kind == 0) {
      for (int e = tid; e < 1024; e += 256) {
        const int i = sg.off + k * 1024 + e;
        if (k * 1024 + e >= sg.n || !do_adam) continue;
        float wi = w[i], mi = m[i], vi = v[i];
        adam1(wi, g[i] * gscale, mi, vi, lr_t, b1, b2, eps);
        w[i] = wi;
        m[i] = mi;
        v[i] = vi;
      }
      continue;
    }
    const bool conv = sg.kind == 1;
    const int R = conv ? sg.Ci : sg.Co, C = conv ? sg.Co : sg.Ci;
    const int nrb = (R + TB - 1) / TB, ncb = (C + TB - 1) / TB;
    const int t = k / (nrb * ncb), rc = k - t * nrb * ncb;
    const int r0 = (rc / ncb) * TB, c0 = (rc % ncb) * TB;
    // phase 1: thread -> (row r0 + tid / 8, columns c0 + 4 (tid % 8) .. + 3)
    const int r = r0 + (tid >> 3), c = c0 + 4 * (tid & 7);
    float wv[4] = {0.f, 0.f, 0.f, 0.f};
    const bool vec = (C % 4) == 0 && (sg.off % 4) == 0;
    const int base = sg.off + (t * R + r) * C + c;
    if (r < R) {
      if (vec && c < C) {
        f32x4 w4 = *(const f32x4*)(w + base);
        if (do_adam) {
          const f32x4 g4 = *(const f32x4*)(g + base);
          f32x4 m4 = *(const f32x4*)(m + base), v4 = *(const f32x4*)(v + base);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float we = w4[e], me = m4[e], ve = v4[e];
            adam1(we, g4[e] * gscale, me, ve, lr_t, b1, b2, eps);
            w4[e] = we;
            m4[e] = me;
            v4[e] = ve;
          }
          *(f32x4*)(w + base) = w4;
          *(f32x4*)(m + base) = m4;
          *(f32x4*)(v + base) = v4;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) wv[e] = w4[e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wv[e] = 0.f;
          if (c + e >= C) continue;
          float wi = w[base + e];
          if (do_adam) {
            float mi = m[base + e], vi = v[base + e];
            adam1(wi, g[base + e] * gscale, mi, vi, lr_t, b1, b2, eps);
            w[base + e] = wi;
            m[base + e] = mi;
            v[base + e] = vi;
          }
          wv[e] = wi;
        }
      }
      // the copy contiguous along C: conv -> dgrad [Ci][(T-1-t) Co + co], tconv -> fwd [(t, co)][ci]
      const long long doff = conv ? (sg.dg_off >= 0 ? sg.dg_off + (long long)r * sg.dg_rowstride + (sg.T - 1 - t) * sg.Co + c : -1)
                                  : (sg.fwd_off >= 0 ? sg.fwd_off + ((long long)t * sg.Co + r) * sg.rowstride + c : -1);
      if (doff >= 0) {
        if ((doff & 3) == 0 && c + 3 < C) {
          u32x2 pk;
          pk[0] = pack2h(wv[0], wv[1]);
          pk[1] = pack2h(wv[2], wv[3]);
          *(u32x2*)(arena + doff) = pk;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (c + e < C) arena[doff + e] = f2h(wv[e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) tr[4 * (tid & 7) + e][tid >> 3] = f2h(wv[e]);
    __syncthreads();
    // phase 2: thread -> (column c0 + tid / 8, rows r0 + 4 (tid % 8) .. + 3)
    const int c2 = c0 + (tid >> 3), r2 = r0 + 4 * (tid & 7);
    // the copy contiguous along R: conv -> fwd [Co][t Ci_pad + ci], tconv -> dgrad [Ci][t Co + co]
    const long long toff = conv ? (sg.fwd_off >= 0 ? sg.fwd_off + (long long)c2 * sg.rowstride + t * sg.Ci_pad + r2 : -1)
                                : (sg.dg_off >= 0 ? sg.dg_off + (long long)c2 * sg.dg_rowstride + t * sg.Co + r2 : -1);
    if (toff >= 0 && c2 < C) {
      const h16* src = &tr[tid >> 3][4 * (tid & 7)];
      if ((toff & 3) == 0 && r2 + 3 < R) {
        u32x2 pk;
        pk[0] = __builtin_bit_cast(uint32_t, (h16x2){src[0], src[1]});
        pk[1] = __builtin_bit_cast(uint32_t, (h16x2){src[2], src[3]});
        *(u32x2*)(arena + toff) = pk;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r2 + e < R) arena[toff + e] = src[e];
      }
    }
    __syncthreads();              // tr is rewritten by the next tile
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
  // work units (~n_total / 1024) are dealt over a fixed grid; blocks past the last
  // unit exit at once
  int grid = (n_total / 1024 + 255) / 256 * 256;
  if (grid > 4096) grid = 4096;
  if (grid < 256) grid = 256;
  UNET_LAUNCH(adam_pack_kernel, dim3(grid), dim3(256), 0, s, w, g, m, v, n_total, (const PackSeg*)segs, nseg,
                     lr_t, b1, b2, eps, gscale, do_adam, dev_scalars, (h16*)arena);
  return launch_status();
}

}  // namespace unet
