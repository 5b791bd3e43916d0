// Composite transposed-conv backward (2D): the gradient through the 2x2 stride-2
// transposed conv u = tconv(b) and the 3x3 'same' conv z = conv_a([u, skip]) that
// consumes it, without materialising du = dL/du.
//
// Forward (conv_epilogue.h pixel shuffle, adam.hip layouts):
//   u[2h + a][2w + c'] [c] = sum_k b[h][w][k] Wt[2a + c'][c][k] + bt[c]     Wt: [4][C][K]
//   z[y][x][o]            = sum_{dh,dw,c} u[y + dh - 1][x + dw - 1][c] Wa[dh][dw][c][o] + ...
//                                                                        Wa: HWIO [3][3][Ca][O]
// Data gradient.  Writing the fine row 2h + a - dh + 1 as 2 (h + Th - 1) + a' (a' in {0,1},
// Th in 0..2) turns db into a coarse 3x3 conv of the space-to-depth image of dz
// (4 O channels (a', b', o)):
//   db[h][w][k] = sum_{T, a', b', o} S2D(dz)[h + Th - 1][w + Tw - 1][a', b', o] Wg[T][a', b', o][k]
//   Wg[T][a', b', o][k] = sum_{a, b, c} Wa[dh][dw][c][o] Wt[2a + b][c][k],
//       dh = a - a' + 3 - 2 Th,  dw = b - b' + 3 - 2 Tw   (terms with dh, dw outside 0..2 vanish)
// Phase group (a', b') only has the taps Th in {1 - a', 2 - a'}, Tw in {1 - b', 2 - b'}:
// conv_win.h XF 4 skips the other five.  tconv_compose writes Wg in the row-window
// forward layout [K][9 * 4 O] from the fp32 masters (once per step).
// Weight / bias gradients.  With H[sh][sw][o][k] = sum_{h,w} dz[2h + sh - 1][2w + sw - 1][o] b[h][w][k]
// (the generic split-K wgrad with 4x4 taps, stride 2, pad 1, bias mode 2 -> per-tap sums
// Bs[sh][sw][o] = sum_{h,w} dz[2h + sh - 1][2w + sw - 1][o]):
//   dWt[2a + b][c][k] = sum_{dh,dw,o} Wa[dh][dw][c][o] H[a - dh + 2][b - dw + 2][o][k]
//   dbt[c]            = sum_{dh,dw,o} Wa[dh][dw][c][o] sum_{a,b} Bs[a - dh + 2][b - dw + 2][o]
// (tconv_chain, after the slab reduction).  Reference: the gradients TF forms for the
// Conv2DTranspose -> concatenate -> Conv2D decoder step (unet model
// builder `upsampling / concatenate` blocks).
#include "common.h"

namespace unet {

namespace {

__global__ void __launch_bounds__(256) tconv_compose_kernel(const float* __restrict__ wt, const float* __restrict__ wa,
                                                            int C, int K, int O, int Ca, int rowstride,
                                                            h16* __restrict__ out) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int n = K * rowstride;
  if (idx >= n) return;
  const int k = idx / rowstride, col = idx - k * rowstride;
  float acc = 0.f;
  if (col < 36 * O) {
    const int o = col % O, g = (col / O) & 3, T = col / (4 * O);
    const int ap = g >> 1, bp = g & 1, Th = T / 3, Tw = T - 3 * Th;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int dh = a - ap + 3 - 2 * Th;
      if (dh < 0 || dh > 2) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int dw = b - bp + 3 - 2 * Tw;
        if (dw < 0 || dw > 2) continue;
        const float* wap = wa + (size_t)(dh * 3 + dw) * Ca * O + o;
        const float* wtp = wt + (size_t)(2 * a + b) * C * K + k;
#pragma unroll 8
        for (int c = 0; c < C; ++c) acc = fmaf(wap[(size_t)c * O], wtp[(size_t)c * K], acc);
      }
    }
  }
  out[idx] = f2h(acc);
}

// blocks [0, nw): dWt elements (t, c, k), k fastest, 4 partial sums over o per element
// (lane bits 4-5: the o quarter, combined by two xor shuffles) -- 4x the threads and a
// quarter of the dependent-load chain of one thread per element (the kernel is latency-
// bound: a few MB of operands); blocks [nw, nw + C): dbt[c], the 9 O products of one c
// summed by the whole block
__global__ void __launch_bounds__(256) tconv_chain_kernel(const float* __restrict__ Hs, const float* __restrict__ bs,
                                                          const float* __restrict__ wa, int C, int K, int O, int Ca,
                                                          int nw, float* __restrict__ dwt, float* __restrict__ dbt) {
  if ((int)blockIdx.x < nw) {
    const int lane = threadIdx.x & 63, part = lane >> 4;
    const int idx = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16 + (lane & 15);
    const bool ok = idx < 4 * C * K;                 // (K % 16 == 0: whole 16-lane groups)
    const int e = ok ? idx : 0;
    const int k = e % K, c = (e / K) % C, t = e / (C * K);
    const int a = t >> 1, b = t & 1, oq = O >> 2, o0 = part * oq;
    float acc = 0.f;
    for (int dh = 0; dh < 3; ++dh)
      for (int dw = 0; dw < 3; ++dw) {
        const float* wap = wa + ((size_t)(dh * 3 + dw) * Ca + c) * O + o0;
        const float* hp = Hs + ((size_t)((a - dh + 2) * 4 + (b - dw + 2)) * O + o0) * K + k;
#pragma unroll 4
        for (int o = 0; o < oq; ++o) acc = fmaf(wap[o], hp[(size_t)o * K], acc);
      }
    acc += __shfl_xor(acc, 16, 64);
    acc += __shfl_xor(acc, 32, 64);
    if (ok && part == 0) dwt[idx] = acc;
    return;
  }
  __shared__ float red[256];
  const int c = blockIdx.x - nw;
  float acc = 0.f;
  for (int i = threadIdx.x; i < 9 * O; i += 256) {
    const int tap = i / O, o = i - tap * O, dh = tap / 3, dw = tap - 3 * dh;
    float sb = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) sb += bs[((a - dh + 2) * 4 + (b - dw + 2)) * O + o];
    acc = fmaf(wa[((size_t)tap * Ca + c) * O + o], sb, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st > 0; st >>= 1) {
    if ((int)threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
    __syncthreads();
  }
  if (threadIdx.x == 0) dbt[c] = red[0];
}

// Weight gradient of the consumer conv when u was never formed (composite forward):
// dWa[dh][dw][c][o] (HWIO) = sum_{a,b} sum_k Wt[2a + b][c][k] H[a - dh + 2][b - dw + 2][o][k]
//                          + bt[c] Bs[a - dh + 2][b - dw + 2][o]       for the u rows c < C,
// and the skip rows c >= C copied from their own (skip-only) weight gradient skg [9][Cs][O].
__global__ void __launch_bounds__(256) tconv_chain_wa_kernel(const float* __restrict__ Hs, const float* __restrict__ bs,
                                                             const float* __restrict__ wt, const float* __restrict__ bt,
                                                             const float* __restrict__ skg, int C, int K, int O,
                                                             int Ca, float* __restrict__ dwa) {
  // 16 lanes per output element: the K-long dot products read contiguous 64-byte runs
  const int idx = blockIdx.x * 16 + (threadIdx.x >> 4), l16 = threadIdx.x & 15;
  if (idx >= 9 * Ca * O) return;                    // (whole 16-lane groups)
  const int o = idx % O, c = (idx / O) % Ca, tap = idx / (Ca * O);
  if (c >= C) {
    if (l16 == 0) dwa[idx] = skg[((size_t)tap * (Ca - C) + (c - C)) * O + o];
    return;
  }
  const int dh = tap / 3, dw = tap - 3 * dh;
  float acc = 0.f, bsum = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int sl = (a - dh + 2) * 4 + (b - dw + 2);
      const float* hp = Hs + ((size_t)sl * O + o) * K;
      const float* wtp = wt + ((size_t)(2 * a + b) * C + c) * K;
#pragma unroll 4
      for (int k = l16; k < K; k += 16) acc = fmaf(wtp[k], hp[k], acc);
      bsum += bs[sl * O + o];
    }
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (l16 == 0) dwa[idx] = fmaf(bt[c], bsum, acc);
}

}  // namespace

const char* tconv_fused_check(int C, int K, int O, int Ca) {
  if (C <= 0 || K <= 0 || O <= 0 || Ca < C) return "tconv_fused: bad channel counts";
  if (O % 32 || K % 32) return "tconv_fused: O and K must be multiples of 32";
  return nullptr;
}

hipError_t tconv_compose_launch(const float* wt, const float* wa, int C, int K, int O, int Ca, int rowstride,
                                void* out, hipStream_t s) {
  const int n = K * rowstride;
  UNET_LAUNCH(tconv_compose_kernel, dim3((n + 255) / 256), dim3(256), 0, s, wt, wa, C, K, O, Ca, rowstride,
                     (h16*)out);
  return launch_status();
}

hipError_t tconv_chain_launch(const float* Hs, const float* bs, const float* wa, int C, int K, int O, int Ca,
                              float* dwt, float* dbt, const float* wt, const float* bt, const float* skg, float* dwa,
                              hipStream_t s) {
  const int nw = (4 * C * K + 63) / 64;            // 64 elements (x 4 o quarters) per block
  UNET_LAUNCH(tconv_chain_kernel, dim3(nw + C), dim3(256), 0, s, Hs, bs, wa, C, K, O, Ca, nw, dwt, dbt);
  if (dwa) {
    const int n = 9 * Ca * O;
    UNET_LAUNCH(tconv_chain_wa_kernel, dim3((n + 15) / 16), dim3(256), 0, s, Hs, bs, wt, bt, skg, C, K, O,
                       Ca, dwa);
  }
  return launch_status();
}

}  // namespace unet
