// BatchNorm / GroupNorm for the native executor (the [EXT] `--norm batch|group`
// variants of the reference's conv blocks, models/reference.py::_norm:
// torch F.batch_norm(momentum=0.01, eps=1e-3) / F.group_norm(eps=1e-3)).
//
// Layout: NHWC bf16, a conv layer's pre-norm output z[N][P][C] (P pixels per sample).
// Every statistic the forward and backward need is a per-(sample, channel) pair of
// sums over pixels, so one deterministic reduction kernel serves both:
//   forward   S1 = sum z,   S2 = sum z^2
//   backward  S1 = sum g,   S2 = sum g*z      (g = dL/d(norm output), ReLU-masked)
// BatchNorm aggregates the pairs over samples per channel, GroupNorm over the
// channels of a group per sample.  With x^ = (z - mu) r the backward is
//   dz = a*g + b*z + c   with per-(n, c) coefficients
//   BN: a = gamma r, b = -gamma r^2 m2, c = -gamma r m1 + gamma r^2 mu m2
//       (m1 = mean g, m2 = mean g x^ over N*P),
//   GN: a = gamma_c r, b = -r^2 M2, c = -r M1 + r^2 mu M2
//       (M1 = mean gamma g, M2 = mean gamma g x^ over P * C/G of the group),
// and dgamma_c = sum_n r (S2 - mu S1), dbeta_c = sum_n S1.
// No float atomics anywhere: block partials are reduced in a fixed order.
#include "common.h"

namespace unet {

namespace {

constexpr int NT = 256;

// partial[(n * nbp + blk)][2][C]: sums over this block's pixels of sample n
__global__ void __launch_bounds__(NT) chan_moments_kernel(const h16* __restrict__ A, const h16* __restrict__ B,
                                                          int P, int C, int nbp, float* __restrict__ partial) {
  extern __shared__ float red[];   // [NT][2][8]
  const int n = blockIdx.x / nbp, blk = blockIdx.x - n * nbp;
  const int cpr = C / 8;                       // 16-byte chunk columns
  const int cc = threadIdx.x % cpr, rs = threadIdx.x / cpr, rstep = NT / cpr;
  const int p0 = (int)((long long)blk * P / nbp), p1 = (int)((long long)(blk + 1) * P / nbp);
  float s1[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, s2[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rs < rstep) {
    const size_t base = (size_t)n * P * C + cc * 8;
    for (int p = p0 + rs; p < p1; p += rstep) {
      float a[8], b[8];
      unpack8(*(const u32x4*)(A + base + (size_t)p * C), a);
      unpack8(*(const u32x4*)(B + base + (size_t)p * C), b);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += a[e];
        s2[e] += a[e] * b[e];
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(threadIdx.x * 2 + 0) * 8 + e] = s1[e];
    red[(threadIdx.x * 2 + 1) * 8 + e] = s2[e];
  }
  __syncthreads();
  // thread t < 2C sums its (moment, channel) over the row-threads in order
  for (int t = threadIdx.x; t < 2 * C; t += NT) {
    const int mom = t / C, c = t - mom * C;
    const int col = c / 8, e = c & 7;
    float s = 0.f;
    for (int r = 0; r < rstep; ++r) s += red[((r * cpr + col) * 2 + mom) * 8 + e];
    partial[((size_t)blockIdx.x * 2 + mom) * C + c] = s;
  }
}

// S[n][2][C] = sum over the nbp block partials of sample n
__global__ void __launch_bounds__(NT) moments_collect_kernel(const float* __restrict__ partial, int N, int C, int nbp,
                                                             float* __restrict__ S) {
  const int total = N * 2 * C;
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const int n = i / (2 * C), r = i - n * 2 * C;
    float s = 0.f;
    for (int b = 0; b < nbp; ++b) s += partial[((size_t)n * nbp + b) * 2 * C + r];
    S[i] = s;
  }
}

// Sample-slice sums of the per-sample moments (deterministic first level of every
// reduction over samples; the finalize kernels then sum <= 64 slices per channel):
//   partial[sl][0][c] = sum_{n in sl} S1[n][c]
//   partial[sl][1][c] = sum_{n in sl} S2[n][c]                      (mean == nullptr)
//                     = sum_{n in sl} rstd[n][c] (S2 - mean[n][c] S1)  (GroupNorm dgamma)
// grid: (ceil(C / 64), nsl), 256 threads = 64 channels x 4 sample lanes
__global__ void __launch_bounds__(NT) sample_slices_kernel(const float* __restrict__ S, int N, int C, int nsl,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           float* __restrict__ partial) {
  __shared__ float red[4][2][64];
  const int cl = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl, sl = blockIdx.y;
  const int n0 = (int)((long long)sl * N / nsl), n1 = (int)((long long)(sl + 1) * N / nsl);
  float a = 0.f, b = 0.f;
  if (c < C) {
    for (int n = n0 + sub; n < n1; n += 4) {
      const float s1 = S[((size_t)n * 2 + 0) * C + c], s2 = S[((size_t)n * 2 + 1) * C + c];
      a += s1;
      b += mean ? rstd[(size_t)n * C + c] * (s2 - mean[(size_t)n * C + c] * s1) : s2;
    }
  }
  red[sub][0][cl] = a;
  red[sub][1][cl] = b;
  __syncthreads();
  if (sub == 0 && c < C) {
    partial[((size_t)sl * 2 + 0) * C + c] = red[0][0][cl] + red[1][0][cl] + red[2][0][cl] + red[3][0][cl];
    partial[((size_t)sl * 2 + 1) * C + c] = red[0][1][cl] + red[1][1][cl] + red[2][1][cl] + red[3][1][cl];
  }
}

// BatchNorm per channel from the sample-slice sums (thread per channel).
//   mode 0 (forward, training): mean/rstd[c] from the batch, running stats updated
//   mode 1 (backward): coefficients a/b/c[c], dgamma/dbeta
//   mode 2 (forward, inference): mean/rstd[c] from the running stats
__global__ void __launch_bounds__(NT) bn_finalize_kernel(const float* __restrict__ part, int nsl, int C, float count,
                                                         int mode, const float* __restrict__ gamma, float eps,
                                                         float momentum, float* __restrict__ run_mean,
                                                         float* __restrict__ run_var, float* __restrict__ mean,
                                                         float* __restrict__ rstd, float* __restrict__ ca,
                                                         float* __restrict__ cb, float* __restrict__ cc,
                                                         float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                         const float* __restrict__ beta, float* __restrict__ fa,
                                                         float* __restrict__ fc) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  if (mode == 2) {
    const float mu = run_mean[c], r = rsqrtf(run_var[c] + eps);
    mean[c] = mu;
    rstd[c] = r;
    if (fa) {
      fa[c] = gamma[c] * r;
      fc[c] = beta[c] - mu * gamma[c] * r;
    }
    return;
  }
  float s1 = 0.f, s2 = 0.f;
  for (int sl = 0; sl < nsl; ++sl) {
    s1 += part[((size_t)sl * 2 + 0) * C + c];
    s2 += part[((size_t)sl * 2 + 1) * C + c];
  }
  if (mode == 0) {
    const float mu = s1 / count;
    const float var = fmaxf(s2 / count - mu * mu, 0.f);
    const float r = rsqrtf(var + eps);
    mean[c] = mu;
    rstd[c] = r;
    if (fa) {            // relu-input coefficients u = fa z + fc (fused consumers)
      fa[c] = gamma[c] * r;
      fc[c] = beta[c] - mu * gamma[c] * r;
    }
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * (count / fmaxf(count - 1.f, 1.f));
  } else {
    const float mu = mean[c], r = rstd[c], gm = gamma[c];
    const float sgx = r * (s2 - mu * s1);       // sum g x^
    dbeta[c] = s1;
    dgamma[c] = sgx;
    const float m1 = s1 / count, m2 = sgx / count;
    ca[c] = gm * r;
    cb[c] = -gm * r * r * m2;
    cc[c] = -gm * r * m1 + gm * r * r * mu * m2;
  }
}

// GroupNorm per (sample, group): one thread per (n, g).
//   mode 0: mean/rstd[n][c] (training and inference are the same)
//   mode 1: coefficients a/b/c[n][c]
__global__ void __launch_bounds__(NT) gn_finalize_kernel(const float* __restrict__ S, int N, int C, int G, float P,
                                                         int mode, const float* __restrict__ gamma, float eps,
                                                         float* __restrict__ mean, float* __restrict__ rstd,
                                                         float* __restrict__ ca, float* __restrict__ cb,
                                                         float* __restrict__ cc, const float* __restrict__ beta,
                                                         float* __restrict__ fa, float* __restrict__ fc) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i >= N * G) return;
  const int n = i / G, g = i - n * G;
  const int Cg = C / G;
  const float count = P * Cg;
  const float* S1 = S + (size_t)n * 2 * C;
  const float* S2 = S1 + C;
  if (mode == 0) {
    float s1 = 0.f, s2 = 0.f;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      s1 += S1[c];
      s2 += S2[c];
    }
    const float mu = s1 / count;
    const float r = rsqrtf(fmaxf(s2 / count - mu * mu, 0.f) + eps);
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      mean[(size_t)n * C + c] = mu;
      rstd[(size_t)n * C + c] = r;
      if (fa) {
        fa[(size_t)n * C + c] = gamma[c] * r;
        fc[(size_t)n * C + c] = beta[c] - mu * gamma[c] * r;
      }
    }
  } else {
    const float mu = mean[(size_t)n * C + g * Cg], r = rstd[(size_t)n * C + g * Cg];
    float M1 = 0.f, M2 = 0.f;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      M1 += gamma[c] * S1[c];
      M2 += gamma[c] * r * (S2[c] - mu * S1[c]);
    }
    M1 /= count;
    M2 /= count;
    for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
      ca[(size_t)n * C + c] = gamma[c] * r;
      cb[(size_t)n * C + c] = -r * r * M2;
      cc[(size_t)n * C + c] = -r * M1 + r * r * mu * M2;
    }
  }
}

// GroupNorm parameter gradients from the sample-slice sums (thread per channel)
__global__ void __launch_bounds__(NT) gn_param_grad_kernel(const float* __restrict__ part, int nsl, int C,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x * NT + threadIdx.x;
  if (c >= C) return;
  float db = 0.f, dg = 0.f;
  for (int sl = 0; sl < nsl; ++sl) {
    db += part[((size_t)sl * 2 + 0) * C + c];
    dg += part[((size_t)sl * 2 + 1) * C + c];
  }
  dgamma[c] = dg;
  dbeta[c] = db;
}

// Elementwise passes: grid (blocks per sample, N).  A thread keeps ONE 8-channel
// column (cc) for the whole pass, so its per-(n, c) coefficients are loaded once and
// the pixel loop is one 16-byte load, 8 FMAs and one 16-byte store per step (unrolled
// 4x for memory-level parallelism).  Rows of the block: rstep = NT / cpr.
constexpr int kUnroll = 4;

// y = relu(A z + B) with A = gamma rstd, B = beta - mean A (coefficients [C] or [N][C]),
// optional inverted dropout (counter hash, same stream as the conv epilogue's)
__global__ void __launch_bounds__(NT) norm_apply_kernel(const h16* __restrict__ z, int P, int C,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, int cstride,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, int relu, float drop_rate,
                                                        uint32_t seed0, const uint32_t* __restrict__ seed_ptr,
                                                        uint32_t salt, int n0, h16* __restrict__ y) {
  // n0: the launch's first sample in the whole batch (a half-batch chunk of the two-stream
  // forward): dropout hashes whole-batch element indices, like the conv epilogue's drop_idx0
  const int n = blockIdx.y, nbp = gridDim.x, blk = blockIdx.x;
  const int cpr = C / 8, rstep = NT / cpr;
  const int cc = threadIdx.x % cpr, rs = threadIdx.x / cpr;
  if (rs >= rstep) return;
  const int c0 = cc * 8;
  float A[8], B[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const size_t k = (size_t)n * cstride + c0 + e;
    A[e] = gamma[c0 + e] * rstd[k];
    B[e] = beta[c0 + e] - mean[k] * A[e];
  }
  const int p0 = (int)((long long)blk * P / nbp), p1 = (int)((long long)(blk + 1) * P / nbp);
  const size_t base = (size_t)n * P * C + c0;
  if (drop_rate > 0.f) {
    const uint32_t seed = seed_ptr ? *seed_ptr : seed0;
    const float inv_keep = 1.f / (1.f - drop_rate);
    const uint32_t thr = (uint32_t)(drop_rate * 4294967296.0);
    for (int p = p0 + rs; p < p1; p += rstep) {
      const size_t q = (size_t)(n0 + n) * P + p;
      float v[8];
      unpack8(*(const u32x4*)(z + base + (size_t)p * C), v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = fmaf(A[e], v[e], B[e]);
        if (relu) x = fmaxf(x, 0.f);
        const uint32_t h = drop_hash((uint64_t)q * C + c0 + e, seed, salt);
        v[e] = (h >= thr) ? x * inv_keep : 0.f;
      }
      *(u32x4*)(y + base + (size_t)p * C) = pack8(v);
    }
    return;
  }
  const float lo = relu ? 0.f : -INFINITY;
  int p = p0 + rs;
  for (; p + (kUnroll - 1) * rstep < p1; p += kUnroll * rstep) {
    u32x4 raw[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) raw[u] = *(const u32x4*)(z + base + (size_t)(p + u * rstep) * C);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      float v[8];
      unpack8(raw[u], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(A[e], v[e], B[e]), lo);
      *(u32x4*)(y + base + (size_t)(p + u * rstep) * C) = pack8(v);
    }
  }
  for (; p < p1; p += rstep) {
    float v[8];
    unpack8(*(const u32x4*)(z + base + (size_t)p * C), v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(A[e], v[e], B[e]), lo);
    *(u32x4*)(y + base + (size_t)p * C) = pack8(v);
  }
}

// dz = a g + b z + c  (coefficients [C] or [N][C]); U pixel steps of loads in flight per
// thread, NTL: non-temporal (read-once) loads
template <int U, bool NTL>
__global__ void __launch_bounds__(NT) norm_bwd_apply_kernel(const h16* __restrict__ g, const h16* __restrict__ z,
                                                            int P, int C, const float* __restrict__ ca,
                                                            const float* __restrict__ cb,
                                                            const float* __restrict__ ccf, int cstride,
                                                            h16* __restrict__ dz) {
  const int n = blockIdx.y, nbp = gridDim.x, blk = blockIdx.x;
  const int cpr = C / 8, rstep = NT / cpr;
  const int cc = threadIdx.x % cpr, rs = threadIdx.x / cpr;
  if (rs >= rstep) return;
  const int c0 = cc * 8;
  float a[8], b[8], c[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const size_t k = (size_t)n * cstride + c0 + e;
    a[e] = ca[k];
    b[e] = cb[k];
    c[e] = ccf[k];
  }
  const int p0 = (int)((long long)blk * P / nbp), p1 = (int)((long long)(blk + 1) * P / nbp);
  const size_t base = (size_t)n * P * C + c0;
  auto ld = [&](const h16* src, int px) {
    const u32x4* a = (const u32x4*)(src + base + (size_t)px * C);
    if constexpr (NTL) return __builtin_nontemporal_load(a);
    else return *a;
  };
  int p = p0 + rs;
  for (; p + (U - 1) * rstep < p1; p += U * rstep) {
    u32x4 rg[U], rz[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // streaming reads (read once): non-temporal, so they do not evict the freshly
      // written tensors the next kernels read from the last-level cache
      rg[u] = ld(g, p + u * rstep);
      rz[u] = ld(z, p + u * rstep);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float gv[8], zv[8];
      unpack8(rg[u], gv);
      unpack8(rz[u], zv);
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[e] = fmaf(a[e], gv[e], fmaf(b[e], zv[e], c[e]));
      *(u32x4*)(dz + base + (size_t)(p + u * rstep) * C) = pack8(gv);
    }
  }
  for (; p < p1; p += rstep) {
    float gv[8], zv[8];
    unpack8(*(const u32x4*)(g + base + (size_t)p * C), gv);
    unpack8(*(const u32x4*)(z + base + (size_t)p * C), zv);
#pragma unroll
    for (int e = 0; e < 8; ++e) gv[e] = fmaf(a[e], gv[e], fmaf(b[e], zv[e], c[e]));
    *(u32x4*)(dz + base + (size_t)p * C) = pack8(gv);
  }
}

// ---------------------------------------------------------------------------------
// Statistics reductions over partial rows (one row per conv tile / moments block):
// rows[R][2][C] -> per-channel (BatchNorm) or per-sample (GroupNorm) coefficients.
// Two fixed-order levels, no atomics; every level keeps >= 4 independent loads in
// flight per thread (the previous single-thread-per-channel finalize was a serial
// latency chain: ~19 us per launch at 64 slices).

constexpr int SL_ROWS = 32;          // rows per slice of the first level

// slices[sl][col] = sum of rows sl*SL_ROWS .. +SL_ROWS-1 (col < W = 2C);
// grid (nsl, ceil(W / 64)), 256 threads = 64 columns x 4 row lanes
__global__ void __launch_bounds__(NT) row_slices_kernel(const float* __restrict__ rows, int R, int W,
                                                        float* __restrict__ slices) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = blockIdx.y * 64 + cl, sl = blockIdx.x;
  const int r0 = sl * SL_ROWS, r1 = min(R, r0 + SL_ROWS);
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (col < W) {
#pragma unroll
    for (int u = 0; u < SL_ROWS / 16; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int r = r0 + rl + 4 * (4 * u + k);
        if (r < r1) a[k] += rows[(size_t)r * W + col];
      }
  }
  red[rl][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (rl == 0 && col < W) slices[(size_t)sl * W + col] = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
}

// sum over nsl slices of column col (fixed order: 4 lanes x unrolled accumulators)
__device__ __forceinline__ float slice_sum(const float* __restrict__ sl, int nsl, int W, int col, int rl) {
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int s = rl;
  for (; s + 12 < nsl; s += 16)
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] += sl[(size_t)(s + 4 * k) * W + col];
  for (; s < nsl; s += 4) a[0] += sl[(size_t)s * W + col];
  return (a[0] + a[1]) + (a[2] + a[3]);
}

__device__ __forceinline__ void bn_final_channel(int c, float s1, float s2, float count, int mode,
                                                 const float* __restrict__ gamma, const float* __restrict__ beta,
                                                 float eps, float momentum, float* __restrict__ run_mean,
                                                 float* __restrict__ run_var, float* __restrict__ mean,
                                                 float* __restrict__ rstd, float* __restrict__ fa,
                                                 float* __restrict__ fc, float* __restrict__ ca, float* __restrict__ cb,
                                                 float* __restrict__ cc, float* __restrict__ dgamma,
                                                 float* __restrict__ dbeta);

// BatchNorm coefficients from the slices; grid ceil(C / 32), 256 threads = 32 channels x
// 2 moments x 4 slice lanes.  mode 0: forward (batch stats, running stats, fa / fc);
// 1: backward (ca / cb / cc, dgamma / dbeta); 2: forward inference (running stats; no
// slices read); 3: plain column sums -> dbeta = S1, dgamma = S2 (GroupNorm parameter grads).
__global__ void __launch_bounds__(NT) bn_final_kernel(const float* __restrict__ slices, int nsl, int C, float count,
                                                      int mode, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, float eps, float momentum,
                                                      float* __restrict__ run_mean, float* __restrict__ run_var,
                                                      float* __restrict__ mean, float* __restrict__ rstd,
                                                      float* __restrict__ fa, float* __restrict__ fc,
                                                      float* __restrict__ ca, float* __restrict__ cb,
                                                      float* __restrict__ cc, float* __restrict__ dgamma,
                                                      float* __restrict__ dbeta) {
  __shared__ float red[4][64];
  const int t = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 32 + (t & 31), mom = t >> 5;
  if (mode != 2) {
    red[rl][t] = c < C ? slice_sum(slices, nsl, 2 * C, mom * C + c, rl) : 0.f;
    __syncthreads();
  }
  if (threadIdx.x >= 32 || c >= C) return;
  const int i = t;      // channel lane (mom 0)
  float s1 = 0.f, s2 = 0.f;
  if (mode != 2) {
    s1 = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    s2 = red[0][i + 32] + red[1][i + 32] + red[2][i + 32] + red[3][i + 32];
  }
  bn_final_channel(c, s1, s2, count, mode, gamma, beta, eps, momentum, run_mean, run_var, mean, rstd, fa, fc, ca, cb, cc,
                   dgamma, dbeta);
}

// one channel of bn_final from its column sums s1 = sum x, s2 = sum x^2 (forward) or
// s1 = sum g, s2 = sum g z (backward)
__device__ __forceinline__ void bn_final_channel(const int c, const float s1, const float s2, const float count,
                                                 const int mode, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, const float eps, const float momentum,
                                                 float* __restrict__ run_mean, float* __restrict__ run_var,
                                                 float* __restrict__ mean, float* __restrict__ rstd,
                                                 float* __restrict__ fa, float* __restrict__ fc, float* __restrict__ ca,
                                                 float* __restrict__ cb, float* __restrict__ cc,
                                                 float* __restrict__ dgamma, float* __restrict__ dbeta) {
  if (mode == 2) {
    const float mu = run_mean[c], r = rsqrtf(run_var[c] + eps);
    mean[c] = mu;
    rstd[c] = r;
    fa[c] = gamma[c] * r;
    fc[c] = beta[c] - mu * gamma[c] * r;
    return;
  }
  if (mode == 3) {
    dbeta[c] = s1;
    dgamma[c] = s2;
    return;
  }
  if (mode == 0) {
    const float mu = s1 / count;
    const float var = fmaxf(s2 / count - mu * mu, 0.f);
    const float r = rsqrtf(var + eps);
    mean[c] = mu;
    rstd[c] = r;
    fa[c] = gamma[c] * r;
    fc[c] = beta[c] - mu * gamma[c] * r;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mu;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * (count / fmaxf(count - 1.f, 1.f));
  } else {
    const float mu = mean[c], r = rstd[c], gm = gamma[c];
    const float sgx = r * (s2 - mu * s1);
    dbeta[c] = s1;
    dgamma[c] = sgx;
    const float m1 = s1 / count, m2 = sgx / count;
    ca[c] = gm * r;
    cb[c] = -gm * r * r * m2;
    cc[c] = -gm * r * m1 + gm * r * r * mu * m2;
  }
}

// Single-launch BatchNorm statistics (forward / backward / plain column sums, modes 0 / 1
// / 3).  Block (sl, cb) owns 32 channels -- lane cl < 64 is column (cl >> 5) * C + 32 cb +
// (cl & 31), i.e. both moments of its channels -- and sums rpb rows of them into slice sl;
// then the LAST of the nsl blocks of column block cb to finish -- told by the value its
// agent-scope add on counter[cb] returns -- sums the slices of those 64 columns and
// finalises its 32 channels (bn_final_channel).  The column blocks finalise in parallel
// (one block finalising every channel serialised C / 32 rounds of dependent slice loads:
// ~30 us per launch at C = 128).
// Hand-off (HIP scoped memory model, no reliance on undocumented hardware ordering):
//   * every slice value is stored by an agent-scope atomic store (written through to the
//     device-coherent level: the 8 XCDs have separate L2s, so a plain store could sit in
//     the producing XCD's L2);
//   * every thread then executes an agent-scope RELEASE fence and the workgroup barrier,
//     after which one lane does the counter add with ACQ_REL semantics (the fences of all
//     threads happen-before the add through the barrier);
//   * the last block's lane observes the final count (its add acquires every earlier
//     block's release), the barrier hands that to the block, and every thread executes an
//     agent-scope ACQUIRE fence before its agent-scope atomic loads of the slices.
// The last block resets its counter (graph replays).  Fixed summation order:
// deterministic, no float atomics.  counter: ceil(C / 32) <= 64 ints.
__global__ void __launch_bounds__(NT) bn_stats_fused_kernel(const float* __restrict__ rows, int R, int C, int rpb,
                                                            float* __restrict__ slices, int* __restrict__ counter,
                                                            float count, int mode, const float* __restrict__ gamma,
                                                            const float* __restrict__ beta, float eps, float momentum,
                                                            float* __restrict__ run_mean, float* __restrict__ run_var,
                                                            float* __restrict__ mean, float* __restrict__ rstd,
                                                            float* __restrict__ fa, float* __restrict__ fc,
                                                            float* __restrict__ ca, float* __restrict__ cb,
                                                            float* __restrict__ cc, float* __restrict__ dgamma,
                                                            float* __restrict__ dbeta) {
  __shared__ float red[4][64];
  __shared__ f32x4 red4[16][17];
  __shared__ int last;
  const int W = 2 * C;
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.y * 32 + (cl & 31);
  const bool valid = c < C;
  const int col = (cl >> 5) * C + c;
  {
    // phase 1: thread (row lane r4 = t >> 4, float4 column f = t & 15) sums float4 f of
    // the block's 64 columns (f < 8: first moments of channels 32 cb + 4 f .., f >= 8:
    // second) over rows r0 + r4, + 16, ..: 16-byte loads, 8 in flight (the scalar-load
    // version kept one float per load and ~32 dependent load rounds at level 1)
    const int f = threadIdx.x & 15, r4 = threadIdx.x >> 4;
    const int c4 = blockIdx.y * 32 + 4 * (f & 7);
    const bool v4 = c4 < C;
    const int col4 = (f >> 3) * C + c4;
    const int sl = blockIdx.x;
    const int r0 = sl * rpb, r1 = min(R, r0 + rpb);
    f32x4 a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (v4) {
      int r = r0 + r4;
      for (; r + 112 < r1; r += 128)
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += *(const f32x4*)(rows + (size_t)(r + 16 * k) * W + col4);
      for (; r < r1; r += 16) a[0] += *(const f32x4*)(rows + (size_t)r * W + col4);
    }
    red4[r4][f] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
    __syncthreads();
    if (threadIdx.x < 64) {
      // thread cl: column (cl >> 5) * C + 32 cb + (cl & 31) = element (cl & 3) of float4
      // (cl >> 5) * 8 + ((cl & 31) >> 2)
      const int ff = (cl >> 5) * 8 + ((cl & 31) >> 2), e = cl & 3;
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sm += red4[k][ff][e];
      if (valid) __hip_atomic_store(slices + (size_t)sl * W + col, sm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int done = __hip_atomic_fetch_add(counter + blockIdx.y, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = done == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int nsl = gridDim.x;
  float a[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) a[k] = 0.f;
  if (valid) {
    const float* sp = slices + col;
    int sl = rl;
    for (; sl + 60 < nsl; sl += 64)
#pragma unroll
      for (int k = 0; k < 16; ++k)
        a[k] += __hip_atomic_load(sp + (size_t)(sl + 4 * k) * W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (; sl < nsl; sl += 4) a[0] += __hip_atomic_load(sp + (size_t)sl * W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();                                     // (phase-1 red reads done)
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] += a[k + 8];
  red[rl][cl] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
  __syncthreads();
  if (threadIdx.x < 32 && valid) {
    const float s1 = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    const float s2 = red[0][cl + 32] + red[1][cl + 32] + red[2][cl + 32] + red[3][cl + 32];
    bn_final_channel(c, s1, s2, count, mode, gamma, beta, eps, momentum, run_mean, run_var, mean, rstd, fa, fc, ca,
                     cb, cc, dgamma, dbeta);
  }
  if (threadIdx.x == 0) __hip_atomic_store(counter + blockIdx.y, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// rows per phase-1 block of bn_stats_fused: a multiple of 32 rows (so at most row_slices(R)
// slices, the workspace's count) and at most min(64, 128 / column blocks) slices -- the
// launch's cost follows its block count (every block's agent-scope release and counter add):
// slice-count A/B on the BN step (r6_bench_history.md), 128 blocks for 64..128 channels,
// 64 slices at 32 channels; the 16-byte phase-1 loads cover the longer slices
int fused_rows_per_block(int R, int C) {
  const int ncb = (C + 31) / 32;
  int ms = 128 / ncb;
  ms = ms > 64 ? 64 : (ms < 8 ? 8 : ms);
  int rpb = (R + ms - 1) / ms;
  rpb = (rpb + 31) / 32 * 32;
  return rpb < 32 ? 32 : rpb;
}

// GroupNorm per sample: block n sums its rps rows (sample n) into S[2][C] in LDS, then
// one thread per group finalises.  mode 0: mean / rstd / fa / fc;  mode 1: ca / cb / cc
// and contrib[n][2][C] = {sum g, r (sum g z - mu sum g)} (summed over samples for
// dbeta / dgamma by row_slices + bn_final mode 3).
__global__ void __launch_bounds__(NT) gn_sample_kernel(const float* __restrict__ rows, int rps, int C, int G, float P,
                                                       int mode, const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       float* __restrict__ mean, float* __restrict__ rstd,
                                                       float* __restrict__ fa, float* __restrict__ fc,
                                                       float* __restrict__ ca, float* __restrict__ cb,
                                                       float* __restrict__ cc, float* __restrict__ contrib) {
  extern __shared__ float S[];   // [2C] + max([4][64], [4][G]) scratch + [2C] (mode 1)
  float* red = S + 2 * C;
  const int n = blockIdx.x, W = 2 * C;
  // column sums over the sample's rps rows: passes of CH columns x RL row lanes (wide
  // rows -- the coarse levels, few rows -- use all 256 threads on columns)
  const int CH = W >= NT ? NT : 64, RL = NT / CH;
  const int cl = threadIdx.x % CH, rl = threadIdx.x / CH;
  const float* base = rows + (size_t)n * rps * W;
  for (int c0 = 0; c0 < W; c0 += CH) {
    const int col = c0 + cl;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (col < W) {
      int r = rl;
      for (; r + 3 * RL < rps; r += 4 * RL)
#pragma unroll
        for (int k = 0; k < 4; ++k) a[k] += base[(size_t)(r + k * RL) * W + col];
      for (; r < rps; r += RL) a[0] += base[(size_t)r * W + col];
    }
    red[rl * CH + cl] = (a[0] + a[1]) + (a[2] + a[3]);
    __syncthreads();
    if (rl == 0 && col < W) {
      float sm = red[cl];
      for (int k = 1; k < RL; ++k) sm += red[k * CH + cl];
      S[col] = sm;
    }
    __syncthreads();
  }
  // per group (thread g): mean / rstd (mode 0) or the backward's M1 / M2 (mode 1) into
  // LDS, then every channel's outputs in parallel (coalesced stores; a serial per-group
  // loop over C / G channels with global loads made the level-5 finalize ~20x slower).
  // Mode 1 first forms the per-channel terms gamma S1, gamma r (S2 - mu S1) in parallel.
  const int Cg = C / G;
  const float count = P * Cg;
  float* gs = red;                                   // [G][2] (the row scratch is free now)
  float* gs2 = red + 2 * G;                          // mode 1: [G][2] = mu, r
  float* T = S + 2 * C + (4 * G > 4 * 64 ? 4 * G : 4 * 64);   // mode 1: [2][C]
  if (mode == 1) {
    for (int c = threadIdx.x; c < C; c += NT) {
      const size_t k0 = (size_t)n * C + (c / Cg) * Cg;
      const float mu = mean[k0], r = rstd[k0];
      T[c] = gamma[c] * S[c];
      T[C + c] = gamma[c] * (r * (S[C + c] - mu * S[c]));
    }
    __syncthreads();
  }
  for (int g = threadIdx.x; g < G; g += NT) {
    if (mode == 0) {
      float s1 = 0.f, s2 = 0.f;
      for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
        s1 += S[c];
        s2 += S[C + c];
      }
      const float mu = s1 / count;
      gs[2 * g] = mu;
      gs[2 * g + 1] = rsqrtf(fmaxf(s2 / count - mu * mu, 0.f) + eps);
    } else {
      float M1 = 0.f, M2 = 0.f;
      for (int c = g * Cg; c < (g + 1) * Cg; ++c) {
        M1 += T[c];
        M2 += T[C + c];
      }
      gs[2 * g] = M1 / count;
      gs[2 * g + 1] = M2 / count;
      gs2[2 * g] = mean[(size_t)n * C + g * Cg];
      gs2[2 * g + 1] = rstd[(size_t)n * C + g * Cg];
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NT) {
    const int g = c / Cg;
    const size_t k = (size_t)n * C + c;
    if (mode == 0) {
      const float mu = gs[2 * g], r = gs[2 * g + 1];
      mean[k] = mu;
      rstd[k] = r;
      fa[k] = gamma[c] * r;
      fc[k] = beta[c] - mu * gamma[c] * r;
    } else {
      const float M1 = gs[2 * g], M2 = gs[2 * g + 1], mu = gs2[2 * g], r = gs2[2 * g + 1];
      contrib[((size_t)n * 2 + 0) * C + c] = S[c];
      contrib[((size_t)n * 2 + 1) * C + c] = r * (S[C + c] - mu * S[c]);
      ca[k] = gamma[c] * r;
      cb[k] = -r * r * M2;
      cc[k] = -r * M1 + r * r * mu * M2;
    }
  }
}

int ew_grid(long long work) {
  long long b = (work + NT - 1) / NT;
  return (int)(b < 8192 ? (b < 1 ? 1 : b) : 8192);
}

}  // namespace

int norm_blocks_per_sample(int N, int P) {
  int nbp = (512 + N - 1) / N;
  const int maxb = (P + 63) / 64;
  if (nbp > maxb) nbp = maxb;
  return nbp < 1 ? 1 : nbp;
}

// grid width (blocks per sample) of the streaming passes norm_apply / norm_bwd_apply: at
// least 16 (batch 1024: 16k blocks; one block per sample left the level-2 / 3 passes 5-8 %
// slower, profiles/r5_norm_ew_grid.md)
static int ew_blocks_per_sample(int N, int P) {
  const int maxb = (P + 63) / 64;
  const int nbp = norm_blocks_per_sample(N, P);
  return nbp >= 16 ? nbp : (maxb < 16 ? maxb : 16);
}

const char* norm_check(int C, int G) {
  if (C % 8) return "norm: channels must be a multiple of 8";
  if (C > 2048) return "norm: at most 2048 channels";
  if (G > 0 && C % G) return "norm: channels not divisible by groups";
  return nullptr;
}

// stats over pixels per (sample, channel): partial [N*nbp][2][C], S [N][2][C]
hipError_t norm_moments_launch(const void* A, const void* B, int N, int P, int C, float* partial, float* S,
                               hipStream_t s) {
  const int nbp = norm_blocks_per_sample(N, P);
  UNET_LAUNCH(chan_moments_kernel, dim3(N * nbp), dim3(NT), NT * 2 * 8 * sizeof(float), s,
                     (const h16*)A, (const h16*)B, P, C, nbp, partial);
  UNET_LAUNCH(moments_collect_kernel, dim3(ew_grid((long long)N * 2 * C)), dim3(NT), 0, s, partial, N, C, nbp,
                     S);
  return launch_status();
}

// S[n][2][C] = sum of the nbp consecutive partial rows of sample n (rows written by
// a conv epilogue's per-tile statistics, conv_epilogue.h EPI_STATS / EPI_DGRAD_NORM)
hipError_t moments_collect_launch(const float* partial, int N, int C, int nbp, float* S, hipStream_t s) {
  UNET_LAUNCH(moments_collect_kernel, dim3(ew_grid((long long)N * 2 * C)), dim3(NT), 0, s, partial, N, C, nbp,
                     S);
  return launch_status();
}

int sample_slices(int N) { return N < 64 ? N : 64; }

hipError_t bn_finalize_launch(const float* S, int N, int C, float count, int mode, const float* gamma, float eps,
                              float momentum, float* run_mean, float* run_var, float* mean, float* rstd, float* ca,
                              float* cb, float* cc, float* dgamma, float* dbeta, float* partial, const float* beta,
                              float* fa, float* fc, hipStream_t s) {
  const int nsl = sample_slices(N);
  if (mode != 2)
    UNET_LAUNCH(sample_slices_kernel, dim3((C + 63) / 64, nsl), dim3(NT), 0, s, S, N, C, nsl,
                       (const float*)nullptr, (const float*)nullptr, partial);
  UNET_LAUNCH(bn_finalize_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, s, partial, nsl, C, count, mode, gamma,
                     eps, momentum, run_mean, run_var, mean, rstd, ca, cb, cc, dgamma, dbeta, beta, fa, fc);
  return launch_status();
}

hipError_t gn_finalize_launch(const float* S, int N, int C, int G, int P, int mode, const float* gamma, float eps,
                              float* mean, float* rstd, float* ca, float* cb, float* cc, float* dgamma, float* dbeta,
                              float* partial, const float* beta, float* fa, float* fc, hipStream_t s) {
  UNET_LAUNCH(gn_finalize_kernel, dim3((N * G + NT - 1) / NT), dim3(NT), 0, s, S, N, C, G, (float)P, mode,
                     gamma, eps, mean, rstd, ca, cb, cc, beta, fa, fc);
  if (mode == 1) {
    const int nsl = sample_slices(N);
    UNET_LAUNCH(sample_slices_kernel, dim3((C + 63) / 64, nsl), dim3(NT), 0, s, S, N, C, nsl,
                       (const float*)mean, (const float*)rstd, partial);
    UNET_LAUNCH(gn_param_grad_kernel, dim3((C + NT - 1) / NT), dim3(NT), 0, s, (const float*)partial, nsl, C,
                       dgamma, dbeta);
  }
  return launch_status();
}

int row_slices(int R) { return (R + SL_ROWS - 1) / SL_ROWS; }

// BatchNorm from partial rows [R][2][C]: row_slices -> bn_final (mode 2 reads no rows)
hipError_t bn_stats_launch(const float* rows, int R, int C, float count, int mode, const float* gamma,
                           const float* beta, float eps, float momentum, float* run_mean, float* run_var, float* mean,
                           float* rstd, float* fa, float* fc, float* ca, float* cb, float* cc, float* dgamma,
                           float* dbeta, float* slices, hipStream_t s) {
  if (mode == 2) {                  // inference: running statistics only
    UNET_LAUNCH(bn_final_kernel, dim3((C + 31) / 32), dim3(NT), 0, s, slices, 0, C, count, mode, gamma, beta,
                       eps, momentum, run_mean, run_var, mean, rstd, fa, fc, ca, cb, cc, dgamma, dbeta);
    return launch_status();
  }
  // one launch: slices, then the finalize by the last block of each 32-channel column
  // block; the ceil(C / 32) <= 64 counters live just past the row_slices(R) * 2C slice
  // floats of the workspace (zeroed once, reset every use)
  const int rpb = fused_rows_per_block(R, C);
  const int nsl = (R + rpb - 1) / rpb;
  int* counter = (int*)(slices + (size_t)row_slices(R) * 2 * C);
  UNET_LAUNCH(bn_stats_fused_kernel, dim3(nsl, (C + 31) / 32), dim3(NT), 0, s, rows, R, C, rpb, slices,
                     counter, count, mode, gamma, beta, eps, momentum, run_mean, run_var, mean, rstd, fa, fc, ca, cb, cc,
                     dgamma, dbeta);
  return launch_status();
}

// GroupNorm from partial rows [N * rps][2][C] (rows of sample n consecutive).  mode 1 also
// reduces the per-sample parameter-gradient contributions (work: N * 2 * C floats of
// contrib + row_slices(N) * 2 * C floats of slices) into dgamma / dbeta.
hipError_t gn_stats_launch(const float* rows, int N, int rps, int C, int G, int P, int mode, const float* gamma,
                           const float* beta, float eps, float* mean, float* rstd, float* fa, float* fc, float* ca,
                           float* cb, float* cc, float* dgamma, float* dbeta, float* work, hipStream_t s) {
  const size_t lds = (4 * C + (4 * G > 4 * 64 ? 4 * G : 4 * 64)) * sizeof(float);
  UNET_LAUNCH(gn_sample_kernel, dim3(N), dim3(NT), lds, s, rows, rps, C, G, (float)P, mode, gamma, beta, eps,
                     mean, rstd, fa, fc, ca, cb, cc, work);
  if (mode == 1) {
    // dgamma / dbeta = column sums of the per-sample contributions (fused single launch)
    float* slices = work + (size_t)N * 2 * C;
    const int rpb = fused_rows_per_block(N, C);
    const int nsl = (N + rpb - 1) / rpb;
    int* counter = (int*)(slices + (size_t)row_slices(N) * 2 * C);
    UNET_LAUNCH(bn_stats_fused_kernel, dim3(nsl, (C + 31) / 32), dim3(NT), 0, s, (const float*)work, N, C,
                       rpb, slices, counter, 1.f, 3, gamma, beta, eps, 0.f, (float*)nullptr, (float*)nullptr,
                       (float*)nullptr, (float*)nullptr, (float*)nullptr, (float*)nullptr, (float*)nullptr,
                       (float*)nullptr, (float*)nullptr, dgamma, dbeta);
  }
  return launch_status();
}

// chan_moments only (no collect): partial rows [N * nbp][2][C] for bn/gn_stats
hipError_t norm_rows_launch(const void* A, const void* B, int N, int P, int C, float* rows, hipStream_t s) {
  const int nbp = norm_blocks_per_sample(N, P);
  UNET_LAUNCH(chan_moments_kernel, dim3(N * nbp), dim3(NT), NT * 2 * 8 * sizeof(float), s, (const h16*)A,
                     (const h16*)B, P, C, nbp, rows);
  return launch_status();
}

hipError_t norm_apply_launch(const void* z, int N, int P, int C, const float* mean, const float* rstd, int cstride,
                             const float* gamma, const float* beta, int relu, float drop_rate, uint32_t seed,
                             const uint32_t* seed_ptr, uint32_t salt, int n0, void* y, hipStream_t s) {
  UNET_LAUNCH(norm_apply_kernel, dim3(ew_blocks_per_sample(N, P), N), dim3(NT), 0, s, (const h16*)z, P, C,
                     mean, rstd, cstride, gamma, beta, relu, drop_rate, seed, seed_ptr, salt, n0, (h16*)y);
  return launch_status();
}

hipError_t norm_bwd_apply_launch(const void* g, const void* z, int N, int P, int C, const float* ca, const float* cb,
                                 const float* cc, int cstride, void* dz, hipStream_t s) {
  // unroll 4 with non-temporal loads: unroll 8 and / or plain loads measured equal or up to
  // 20 % slower (profiles/r5_norm_ew_grid.md)
  UNET_LAUNCH((norm_bwd_apply_kernel<4, true>), dim3(ew_blocks_per_sample(N, P), N), dim3(NT), 0, s,
              (const h16*)g, (const h16*)z, P, C, ca, cb, cc, cstride, (h16*)dz);
  return launch_status();
}

}  // namespace unet
