// Memory-bound kernels of the UNet step on gfx950: all 16-byte vectorised
// (8 x bf16 per lane, cdna_hip_programming.md §6 Guideline 13).
//
//  * cast_input: fp32 NHWC image -> bf16 with channel padding (first layer reads 4/8 channels)
//  * maxpool2_fwd / maxpool2_bwd: 2x2(x2) max-pool (`model.py:53-69`); the backward
//    routes to the FIRST maximum of each window (TF MaxPoolGrad tie rule) and
//    fuses the add of the skip-connection gradient coming from the decoder
//    (the concat's dgrad), so the encoder output gradient is written once.  The
//    forward can record the argmax per channel (2-3 bit codes) for the backward.
//    The pooled tensor is always a ReLU output (convNb), and the backward applies
//    that ReLU's derivative too: a window whose maximum is 0 (every input clipped)
//    routes nothing (TF: relu'(0) = 0), so the encoder gradient needs no extra mask.
//  * upsample2_bwd: 2x2(x2) sum of the full-res gradient of the folded nearest
//    upsample (`model.py:76-109` upsampling variant), masked by the source's ReLU.
#include "common.h"

namespace unet {

namespace {

__device__ __forceinline__ uint32_t bf_pos_mask(uint32_t w) {
  const uint32_t lo = w & 0xffffu, hi = w >> 16;
  return ((lo != 0u && !(lo & 0x8000u)) ? 0xffffu : 0u) | ((hi != 0u && !(hi & 0x8000u)) ? 0xffff0000u : 0u);
}

__global__ void __launch_bounds__(256) cast_input_kernel(const float* __restrict__ x, int P, int Cin, int Cpad,
                                                         h16* __restrict__ y) {
  const int total = P * Cpad;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int p = i / Cpad, c = i - p * Cpad;
    y[i] = (h16)(c < Cin ? x[(size_t)p * Cin + c] : 0.f);
  }
}

// Batch load from the HBM-resident training set (trainer hot path): sample idx[b] of
// x_all [Nall][P][Cin] and y_all [Nall][P] (fp32) -> the channel-padded 16-bit input
// [B][P][Cpad] (pad channels written as zeros) and the 16-bit target [B][P].  One
// launch replaces index_select + cast copies; one thread per pixel.
__global__ void __launch_bounds__(256) gather_batch_kernel(const float* __restrict__ x_all,
                                                           const float* __restrict__ y_all,
                                                           const long long* __restrict__ idx, int B, int P, int Cin,
                                                           int Cpad, h16* __restrict__ xb, h16* __restrict__ tb) {
  const long long total = (long long)B * P;
  auto one = [&](const size_t i, const int b, const int p) {
    const size_t s = (size_t)idx[b] * P + p;
    const float* src = x_all + s * Cin;
    h16* dst = xb + i * Cpad;
    if (Cin == 4 && Cpad == 4) {
      const float4 v = *(const float4*)src;
      u32x2 o;
      o[0] = pack2h(v.x, v.y);
      o[1] = pack2h(v.z, v.w);
      *(u32x2*)dst = o;
    } else {
      for (int c = 0; c < Cpad; ++c) dst[c] = (h16)(c < Cin ? src[c] : 0.f);
    }
    tb[i] = (h16)y_all[s];
  };
  if (total <= 0x7fffffffLL) {
    // 32-bit index math (a 64-bit division per pixel dominated this streaming pass)
    const int n = (int)total;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
      const int b = i / P;
      one((size_t)i, b, i - b * P);
    }
    return;
  }
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(i / P);
    one((size_t)i, b, (int)(i - (long long)b * P));
  }
}

// Pooling thread map: one thread = one pooled pixel x 8 channels, 32-bit index math
// (the 64-bit divisions of a long-long decomposition dominated these memory-bound
// kernels).  Window corner k = (dz, dy, dx) -> input pixel base + k-offset.
struct PoolIdx {
  int cc;        // 8-channel chunk
  int base;      // input pixel of window corner (0, 0, 0)
};
__device__ __forceinline__ PoolIdx pool_idx(int i, int cpp, int OW, int OH, int H, int W, int dims3) {
  PoolIdx r;
  r.cc = i % cpp;
  const int t = i / cpp;
  const int ow = t % OW, rr = t / OW;
  const int ndo = rr / OH, oh = rr - ndo * OH;
  const int dbase = dims3 ? 2 * ndo : ndo;           // n * D + 2 od  (3D: D = 2 OD)
  r.base = (dbase * H + 2 * oh) * W + 2 * ow;
  return r;
}

// y = max over the window; code (optional): per channel the index of the FIRST
// maximum (2 bits in 2D, 3 bits in 3D) packed into one 32-bit word per thread, so
// the backward routes the gradient without re-reading the 4-8x larger input
__global__ void __launch_bounds__(256) maxpool2_fwd_kernel(const h16* __restrict__ x, int N, int D, int H, int W,
                                                           int C, int dims3, h16* __restrict__ y,
                                                           uint32_t* __restrict__ code) {
  const int OD = dims3 ? D / 2 : 1, OH = H / 2, OW = W / 2;
  const int cpp = C / 8;
  const int total = N * OD * OH * OW * cpp;
  const int nz = dims3 ? 2 : 1;
  const int bits = dims3 ? 3 : 2;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const PoolIdx pi = pool_idx(i, cpp, OW, OH, H, W, dims3);
    float m[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      m[e] = -INFINITY;
      arg[e] = 0;
    }
    for (int dz = 0; dz < nz; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          const int k = dz * 4 + dy * 2 + dx;
          const int pix = pi.base + (dz * H + dy) * W + dx;
          const u32x4 v = *(const u32x4*)(x + (size_t)pix * C + pi.cc * 8);
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (f[e] > m[e]) {
              m[e] = f[e];
              arg[e] = k;
            }
        }
    *(u32x4*)(y + (size_t)i * 8) = pack8(m);
    if (code) {
      // bits [bits*e ..): argmax of channel e; bit 24 + e: its maximum is positive
      uint32_t w = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) w |= ((uint32_t)arg[e] << (bits * e)) | ((m[e] > 0.f ? 1u : 0u) << (24 + e));
      code[i] = w;
    }
  }
}

// Normalisation + 2x2 max-pool of a convNb output in one pass: y = relu(fa z + fc) of
// every window pixel is stored (the decoder's skip reads it), and the pooled tensor and
// the argmax codes of maxpool2_fwd_kernel are formed from the same registers -- the
// pool's re-read of y disappears.  fa / fc: [C] (BatchNorm, cstride 0) or [N][C]
// (GroupNorm, cstride C); sample of pooled item i is i / (OD OH OW cpp).
template <bool D3>
__global__ void __launch_bounds__(256) norm_pool_kernel(const h16* __restrict__ z, const float* __restrict__ fa,
                                                        const float* __restrict__ fc, int cstride, int N, int D,
                                                        int H, int W, int C, h16* __restrict__ y,
                                                        h16* __restrict__ py, uint32_t* __restrict__ code) {
  constexpr int NK = D3 ? 8 : 4, BITS = D3 ? 3 : 2;
  const int OD = D3 ? D / 2 : 1, OH = H / 2, OW = W / 2;
  const int cpp = C / 8;
  const int per_n = OD * OH * OW * cpp;
  const int total = N * per_n;
  const int step = gridDim.x * blockDim.x;
  // the window's NK input vectors of two grid-stride items are loaded before either is
  // used (the per-item chain load -> normalise -> store is otherwise exposed)
  auto load = [&](const int i, u32x4 (&raw)[NK]) {
    const PoolIdx pi = pool_idx(i, cpp, OW, OH, H, W, D3);
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int dz = k >> 2, dy = (k >> 1) & 1, dx = k & 1;
      raw[k] = *(const u32x4*)(z + (size_t)(pi.base + (dz * H + dy) * W + dx) * C + pi.cc * 8);
    }
  };
  auto finish = [&](const int i, const u32x4 (&raw)[NK]) {
    const PoolIdx pi = pool_idx(i, cpp, OW, OH, H, W, D3);
    const size_t cb = (size_t)(i / per_n) * cstride + pi.cc * 8;
    float A[8], B[8], m[8];
    uint32_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      A[e] = fa[cb + e];
      B[e] = fc[cb + e];
      m[e] = -INFINITY;
      arg[e] = 0u;
    }
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int dz = k >> 2, dy = (k >> 1) & 1, dx = k & 1;
      float f[8];
      unpack8(raw[k], f);
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(A[e], f[e], B[e]), 0.f);
      const u32x4 v = pack8(f);
      // (y == nullptr: the activation's readers normalise z on load -- only the pool is stored)
      if (y) *(u32x4*)(y + (size_t)(pi.base + (dz * H + dy) * W + dx) * C + pi.cc * 8) = v;
      unpack8(v, f);                                 // the stored (rounded) activation
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool gt = f[e] > m[e];                 // first maximum wins ties
        m[e] = gt ? f[e] : m[e];
        arg[e] = gt ? (uint32_t)k : arg[e];
      }
    }
    *(u32x4*)(py + (size_t)i * 8) = pack8(m);
    uint32_t w = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) w |= (arg[e] << (BITS * e)) | ((m[e] > 0.f ? 1u : 0u) << (24 + e));
    code[i] = w;
  };
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + step < total; i += 2 * step) {
    u32x4 r0[NK], r1[NK];
    load(i, r0);
    load(i + step, r1);
    finish(i, r0);
    finish(i + step, r1);
  }
  if (i < total) {
    u32x4 r0[NK];
    load(i, r0);
    finish(i, r0);
  }
}

// dx[window] = (first argmax ? dy : 0) + skip_grad (optional); argmax recomputed
// from the forward input x
__global__ void __launch_bounds__(256) maxpool2_bwd_kernel(const h16* __restrict__ x, const h16* __restrict__ dy,
                                                           const h16* __restrict__ skip, int N, int D, int H, int W,
                                                           int C, int dims3, h16* __restrict__ dx) {
  const int OD = dims3 ? D / 2 : 1, OH = H / 2, OW = W / 2;
  const int cpp = C / 8;
  const int total = N * OD * OH * OW * cpp;
  const int nz = dims3 ? 2 : 1;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const PoolIdx pi = pool_idx(i, cpp, OW, OH, H, W, dims3);
    float g[8];
    unpack8(*(const u32x4*)(dy + (size_t)i * 8), g);
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      arg[e] = 0;
    }
    for (int dz = 0; dz < nz; ++dz)
#pragma unroll
      for (int dyy = 0; dyy < 2; ++dyy)
#pragma unroll
        for (int dxx = 0; dxx < 2; ++dxx) {
          const int k = dz * 4 + dyy * 2 + dxx;
          const int pix = pi.base + (dz * H + dyy) * W + dxx;
          float f[8];
          unpack8(*(const u32x4*)(x + (size_t)pix * C + pi.cc * 8), f);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (f[e] > best[e]) {
              best[e] = f[e];
              arg[e] = k;
            }
        }
    for (int dz = 0; dz < nz; ++dz)
#pragma unroll
      for (int dyy = 0; dyy < 2; ++dyy)
#pragma unroll
        for (int dxx = 0; dxx < 2; ++dxx) {
          const int k = dz * 4 + dyy * 2 + dxx;
          const size_t off = (size_t)(pi.base + (dz * H + dyy) * W + dxx) * C + pi.cc * 8;
          float o[8];
          if (skip) {
            unpack8(*(const u32x4*)(skip + off), o);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (arg[e] == k && best[e] > 0.f) o[e] += g[e];
          *(u32x4*)(dx + off) = pack8(o);
        }
  }
}

// the same from the forward's argmax codes: reads 4 bytes per 8 pooled channels
// instead of the 4 (8 in 3D) input pixels
__global__ void __launch_bounds__(256) maxpool2_bwd_code_kernel(const uint32_t* __restrict__ code,
                                                                const h16* __restrict__ dy,
                                                                const h16* __restrict__ skip, int N, int D, int H,
                                                                int W, int C, int dims3, h16* __restrict__ dx) {
  const int OD = dims3 ? D / 2 : 1, OH = H / 2, OW = W / 2;
  const int cpp = C / 8;
  const int total = N * OD * OH * OW * cpp;
  const int nz = dims3 ? 2 : 1;
  const int bits = dims3 ? 3 : 2;
  const uint32_t kmask = dims3 ? 7u : 3u;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const PoolIdx pi = pool_idx(i, cpp, OW, OH, H, W, dims3);
    float g[8];
    unpack8(*(const u32x4*)(dy + (size_t)i * 8), g);
    const uint32_t w = code[i];
    for (int dz = 0; dz < nz; ++dz)
#pragma unroll
      for (int dyy = 0; dyy < 2; ++dyy)
#pragma unroll
        for (int dxx = 0; dxx < 2; ++dxx) {
          const uint32_t k = dz * 4 + dyy * 2 + dxx;
          const size_t off = (size_t)(pi.base + (dz * H + dyy) * W + dxx) * C + pi.cc * 8;
          float o[8];
          if (skip) {
            unpack8(*(const u32x4*)(skip + off), o);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (((w >> (bits * e)) & kmask) == k && ((w >> (24 + e)) & 1u)) o[e] += g[e];
          *(u32x4*)(dx + off) = pack8(o);
        }
  }
}

// Pool backward of a normalised convNb output: as maxpool2_bwd_code_kernel (argmax
// codes + the decoder's skip gradient), plus the backward statistics of the norm
// {sum g, sum g z} over the sample's full-resolution pixels (z = the pre-norm tensor):
// one row per block, rows[(n * nbp + blk)][2][C] (GroupNorm / BatchNorm finalize read
// them like the conv epilogues' tile rows).  Grid (nbp, N); a thread keeps one 8-channel
// column for the whole block (fixed-order reduction over the block's threads).
__global__ void __launch_bounds__(256) maxpool2_bwd_norm_kernel(const uint32_t* __restrict__ code,
                                                                const h16* __restrict__ dy,
                                                                const h16* __restrict__ skip,
                                                                const h16* __restrict__ z, int D, int H, int W, int C,
                                                                int dims3, h16* __restrict__ dx,
                                                                float* __restrict__ rows) {
  __shared__ float red[256 * 2 * 8];     // [thread][moment][8 channels]
  const int OD = dims3 ? D / 2 : 1, OH = H / 2, OW = W / 2;
  const int cpp = C / 8, rstep = 256 / cpp;
  const int n = blockIdx.y, nbp = gridDim.x, blk = blockIdx.x;
  const int OP = OD * OH * OW;
  const int cc = threadIdx.x % cpp, rs = threadIdx.x / cpp;
  const int nz = dims3 ? 2 : 1;
  const int bits = dims3 ? 3 : 2;
  const uint32_t kmask = dims3 ? 7u : 3u;
  const int p0 = (int)((long long)blk * OP / nbp), p1 = (int)((long long)(blk + 1) * OP / nbp);
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  for (int pp = p0 + rs; pp < p1; pp += rstep) {
    const int i = (n * OP + pp) * cpp + cc;
    const PoolIdx pi = pool_idx(i, cpp, OW, OH, H, W, dims3);
    float g[8];
    unpack8(*(const u32x4*)(dy + (size_t)i * 8), g);
    const uint32_t w = code[i];
    for (int dz = 0; dz < nz; ++dz)
#pragma unroll
      for (int dyy = 0; dyy < 2; ++dyy)
#pragma unroll
        for (int dxx = 0; dxx < 2; ++dxx) {
          const uint32_t k = dz * 4 + dyy * 2 + dxx;
          const size_t off = (size_t)(pi.base + (dz * H + dyy) * W + dxx) * C + pi.cc * 8;
          float o[8], zf[8];
          if (skip) {
            unpack8(*(const u32x4*)(skip + off), o);
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = 0.f;
          }
          unpack8(*(const u32x4*)(z + off), zf);
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (((w >> (bits * e)) & kmask) == k && ((w >> (24 + e)) & 1u)) o[e] += g[e];
          const u32x4 ov = pack8(o);
          *(u32x4*)(dx + off) = ov;
          unpack8(ov, o);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += o[e];
            s2[e] = fmaf(o[e], zf[e], s2[e]);
          }
        }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(threadIdx.x * 2 + 0) * 8 + e] = s1[e];
    red[(threadIdx.x * 2 + 1) * 8 + e] = s2[e];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * C; t += 256) {
    const int mom = t / C, c = t - mom * C;
    const int col = c / 8, e = c & 7;
    float a = 0.f;
    for (int r = 0; r < rstep; ++r) a += red[((r * cpp + col) * 2 + mom) * 8 + e];
    rows[((size_t)(n * nbp + blk) * 2 + mom) * C + c] = a;
  }
}

// Nearest 2x(2x2) upsample, materialised: y[child] = x[p] for the 4 (8 in 3D) children of
// each low-resolution pixel; one thread = one low pixel x 8 channels (16-byte accesses).
// The decoder convs of the upsampling variant then read a full-resolution source and
// run on the row-window kernels (the folded-upsample implicit GEMM was 3-10x slower).
__global__ void __launch_bounds__(256) upsample2_fwd_kernel(const h16* __restrict__ x, int N, int D, int H, int W,
                                                            int C, int dims3, h16* __restrict__ y) {
  // D, H, W: LOW resolution dims
  const int cpp = C / 8;
  const int FD = dims3 ? 2 : 1;
  const int total = N * D * H * W * cpp;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int cc = i % cpp;
    int r = i / cpp;
    const int w = r % W;
    r /= W;
    const int h = r % H;
    const int nd = r / H;                 // n * D + d
    const u32x4 v = *(const u32x4*)(x + (size_t)i * 8);
    for (int dz = 0; dz < FD; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const size_t row = ((size_t)(nd * FD + dz) * (2 * H) + 2 * h + dy) * (2 * W) + 2 * w;
        *(u32x4*)(y + row * C + cc * 8) = v;
        *(u32x4*)(y + (row + 1) * C + cc * 8) = v;
      }
  }
}

// dlow[p] = sum_{2x2(x2) children} dup[child] * (mask[p] > 0)
__global__ void __launch_bounds__(256) upsample2_bwd_kernel(const h16* __restrict__ dup, const h16* __restrict__ mask,
                                                            int N, int D, int H, int W, int C, int dims3,
                                                            h16* __restrict__ dlow) {
  // D, H, W: LOW resolution dims
  const int cpp = C / 8;
  const int FD = dims3 ? 2 : 1;
  const long long total = (long long)N * D * H * W * cpp;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int cc = i % cpp;
    long long r = i / cpp;
    const int w = r % W;
    r /= W;
    const int h = r % H;
    r /= H;
    const int d = r % D;
    const int n = r / D;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int dz = 0; dz < FD; ++dz)
      for (int dy = 0; dy < 2; ++dy)
        for (int dx = 0; dx < 2; ++dx) {
          const size_t pix = (((size_t)n * (D * FD) + d * FD + dz) * (2 * H) + 2 * h + dy) * (2 * W) + 2 * w + dx;
          float f[8];
          unpack8(*(const u32x4*)(dup + pix * C + cc * 8), f);
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] += f[e];
        }
    u32x4 v = pack8(s);
    if (mask) {
      const u32x4 mv = *(const u32x4*)(mask + (size_t)i * 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] &= bf_pos_mask(mv[e]);
    }
    *(u32x4*)(dlow + (size_t)i * 8) = v;
  }
}

inline int grid_for(long long work, int per_block = 256) {
  long long g = (work + per_block - 1) / per_block;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

hipError_t cast_input_launch(const float* x, int P, int Cin, int Cpad, void* y, hipStream_t s) {
  UNET_LAUNCH(cast_input_kernel, dim3(grid_for((long long)P * Cpad)), dim3(256), 0, s, x, P, Cin, Cpad,
                     (h16*)y);
  return launch_status();
}

hipError_t gather_batch_launch(const float* x_all, const float* y_all, const long long* idx, int B, int P, int Cin,
                               int Cpad, void* xb, void* tb, hipStream_t s) {
  UNET_LAUNCH(gather_batch_kernel, dim3(grid_for((long long)B * P)), dim3(256), 0, s, x_all, y_all, idx, B, P,
                     Cin, Cpad, (h16*)xb, (h16*)tb);
  return launch_status();
}

hipError_t maxpool2_fwd_launch(const void* x, int N, int D, int H, int W, int C, int dims3, void* y, void* code,
                               hipStream_t s) {
  const long long work = (long long)N * (dims3 ? D / 2 : 1) * (H / 2) * (W / 2) * (C / 8);
  UNET_LAUNCH(maxpool2_fwd_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const h16*)x, N, D, H, W, C,
                     dims3, (h16*)y, (uint32_t*)code);
  return launch_status();
}

hipError_t norm_pool_launch(const void* z, const float* fa, const float* fc, int cstride, int N, int D, int H, int W,
                            int C, int dims3, void* y, void* py, void* code, hipStream_t s) {
  const long long work = (long long)N * (dims3 ? D / 2 : 1) * (H / 2) * (W / 2) * (C / 8);
  if (dims3)
    UNET_LAUNCH(norm_pool_kernel<true>, dim3(grid_for(work)), dim3(256), 0, s, (const h16*)z, fa, fc, cstride,
                       N, D, H, W, C, (h16*)y, (h16*)py, (uint32_t*)code);
  else
    UNET_LAUNCH(norm_pool_kernel<false>, dim3(grid_for(work)), dim3(256), 0, s, (const h16*)z, fa, fc,
                       cstride, N, D, H, W, C, (h16*)y, (h16*)py, (uint32_t*)code);
  return launch_status();
}

hipError_t maxpool2_bwd_launch(const void* x, const void* code, const void* dy, const void* skip, int N, int D, int H,
                               int W, int C, int dims3, void* dx, hipStream_t s) {
  const long long work = (long long)N * (dims3 ? D / 2 : 1) * (H / 2) * (W / 2) * (C / 8);
  if (code)
    UNET_LAUNCH(maxpool2_bwd_code_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const uint32_t*)code,
                       (const h16*)dy, (const h16*)skip, N, D, H, W, C, dims3, (h16*)dx);
  else
    UNET_LAUNCH(maxpool2_bwd_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const h16*)x, (const h16*)dy,
                       (const h16*)skip, N, D, H, W, C, dims3, (h16*)dx);
  return launch_status();
}

hipError_t maxpool2_bwd_norm_launch(const void* code, const void* dy, const void* skip, const void* z, int N, int D,
                                    int H, int W, int C, int dims3, int nbp, void* dx, float* rows, hipStream_t s) {
  UNET_LAUNCH(maxpool2_bwd_norm_kernel, dim3(nbp, N), dim3(256), 0, s, (const uint32_t*)code, (const h16*)dy,
                     (const h16*)skip, (const h16*)z, D, H, W, C, dims3, (h16*)dx, rows);
  return launch_status();
}

hipError_t upsample2_fwd_launch(const void* x, int N, int D, int H, int W, int C, int dims3, void* y, hipStream_t s) {
  const long long work = (long long)N * D * H * W * (C / 8);
  UNET_LAUNCH(upsample2_fwd_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const h16*)x, N, D, H, W, C, dims3,
                     (h16*)y);
  return launch_status();
}

hipError_t upsample2_bwd_launch(const void* dup, const void* mask, int N, int D, int H, int W, int C, int dims3,
                                void* dlow, hipStream_t s) {
  const long long work = (long long)N * D * H * W * (C / 8);
  UNET_LAUNCH(upsample2_bwd_kernel, dim3(grid_for(work)), dim3(256), 0, s, (const h16*)dup,
                     (const h16*)mask, N, D, H, W, C, dims3, (h16*)dlow);
  return launch_status();
}

}  // namespace unet
