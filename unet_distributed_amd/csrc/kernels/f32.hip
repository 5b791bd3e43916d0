// fp32 path: the reference's own precision (test_dist.py:196-202 -- TF 1.x trains fp32
// end to end).  fp32 activations, gradients and weights; every GEMM on
// v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation, 1/16 of the bf16 MFMA
// rate on gfx950 -- 157 TF peak), no operand rounding anywhere.
//
// The bf16 executor's fusions are 16-bit-layout specific (64-byte pixel slots, 8-channel
// chunks, 1-bit masks); this path keeps the structure plain and general instead:
//   * f32_conv_kernel: implicit-GEMM convolution, NHWC / NDHWC, 1..3 taps per dim, stride,
//     padding, a two-source (concat) input, bias / ReLU / inverted-dropout / consumer-mask
//     epilogue, optional transposed-conv pixel-shuffle store.  Serves the conv forward, the
//     conv data gradient (flipped, transposed weight copy), the transposed-conv forward
//     (1x1 GEMM + shuffle) and its data gradient (2x2 stride-2 conv);
//   * f32_wgrad_kernel: weight gradients as per-tap TN GEMMs over pixels, split-K slabs
//     reduced in fixed order (conv_wgrad.hip::wgrad_reduce, deterministic);
//   * pool / upsample / head / column-sum / weight-transpose elementwise kernels.
// Tiles: 64 x 64 outputs per 256-thread workgroup (4 waves of 32 x 32 = 2 x 2 MFMA tiles),
// K in steps of 16 staged through LDS (A rows padded to 17 floats: conflict-free column
// reads by the MFMA lanes).
#include "common.h"
#include "conv_params.h"

namespace unet {
namespace {

constexpr int FT = 256, FBM = 64, FBN = 64, FBK = 16;

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// A tile = im2col rows (pixels) x K slice; B tile = weight rows [k][Cout].  Tiles (BM, BN)
// with 4 waves in a WGM x WGN grid, each wave MI x NJ 16 x 16 MFMA tiles: (128, 32) for
// Cout <= 32 (4 x 1 waves of 32 x 32 -- the 64-wide N tile left half of its MFMAs on zero
// columns at the level-1 convs), (128, 64) / (128, 128) (2 x 2 waves of 64 x 32 / 64 x 64:
// 2-4x the MFMAs per LDS and global byte of the 64 x 64 tile), (64, 64) for small M.
template <int BM, int BN>
__global__ void __launch_bounds__(FT) f32_conv_kernel(const F32Conv p) {
  constexpr int RA = BM / 64;                  // pixel rows per thread in the A loader
  constexpr int WGN = BN == 32 ? 1 : 2, WGM = 4 / WGN;
  constexpr int MI = BM / WGM / 16, NJ = BN / WGN / 16;
  constexpr int BVN = BN / 16;                 // B floats per thread (k row tid >> 4)
  __shared__ float As[BM][FBK + 1];
  __shared__ float Bs[FBK][BN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave - wm * WGN;
  const int M = p.N * p.OD * p.OH * p.OW;
  const int Cin = p.C1 + p.C2;
  const int K = p.KD * p.KH * p.KW * Cin;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  // A loader: thread -> (pixel rows am + 64 r, 4 consecutive k)
  const int am = tid >> 2, ak = (tid & 3) * 4;
  int qv[RA], qn[RA], qd[RA], qh[RA], qw[RA];
#pragma unroll
  for (int r = 0; r < RA; ++r) {
    qv[r] = m0 + am + 64 * r;
    int t = qv[r] < M ? qv[r] : 0;
    qw[r] = t % p.OW;
    t /= p.OW;
    qh[r] = t % p.OH;
    t /= p.OH;
    qd[r] = t % p.OD;
    qn[r] = t / p.OD;
  }
  // B loader: thread -> (k row, BVN consecutive n)
  const int bk = tid >> 4, bn = (tid & 15) * BVN;
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const bool vec = (Cin % 4) == 0 && (p.C1 % 4) == 0;
  const bool wvec = (p.ldw % 4) == 0 && (((uintptr_t)p.wgt) & 15) == 0;
  // A loader state of this thread's k = k0 + ak: (tap, c) advanced incrementally by FBK per
  // step (no per-step divisions), tap -> (kd, kh, kw) likewise
  int a_tap = ak / Cin, a_c = ak - (ak / Cin) * Cin;
  int a_kw = a_tap % p.KW, a_kh = (a_tap / p.KW) % p.KH, a_kd = a_tap / (p.KW * p.KH);
  const int padd = p.KD > 1 ? p.pad : 0;
  float av[RA][4], bv[BVN];
  auto load = [&](const int k0) {
#pragma unroll
    for (int r = 0; r < RA; ++r) {
#pragma unroll
      for (int e = 0; e < 4; ++e) av[r][e] = 0.f;
      if (qv[r] >= M) continue;
      if (vec) {
        if (k0 + ak < K) {
          const int id = qd[r] * p.stride + a_kd - padd;
          const int ih = qh[r] * p.stride + a_kh - p.pad, iw = qw[r] * p.stride + a_kw - p.pad;
          if ((unsigned)id < (unsigned)p.ID && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW) {
            const size_t pix = (((size_t)qn[r] * p.ID + id) * p.IH + ih) * p.IW + iw;
            const f32x4 v = a_c < p.C1 ? *(const f32x4*)(p.src1 + pix * p.C1 + a_c)
                                       : *(const f32x4*)(p.src2 + pix * p.C2 + (a_c - p.C1));
#pragma unroll
            for (int e = 0; e < 4; ++e) av[r][e] = v[e];
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = k0 + ak + e;
          if (k >= K) continue;
          const int tap = k / Cin, c = k - tap * Cin;
          const int kw = tap % p.KW, kh = (tap / p.KW) % p.KH, kd = tap / (p.KW * p.KH);
          const int id = qd[r] * p.stride + kd - padd;
          const int ih = qh[r] * p.stride + kh - p.pad, iw = qw[r] * p.stride + kw - p.pad;
          if ((unsigned)id < (unsigned)p.ID && (unsigned)ih < (unsigned)p.IH && (unsigned)iw < (unsigned)p.IW) {
            const size_t pix = (((size_t)qn[r] * p.ID + id) * p.IH + ih) * p.IW + iw;
            av[r][e] = c < p.C1 ? p.src1[pix * p.C1 + c] : p.src2[pix * p.C2 + (c - p.C1)];
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < BVN; ++e) bv[e] = 0.f;
    const int k = k0 + bk;
    if (k < K) {
      if (wvec && BVN >= 4 && n0 + bn + BVN <= p.Cout) {
#pragma unroll
        for (int h = 0; h < BVN / 4; ++h) {
          const f32x4 v = *(const f32x4*)(p.wgt + (size_t)k * p.ldw + n0 + bn + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) bv[4 * h + e] = v[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < BVN; ++e)
          if (n0 + bn + e < p.Cout) bv[e] = p.wgt[(size_t)k * p.ldw + n0 + bn + e];
      }
    }
  };
  auto advance = [&]() {
    a_c += FBK;
    while (a_c >= Cin) {
      a_c -= Cin;
      if (++a_kw == p.KW) {
        a_kw = 0;
        if (++a_kh == p.KH) {
          a_kh = 0;
          ++a_kd;
        }
      }
    }
  };
  // register prefetch: the next K step's global loads are in flight under this step's MFMAs
  load(0);
  for (int k0 = 0; k0 < K; k0 += FBK) {
    __syncthreads();
#pragma unroll
    for (int r = 0; r < RA; ++r)
#pragma unroll
      for (int e = 0; e < 4; ++e) As[am + 64 * r][ak + e] = av[r][e];
#pragma unroll
    for (int e = 0; e < BVN; ++e) Bs[bk][bn + e] = bv[e];
    __syncthreads();
    if (k0 + FBK < K) {
      advance();
      load(k0 + FBK);
    }
#pragma unroll
    for (int ks = 0; ks < FBK / 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
      float a[MI], b[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = As[wm * (16 * MI) + i * 16 + (lane & 15)][kk];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = Bs[kk][wn * (16 * NJ) + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma4(a[i], b[j], acc[i][j]);
    }
  }
  // epilogue: acc[i][j][r] = out[pixel m0 + wm 16 MI + 16 i + 4 (lane >> 4) + r][chan n0 + wn 16 NJ + 16 j + (lane & 15)]
  const float inv_keep = p.drop_rate > 0.f ? 1.f / (1.f - p.drop_rate) : 1.f;
  const uint32_t thr = (uint32_t)(p.drop_rate * 4294967296.0);
  const uint32_t seed = p.seed_ptr ? *p.seed_ptr : p.seed;
  const int Dt = p.shuffle ? p.Cout >> p.shuffle : p.Cout;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int n = n0 + wn * (16 * NJ) + j * 16 + (lane & 15);
    if (n >= p.Cout) continue;
    const float bias = p.bias ? p.bias[p.shuffle ? n % Dt : n] : 0.f;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int qq = m0 + wm * (16 * MI) + i * 16 + 4 * (lane >> 4) + r;
        if (qq >= M) continue;
        float v = acc[i][j][r] + bias;
        if (p.relu) v = fmaxf(v, 0.f);
        if (p.drop_rate > 0.f) {
          const uint32_t h = drop_hash((uint64_t)qq * p.Cout + n + p.drop_idx0, seed, p.salt);
          v = h >= thr ? v * inv_keep : 0.f;
        }
        size_t off;
        if (p.shuffle) {
          // transposed conv: channel n = tap Dt + co -> fine pixel (2 d + td, 2 h + th, 2 w + tw)
          const int tap = n / Dt, co = n - tap * Dt;
          int t = qq;
          const int w = t % p.OW;
          t /= p.OW;
          const int h = t % p.OH;
          t /= p.OH;
          const int d = t % p.OD, nn = t / p.OD;
          const int td = p.shuffle == 3 ? tap >> 2 : 0, th = (tap >> 1) & 1, tw = tap & 1;
          const int dd = p.shuffle == 3 ? 2 : 1;
          off = ((((size_t)nn * p.OD * dd + d * dd + td) * (2 * p.OH) + 2 * h + th) * (2 * p.OW) + 2 * w + tw) * Dt + co;
        } else {
          off = (size_t)qq * p.Cout + n;
        }
        if (p.mask) v = p.mask[off] > 0.f ? v * p.mask_scale : 0.f;
        p.dst[off] = v;
      }
  }
}

// slab[split][tap][m][n] = sum_{q in split} A[q * stride + tap - pad][m] * B[q][n]
//   conv:  A = forward input x (m = ci, two sources), B = dY (n = co)      -> HWIO per tap
//   tconv: A = dOut (fine grid, stride 2, pad 0), B = coarse input (n = ci) -> (kh, kw, co, ci)
// grid: (m tiles x n tiles, taps, splits)
__global__ void __launch_bounds__(FT) f32_wgrad_kernel(const F32Wgrad p) {
  __shared__ float As[FBK][FBM];
  __shared__ float Bs[FBK][FBN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int Mt = p.M1 + p.M2;
  const int ntn = (p.Nc + FBN - 1) / FBN;
  const int m0 = (blockIdx.x / ntn) * FBM, n0 = (blockIdx.x % ntn) * FBN;
  const int tap = blockIdx.y, split = blockIdx.z;
  const int kw = tap % p.KW, kh = (tap / p.KW) % p.KH, kd = tap / (p.KW * p.KH);
  const int Q = p.N * p.QD * p.QH * p.QW;
  const int q_begin = (int)((long long)split * Q / p.splits), q_end = (int)((long long)(split + 1) * Q / p.splits);
  // loaders: thread -> (pixel row t / 16, 4 consecutive channels)
  const int lr = tid >> 4, lc = (tid & 15) * 4;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  // this thread's pixel q = q0 + lr as (n, d, h, w), advanced incrementally by FBK per step
  int qw_ = 0, qh_ = 0, qd_ = 0, qn_ = 0;
  {
    int t = q_begin + lr;
    qw_ = t % p.QW;
    t /= p.QW;
    qh_ = t % p.QH;
    t /= p.QH;
    qd_ = t % p.QD;
    qn_ = t / p.QD;
  }
  const int padd = p.KD > 1 ? p.pad : 0;
  float av[4], bv[4];
  auto load = [&](const int q0) {
    const int q = q0 + lr;
#pragma unroll
    for (int e = 0; e < 4; ++e) av[e] = bv[e] = 0.f;
    if (q < q_end) {
      const int ad = qd_ * p.stride + kd - padd;
      const int ah = qh_ * p.stride + kh - p.pad, aw = qw_ * p.stride + kw - p.pad;
      if ((unsigned)ad < (unsigned)p.AD && (unsigned)ah < (unsigned)p.AH && (unsigned)aw < (unsigned)p.AW) {
        const size_t pix = (((size_t)qn_ * p.AD + ad) * p.AH + ah) * p.AW + aw;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int m = m0 + lc + e;
          if (m < p.M1) av[e] = p.a1[pix * p.M1 + m];
          else if (m < Mt) av[e] = p.a2[pix * p.M2 + (m - p.M1)];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + lc + e;
        if (n < p.Nc) bv[e] = p.b[(size_t)q * p.Nc + n];
      }
    }
  };
  auto advance = [&]() {
    qw_ += FBK;
    while (qw_ >= p.QW) {
      qw_ -= p.QW;
      if (++qh_ == p.QH) {
        qh_ = 0;
        if (++qd_ == p.QD) {
          qd_ = 0;
          ++qn_;
        }
      }
    }
  };
  // register prefetch: the next pixel step's loads are in flight under this step's MFMAs
  if (q_begin < q_end) load(q_begin);
  for (int q0 = q_begin; q0 < q_end; q0 += FBK) {
    __syncthreads();
    *(f32x4*)&As[lr][lc] = (f32x4){av[0], av[1], av[2], av[3]};
    *(f32x4*)&Bs[lr][lc] = (f32x4){bv[0], bv[1], bv[2], bv[3]};
    __syncthreads();
    if (q0 + FBK < q_end) {
      advance();
      load(q0 + FBK);
    }
#pragma unroll
    for (int ks = 0; ks < FBK / 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk][wm * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma4(a[i], b[j], acc[i][j]);
    }
  }
  const int taps = p.KD * p.KH * p.KW;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + r;
        if (m < Mt && n < p.Nc) p.slab[(((size_t)split * taps + tap) * Mt + m) * p.Nc + n] = acc[i][j][r];
      }
    }
}

// Weight gradient with channel-sized tiles (BM, BN in {32, 64}; every channel count % 4 == 0):
// the 64 x 64 tile of f32_wgrad_kernel leaves 3/4 of its MFMAs on zeros at 32 x 32 (the
// level-1 convs -- 2.2 ms per launch, round-5 fp32 profile).  The 4 waves form a
// (BM / 32) x (BN / 32) grid of 32 x 32 sub-tiles and split each step's KR = 16 WK pixels
// WK ways; the WK partial tiles are summed in fixed order through LDS at the end.  One
// pixel state per thread: thread t loads row t / TPR, its 1 / TPR share of the A row (BM
// channels) and of the B row (BN channels) as float4s; the row's pixel is advanced by KR
// per step without divisions; the next step's loads are in flight under the MFMAs.
template <int BM, int BN>
__global__ void __launch_bounds__(FT) f32_wgrad_cs_kernel(const F32Wgrad p) {
  // wave sub-tiles SM x SN (64 x 64 in the 128 x 128 tile: 4x the MFMAs per LDS read of 32 x 32)
  constexpr int SM = BM == 128 ? 64 : 32, SN = BN == 128 ? 64 : 32, MI = SM / 16, NJ = SN / 16;
  constexpr int WGM = BM / SM, WGN = BN / SN, WK = 4 / (WGM * WGN), KR = FBK * WK, TPR = FT / KR;
  constexpr int AV = BM / TPR / 4, BV = BN / TPR / 4;        // float4s per thread and row
  static_assert(AV >= 1 && BV >= 1, "channel share per thread");
  __shared__ float As[KR][BM + 4];
  __shared__ float Bs[KR][BN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave / (WGM * WGN), wr = wave - wk * (WGM * WGN), wm = wr / WGN, wn = wr - wm * WGN;
  const int Mt = p.M1 + p.M2;
  const int ntn = (p.Nc + BN - 1) / BN;
  const int m0 = (blockIdx.x / ntn) * BM, n0 = (blockIdx.x % ntn) * BN;
  const int tap = blockIdx.y, split = blockIdx.z;
  const int kw = tap % p.KW, kh = (tap / p.KW) % p.KH, kd = tap / (p.KW * p.KH);
  const int Q = p.N * p.QD * p.QH * p.QW;
  const int q_begin = (int)((long long)split * Q / p.splits), q_end = (int)((long long)(split + 1) * Q / p.splits);
  const int lr = tid / TPR, sub = tid - lr * TPR;
  int qw_ = 0, qh_ = 0, qd_ = 0, qn_ = 0;
  {
    int t = q_begin + lr;
    qw_ = t % p.QW;
    t /= p.QW;
    qh_ = t % p.QH;
    t /= p.QH;
    qd_ = t % p.QD;
    qn_ = t / p.QD;
  }
  const int padd = p.KD > 1 ? p.pad : 0;
  f32x4 av[AV], bv[BV];
  auto load = [&](const int q0) {
    const int q = q0 + lr;
#pragma unroll
    for (int v = 0; v < AV; ++v) av[v] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int v = 0; v < BV; ++v) bv[v] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (q < q_end) {
      const int ad = qd_ * p.stride + kd - padd;
      const int ah = qh_ * p.stride + kh - p.pad, aw = qw_ * p.stride + kw - p.pad;
      if ((unsigned)ad < (unsigned)p.AD && (unsigned)ah < (unsigned)p.AH && (unsigned)aw < (unsigned)p.AW) {
        const size_t pix = (((size_t)qn_ * p.AD + ad) * p.AH + ah) * p.AW + aw;
#pragma unroll
        for (int v = 0; v < AV; ++v) {
          const int m = m0 + (sub * AV + v) * 4;
          if (m < p.M1) av[v] = *(const f32x4*)(p.a1 + pix * p.M1 + m);
          else if (m < Mt) av[v] = *(const f32x4*)(p.a2 + pix * p.M2 + (m - p.M1));
        }
      }
#pragma unroll
      for (int v = 0; v < BV; ++v) {
        const int n = n0 + (sub * BV + v) * 4;
        if (n < p.Nc) bv[v] = *(const f32x4*)(p.b + (size_t)q * p.Nc + n);
      }
    }
  };
  auto advance = [&]() {
    qw_ += KR;
    while (qw_ >= p.QW) {
      qw_ -= p.QW;
      if (++qh_ == p.QH) {
        qh_ = 0;
        if (++qd_ == p.QD) {
          qd_ = 0;
          ++qn_;
        }
      }
    }
  };
  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (q_begin < q_end) load(q_begin);
  for (int q0 = q_begin; q0 < q_end; q0 += KR) {
    __syncthreads();
#pragma unroll
    for (int v = 0; v < AV; ++v) *(f32x4*)&As[lr][(sub * AV + v) * 4] = av[v];
#pragma unroll
    for (int v = 0; v < BV; ++v) *(f32x4*)&Bs[lr][(sub * BV + v) * 4] = bv[v];
    __syncthreads();
    if (q0 + KR < q_end) {
      advance();
      load(q0 + KR);
    }
#pragma unroll
    for (int ks = 0; ks < FBK / 4; ++ks) {
      const int kk = wk * FBK + ks * 4 + (lane >> 4);
      float a[MI], b[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = As[kk][wm * SM + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < NJ; ++j) b[j] = Bs[kk][wn * SN + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma4(a[i], b[j], acc[i][j]);
    }
  }
  if constexpr (WK > 1) {
    static_assert(MI == 2 && NJ == 2, "K-split tiles are 32 x 32 per wave");
    // the K-split partial tiles: red[fragment][wave][lane] (fragment-major: lanes 16 B apart)
    __shared__ f32x4 red[4][4][64];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) red[i * 2 + j][wave][lane] = acc[i][j];
    __syncthreads();
    if (wk != 0) return;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int o = 1; o < WK; ++o) acc[i][j] += red[i * 2 + j][o * (WGM * WGN) + wr][lane];
  }
  const int taps = p.KD * p.KH * p.KW;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn * SN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * SM + i * 16 + 4 * (lane >> 4) + r;
        if (m < Mt && n < p.Nc) p.slab[(((size_t)split * taps + tap) * Mt + m) * p.Nc + n] = acc[i][j][r];
      }
    }
}

// 2x2(x2) max-pool forward (2D or 3D, windows never overlap)
__global__ void f32_pool_fwd_kernel(const float* __restrict__ x, int N, int D, int H, int W, int C, int dims3,
                                    float* __restrict__ y) {
  const int Dp = dims3 ? D / 2 : 1, Hp = H / 2, Wp = W / 2;
  const long long total = (long long)N * Dp * Hp * Wp * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % Wp);
    t /= Wp;
    const int h = (int)(t % Hp);
    t /= Hp;
    const int d = (int)(t % Dp);
    const int n = (int)(t / Dp);
    float m = -INFINITY;
    for (int a = 0; a < (dims3 ? 2 : 1); ++a)
      for (int b = 0; b < 2; ++b)
        for (int e = 0; e < 2; ++e) {
          const size_t pix = (((size_t)n * D + (dims3 ? 2 * d + a : 0)) * H + 2 * h + b) * W + 2 * w + e;
          m = fmaxf(m, x[pix * C + c]);
        }
    y[i] = m;
  }
}

// max-pool backward + the skip gradient + the ReLU mask of the pool input x (a ReLU
// output): dx = (dy routed to the window's first argmax + skip) * (x > 0)
__global__ void f32_pool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy,
                                    const float* __restrict__ skip, int N, int D, int H, int W, int C, int dims3,
                                    float* __restrict__ dx) {
  const long long total = (long long)N * D * H * W * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long t = i / C;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    t /= H;
    const int d = (int)(t % D);
    const int n = (int)(t / D);
    const float xv = x[i];
    float g = skip ? skip[i] : 0.f;
    // first argmax of the window in (d, h, w) order
    const int d0 = dims3 ? d & ~1 : 0, h0 = h & ~1, w0 = w & ~1;
    float m = -INFINITY;
    int am = -1, k = 0;
    for (int a = 0; a < (dims3 ? 2 : 1); ++a)
      for (int b = 0; b < 2; ++b)
        for (int e = 0; e < 2; ++e, ++k) {
          const float v = x[((((size_t)n * D + d0 + a) * H + h0 + b) * W + w0 + e) * C + c];
          if (v > m) {
            m = v;
            am = k;
          }
        }
    const int mine = ((dims3 ? (d - d0) * 4 : 0) + (h - h0) * 2 + (w - w0));
    if (am == mine) {
      const int Dp = dims3 ? D / 2 : 1;
      const size_t pq = (((size_t)n * Dp + (dims3 ? d >> 1 : 0)) * (H / 2) + (h >> 1)) * (W / 2) + (w >> 1);
      g += dy[pq * C + c];
    }
    dx[i] = xv > 0.f ? g : 0.f;
  }
}

// nearest 2x upsample forward / backward (sum of the 2x2(x2) children, times mask > 0)
__global__ void f32_ups_kernel(const float* __restrict__ src, const float* __restrict__ mask, int N, int D, int H,
                               int W, int C, int dims3, int bwd, float* __restrict__ dst) {
  // (D, H, W): the low resolution
  const int Df = dims3 ? 2 * D : 1, Hf = 2 * H, Wf = 2 * W;
  const long long total = bwd ? (long long)N * D * H * W * C : (long long)N * Df * Hf * Wf * C;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    long long t = i / C;
    if (!bwd) {
      const int w = (int)(t % Wf);
      t /= Wf;
      const int h = (int)(t % Hf);
      t /= Hf;
      const int d = (int)(t % Df);
      const int n = (int)(t / Df);
      dst[i] = src[((((size_t)n * D + (dims3 ? d >> 1 : 0)) * H + (h >> 1)) * W + (w >> 1)) * C + c];
    } else {
      const int w = (int)(t % W);
      t /= W;
      const int h = (int)(t % H);
      t /= H;
      const int d = (int)(t % D);
      const int n = (int)(t / D);
      float s = 0.f;
      for (int a = 0; a < (dims3 ? 2 : 1); ++a)
        for (int b = 0; b < 2; ++b)
          for (int e = 0; e < 2; ++e)
            s += src[((((size_t)n * Df + (dims3 ? 2 * d + a : 0)) * Hf + 2 * h + b) * Wf + 2 * w + e) * C + c];
      dst[i] = (mask && !(mask[i] > 0.f)) ? 0.f : s;
    }
  }
}

// head forward: logit = x . w + b, p = sigmoid, per-block {I, St, Sp, BCE} partials
template <int C>
__global__ void __launch_bounds__(FT) f32_head_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ b, const float* __restrict__ t,
                                                          int P, float* __restrict__ prob,
                                                          float* __restrict__ partial) {
  __shared__ float red[4][FT / 64];
  float sI = 0.f, sT = 0.f, sP = 0.f, sB = 0.f;
  for (int px = blockIdx.x * FT + threadIdx.x; px < P; px += gridDim.x * FT) {
    float z = b[0];
#pragma unroll
    for (int c = 0; c < C; ++c) z = fmaf(x[(size_t)px * C + c], w[c], z);
    const float pr = 1.f / (1.f + expf(-z));
    prob[px] = pr;
    const float tv = t ? t[px] : 0.f;
    sI += tv * pr;
    sT += tv;
    sP += pr;
    sB += fmaxf(z, 0.f) - z * tv + log1pf(expf(-fabsf(z)));
  }
  sI = wave_sum(sI);
  sT = wave_sum(sT);
  sP = wave_sum(sP);
  sB = wave_sum(sB);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = sI;
    red[1][wv] = sT;
    red[2][wv] = sP;
    red[3][wv] = sB;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int k = 0; k < FT / 64; ++k) s += red[threadIdx.x][k];
    partial[blockIdx.x * 4 + threadIdx.x] = s;
  }
}

// fixed-order column sums of nb partial rows of `width` floats
__global__ void f32_rows_sum_kernel(const float* __restrict__ part, int nb, int width, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= width) return;
  float s = 0.f;
  for (int k = 0; k < nb; ++k) s += part[(size_t)k * width + c];
  out[c] = s;
}

// head backward: dlogit (Dice (+ BCE) loss, head_grad.h formula), the head input's
// gradient dx = dlogit w (x > 0), and per-block partials of the Mask gradients
// {sum dlogit x[c], sum dlogit}
template <int C>
__global__ void __launch_bounds__(FT) f32_head_bwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                          const float* __restrict__ prob, const float* __restrict__ t,
                                                          const float* __restrict__ sums, int P,
                                                          float inv_total, float bce_w, float* __restrict__ dx,
                                                          float* __restrict__ partial) {
  // G = C / 4 consecutive threads per pixel, one float4 channel group each: the pixel's
  // row is read and written as contiguous 16-byte pieces (one thread per pixel walking its
  // C channels made every load a 64-line gather: 1.7 ms for 268 MB, round-5 fp32 profile)
  constexpr int G = C / 4, PPB = FT / G;
  __shared__ f32x4 red[FT];
  __shared__ float redb[FT];
  const float I = sums[0], St = sums[1], Sp = sums[2];
  const float a = -2.f / (2.f * I + 1.f), bb = 1.f / (St + Sp + 1.f);
  const int g = threadIdx.x % G, pl = threadIdx.x / G;
  const f32x4 wg = *(const f32x4*)(w + 4 * g);
  f32x4 gw = (f32x4){0.f, 0.f, 0.f, 0.f};
  float gb = 0.f;
  for (long long px = (long long)blockIdx.x * PPB + pl; px < P; px += (long long)gridDim.x * PPB) {
    const float pr = prob[px], tv = t[px];
    const float dice = fmaf(a, tv, bb) * pr * (1.f - pr);
    const float dz = fmaf(bce_w * (pr - tv), inv_total, dice);
    if (g == 0) gb += dz;
    const f32x4 xv = *(const f32x4*)(x + px * C + 4 * g);
    gw += dz * xv;
    if (dx) {
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = xv[e] > 0.f ? dz * wg[e] : 0.f;
      *(f32x4*)(dx + px * C + 4 * g) = o;
    }
  }
  red[threadIdx.x] = gw;
  redb[threadIdx.x] = gb;
  __syncthreads();
  // fixed-order sums over the threads of each channel group
  if (threadIdx.x < G) {
    f32x4 s4 = red[threadIdx.x];
    for (int k = 1; k < PPB; ++k) s4 += red[k * G + threadIdx.x];
    *(f32x4*)(partial + (size_t)blockIdx.x * (C + 1) + 4 * threadIdx.x) = s4;
  } else if (threadIdx.x == G) {
    float sb = 0.f;
    for (int k = 0; k < PPB; ++k) sb += redb[k * G];
    partial[(size_t)blockIdx.x * (C + 1) + C] = sb;
  }
}

// per-block column sums of x [rows][C] (bias gradients): partial[blk][C]
__global__ void __launch_bounds__(FT) f32_colsum_kernel(const float* __restrict__ x, long long rows, int C,
                                                        float* __restrict__ partial) {
  // C % 4 == 0, C <= 4 FT: a thread owns one float4 column group cg of row lane rl; the
  // FT / (C / 4) row lanes stride the block's row range (4 rows in flight each), then the
  // lanes' sums are added in fixed order through LDS.  (Round-5 profile: the previous
  // one-thread-per-column loop -- C of 256 threads busy, one dependent load per row --
  // took 3 ms per level-1 bias gradient, 28 % of the fp32 step.)
  __shared__ f32x4 red[FT];
  const int G = C >> 2, RL = FT / G;
  const int cg = threadIdx.x % G, rl = threadIdx.x / G;
  const long long r0 = (long long)blockIdx.x * rows / gridDim.x, r1 = (long long)(blockIdx.x + 1) * rows / gridDim.x;
  f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
  if (rl < RL) {
    long long r = r0 + rl;
    for (; r + 3 * RL < r1; r += 4 * RL) {
      const f32x4 a = *(const f32x4*)(x + r * C + 4 * cg), b = *(const f32x4*)(x + (r + RL) * C + 4 * cg);
      const f32x4 c = *(const f32x4*)(x + (r + 2 * RL) * C + 4 * cg), d = *(const f32x4*)(x + (r + 3 * RL) * C + 4 * cg);
      acc += (a + b) + (c + d);
    }
    for (; r < r1; r += RL) acc += *(const f32x4*)(x + r * C + 4 * cg);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < G) {
    f32x4 s = red[threadIdx.x];
    for (int k = 1; k < RL; ++k) s += red[k * G + threadIdx.x];
    *(f32x4*)(partial + (size_t)blockIdx.x * C + 4 * threadIdx.x) = s;
  }
}

// dst[t][b][a] = src[flip ? T - 1 - t : t][a][b]   (weight copies in a GEMM's B layout)
__global__ void f32_transpose_kernel(const float* __restrict__ src, int T, int A, int B, int flip,
                                     float* __restrict__ dst) {
  const long long total = (long long)T * A * B;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int a = (int)(i % A);
    const long long r = i / A;
    const int b = (int)(r % B);
    const int t = (int)(r / B);
    dst[i] = src[((size_t)(flip ? T - 1 - t : t) * A + a) * B + b];
  }
}

int ew_blocks(long long n) {
  const long long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

}  // namespace

const char* f32_conv_check(const F32Conv& p) {
  if (!p.src1 || !p.wgt || !p.dst) return "f32_conv: src1 / wgt / dst required";
  if (p.C1 <= 0 || p.C2 < 0 || (p.C2 && !p.src2) || p.Cout <= 0) return "f32_conv: bad channels";
  if (p.KD < 1 || p.KH < 1 || p.KW < 1 || p.KD > 3 || p.KH > 3 || p.KW > 3 || p.stride < 1 || p.stride > 2)
    return "f32_conv: kernel extents 1..3, stride 1..2";
  if (p.shuffle && (p.shuffle < 2 || p.shuffle > 3 || p.Cout % (1 << p.shuffle)))
    return "f32_conv: shuffle must be 2 / 3 and divide Cout";
  if ((long long)p.N * p.OD * p.OH * p.OW >= (1LL << 31)) return "f32_conv: too many pixels";
  if (p.ldw < p.Cout) return "f32_conv: weight row stride below Cout";
  return nullptr;
}

const char* f32_wgrad_check(const F32Wgrad& p) {
  if (!p.a1 || !p.b || !p.slab || (p.M2 && !p.a2)) return "f32_wgrad: a1 / b / slab required";
  if (p.M1 <= 0 || p.Nc <= 0 || p.splits < 1) return "f32_wgrad: bad shape";
  if ((long long)p.N * p.QD * p.QH * p.QW >= (1LL << 31)) return "f32_wgrad: too many pixels";
  return nullptr;
}

hipError_t f32_conv_launch(const F32Conv& p, hipStream_t s) {
  const int M = p.N * p.OD * p.OH * p.OW;
  // (128-row tiles while they still give >= 2 workgroups per CU)
  const int gm = (M + 127) / 128;
  if (p.Cout <= 32)
    UNET_LAUNCH((f32_conv_kernel<128, 32>), dim3(gm, 1), dim3(FT), 0, s, p);
  else if (p.Cout <= 64 && gm >= 512)
    UNET_LAUNCH((f32_conv_kernel<128, 64>), dim3(gm, 1), dim3(FT), 0, s, p);
  else if (p.Cout % 128 == 0 && gm * (p.Cout / 128) >= 512)
    UNET_LAUNCH((f32_conv_kernel<128, 128>), dim3(gm, p.Cout / 128), dim3(FT), 0, s, p);
  else
    UNET_LAUNCH((f32_conv_kernel<64, 64>), dim3((M + FBM - 1) / FBM, (p.Cout + FBN - 1) / FBN), dim3(FT), 0, s, p);
  return launch_status();
}

// tile of the weight gradient: (BM, BN) of f32_wgrad_cs_kernel when every channel count is a
// multiple of 4 (float4 operand loads), else (0, 0): the generic 64 x 64 kernel
void f32_wgrad_tile(int M1, int M2, int Nc, int* bm, int* bn) {
  const bool vec = M1 % 4 == 0 && M2 % 4 == 0 && Nc % 4 == 0;
  const bool big = (M1 + M2) % 128 == 0 && Nc % 128 == 0;     // 128 x 128: 4x4 MFMA tiles per wave
  *bm = vec ? (big ? 128 : (M1 + M2 <= 32 ? 32 : 64)) : 0;
  *bn = vec ? (big ? 128 : (Nc <= 32 ? 32 : 64)) : 0;
}

hipError_t f32_wgrad_launch(const F32Wgrad& p, hipStream_t s) {
  const int Mt = p.M1 + p.M2;
  int bm, bn;
  f32_wgrad_tile(p.M1, p.M2, p.Nc, &bm, &bn);
  const dim3 gy(1, p.KD * p.KH * p.KW, p.splits);
  if (bm) {
    const int tiles = ((Mt + bm - 1) / bm) * ((p.Nc + bn - 1) / bn);
    const dim3 g(tiles, gy.y, gy.z);
    if (bm == 128) UNET_LAUNCH((f32_wgrad_cs_kernel<128, 128>), g, dim3(FT), 0, s, p);
    else if (bm == 32 && bn == 32) UNET_LAUNCH((f32_wgrad_cs_kernel<32, 32>), g, dim3(FT), 0, s, p);
    else if (bm == 32) UNET_LAUNCH((f32_wgrad_cs_kernel<32, 64>), g, dim3(FT), 0, s, p);
    else if (bn == 32) UNET_LAUNCH((f32_wgrad_cs_kernel<64, 32>), g, dim3(FT), 0, s, p);
    else UNET_LAUNCH((f32_wgrad_cs_kernel<64, 64>), g, dim3(FT), 0, s, p);
    return launch_status();
  }
  const int tiles = ((Mt + FBM - 1) / FBM) * ((p.Nc + FBN - 1) / FBN);
  UNET_LAUNCH(f32_wgrad_kernel, dim3(tiles, gy.y, gy.z), dim3(FT), 0, s, p);
  return launch_status();
}

hipError_t f32_pool_fwd_launch(const float* x, int N, int D, int H, int W, int C, int dims3, float* y,
                               hipStream_t s) {
  const long long n = (long long)N * (dims3 ? D / 2 : 1) * (H / 2) * (W / 2) * C;
  UNET_LAUNCH(f32_pool_fwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, x, N, D, H, W, C, dims3, y);
  return launch_status();
}

hipError_t f32_pool_bwd_launch(const float* x, const float* dy, const float* skip, int N, int D, int H, int W, int C,
                               int dims3, float* dx, hipStream_t s) {
  const long long n = (long long)N * D * H * W * C;
  UNET_LAUNCH(f32_pool_bwd_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, x, dy, skip, N, D, H, W, C, dims3, dx);
  return launch_status();
}

hipError_t f32_ups_launch(const float* src, const float* mask, int N, int D, int H, int W, int C, int dims3, int bwd,
                          float* dst, hipStream_t s) {
  const long long n = (long long)N * D * H * W * C * (bwd ? 1 : (dims3 ? 8 : 4));
  UNET_LAUNCH(f32_ups_kernel, dim3(ew_blocks(n)), dim3(256), 0, s, src, mask, N, D, H, W, C, dims3, bwd, dst);
  return launch_status();
}

int f32_head_blocks(int P) {
  const int b = (P + FT - 1) / FT;
  return b < 1 ? 1 : (b > 1024 ? 1024 : b);
}

hipError_t f32_head_fwd_launch(const float* x, const float* w, const float* b, const float* t, int P, int C,
                               float* prob, float* partial, float* sums, hipStream_t s) {
  const int nb = f32_head_blocks(P);
  if (C == 32)
    UNET_LAUNCH((f32_head_fwd_kernel<32>), dim3(nb), dim3(FT), 0, s, x, w, b, t, P, prob, partial);
  else if (C == 16)
    UNET_LAUNCH((f32_head_fwd_kernel<16>), dim3(nb), dim3(FT), 0, s, x, w, b, t, P, prob, partial);
  else if (C == 64)
    UNET_LAUNCH((f32_head_fwd_kernel<64>), dim3(nb), dim3(FT), 0, s, x, w, b, t, P, prob, partial);
  else
    return hipErrorInvalidValue;
  UNET_LAUNCH(f32_rows_sum_kernel, dim3(1), dim3(64), 0, s, partial, nb, 4, sums);
  return launch_status();
}

hipError_t f32_head_bwd_launch(const float* x, const float* w, const float* prob, const float* t, const float* sums,
                               int P, int C, float inv_total, float bce_w, float* dx, float* partial, float* gw,
                               float* gb, hipStream_t s) {
  const int nb = f32_head_blocks(P);
  if (C == 32)
    UNET_LAUNCH((f32_head_bwd_kernel<32>), dim3(nb), dim3(FT), 0, s, x, w, prob, t, sums, P, inv_total, bce_w, dx,
                partial);
  else if (C == 16)
    UNET_LAUNCH((f32_head_bwd_kernel<16>), dim3(nb), dim3(FT), 0, s, x, w, prob, t, sums, P, inv_total, bce_w, dx,
                partial);
  else if (C == 64)
    UNET_LAUNCH((f32_head_bwd_kernel<64>), dim3(nb), dim3(FT), 0, s, x, w, prob, t, sums, P, inv_total, bce_w, dx,
                partial);
  else
    return hipErrorInvalidValue;
  // gw = column sums 0..C-1 of the partial rows, gb = column C
  float* stage = partial + (size_t)nb * (C + 1);
  UNET_LAUNCH(f32_rows_sum_kernel, dim3(1), dim3(128), 0, s, partial, nb, C + 1, stage);
  UNET_LAUNCH(f32_transpose_kernel, dim3(1), dim3(128), 0, s, stage, 1, C, 1, 0, gw);
  UNET_LAUNCH(f32_transpose_kernel, dim3(1), dim3(64), 0, s, stage + C, 1, 1, 1, 0, gb);
  return launch_status();
}

hipError_t f32_colsum_launch(const float* x, long long rows, int C, int blocks, float* partial, float* out,
                             hipStream_t s) {
  UNET_LAUNCH(f32_colsum_kernel, dim3(blocks), dim3(FT), 0, s, x, rows, C, partial);
  // stage 2: the same fixed-order kernel over the block partials, one block
  UNET_LAUNCH(f32_colsum_kernel, dim3(1), dim3(FT), 0, s, (const float*)partial, (long long)blocks, C, out);
  return launch_status();
}

hipError_t f32_transpose_launch(const float* src, int T, int A, int B, int flip, float* dst, hipStream_t s) {
  UNET_LAUNCH(f32_transpose_kernel, dim3(ew_blocks((long long)T * A * B)), dim3(256), 0, s, src, T, A, B, flip, dst);
  return launch_status();
}

}  // namespace unet
