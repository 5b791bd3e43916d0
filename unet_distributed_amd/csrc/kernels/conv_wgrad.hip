// Weight gradients on gfx950 MFMA: split-K "TN" GEMM over pixels with
// transposed LDS reads (ds_read_b64_tr_b16), plus the deterministic slab
// reduction and the bias-gradient column sums.
//
//   slab[split][tap][m][n] = sum_{q in split} A[q*stride + tap - pad][m] * B[q][n]
//
// * conv 3x3:  A = layer input X (m = Cin, concat of two tensors for decoder
//   convs, nearest-upsample folded in), B = dY_pre (n = Cout)  -> HWIO kernel grad.
// * tconv 2x2/2: A = dOut (m = Cout), B = layer input (n = Cin) -> (kh,kw,Cout,Cin).
// * first layer (SMALLC): m = (tap, ci) jointly, Cin in {4, 8}.
//
// Both operands are pixel-major in memory (channels contiguous), i.e. K is the
// strided dimension.  They are staged into LDS as [k][channel] images and the
// MFMA fragments (8 consecutive k per lane) are read with the gfx950
// hardware-transpose read `ds_read_b64_tr_b16` (cdna_hip_programming.md §5.5
// T10), two reads per fragment.  32-byte column blocks are XOR-swizzled by
// row so a half-wave's 8 rows land on disjoint banks (tools/lds_bank_model.py).
//
// A workgroup handles NTAP taps of one (m-tile, n-tile): the B tile (dY) is
// staged once and reused by every tap.  Splits write fp32 partial slabs that
// `wgrad_reduce_kernel` sums in a fixed order -> bitwise deterministic, no
// float atomics (SURVEY.md §5.2 deterministic-reduction mode).
//
// Reference: the gradients TF computes for Conv2D / Conv2DTranspose kernels
// and biases in `optimizer.compute_gradients` (`test_dist.py:248`).
#include "common.h"
#include "conv_params.h"

namespace unet {

namespace {

constexpr int NTHR = 256;
constexpr int BK = 32;  // pixels per K step

template <int NB>
__device__ __forceinline__ int trswz(int k) {
  if constexpr (NB == 2) return (k >> 3) & 1;
  if constexpr (NB == 4) return ((k >> 1) & 1) | (((k >> 3) & 1) << 1);
  if constexpr (NB >= 8) return (k & 3) | (((k >> 3) & 1) << 2);
  return 0;
}

// byte offset of element (k, c) in a [BK][W] bf16 image with swizzled 32-byte blocks
template <int W>
__device__ __forceinline__ int tr_off(int k, int c) {
  constexpr int NB = W / 16;
  return k * W * 2 + (((c >> 4) ^ trswz<NB>(k)) << 5) + ((c & 15) << 1);
}

template <int W>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int lane, int cbase) {
  // lane (g = lane>>4, i = lane&15, q = i>>2, p = i&3) supplies row 8g + 4h + q, cols cbase + 4p
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      LDS_PTR(short4v, img + tr_off<W>(8 * g + q, cbase + 4 * pp)));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      LDS_PTR(short4v, img + tr_off<W>(8 * g + 4 + q, cbase + 4 * pp)));
  // whole-vector bit casts: per-element short->bf16 casts miscompile (only the
  // first dword of each 64-bit transposed read survived in ROCm 7.2 hipcc)
  const u32x2 a = __builtin_bit_cast(u32x2, lo), b = __builtin_bit_cast(u32x2, hi);
  const u32x4 v = {a[0], a[1], b[0], b[1]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int BM, int BN, int NTAP, int WAVES_M, int WAVES_N, bool SMALLC, bool BIAS>
__global__ void __launch_bounds__(NTHR) wgrad_kernel(const WgradParams p) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_IMG = BK * BM * 2, B_IMG = BK * BN * 2;
  constexpr int STAGE = NTAP * A_IMG + B_IMG;
  constexpr int NA = NTAP * BM / 8;          // A chunks per k row
  constexpr int NCH = NA + BN / 8;           // chunks per k row
  constexpr int CPT = (NCH + 7) / 8;         // chunks per thread (8 threads per row)
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int KT = p.KD * p.KH * p.KW;
  const int Mtot = SMALLC ? (((KT * p.M1 + BM - 1) / BM) * BM) : (p.M1 + p.M2);
  const int tiles_m = Mtot / BM, tiles_n = p.Nc / BN;
  const int ntile = tiles_m * tiles_n * p.tap_groups;
  // blockIdx.x = split * ntile + tile   (splits of one tile spread over XCDs)
  const int split = blockIdx.x / ntile;
  int t = blockIdx.x - split * ntile;
  const int tg = t % p.tap_groups;
  t /= p.tap_groups;
  const int tn = t % tiles_n, tmi = t / tiles_n;
  const int m0 = tmi * BM, n0 = tn * BN;
  const int Q = p.N * p.QD * p.QH * p.QW;
  const int per = ((Q + p.splits - 1) / p.splits + BK - 1) / BK * BK;
  const int kbeg = split * per;
  const int kend = min(Q, kbeg + per);
  const int nks = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int upA = p.upA;
  const int upAd = p.AD > 1 ? upA : 1;  // 2D: depth is never upsampled
  const int AD1 = p.AD / upAd, AH1 = p.AH / upA, AW1 = p.AW / upA;
  const int Cin_s = p.M1;  // SMALLC: channels of the first-layer input
  const int padd = p.KD > 1 ? p.pad : 0;  // 2D: depth is not padded

  const int krow = tid >> 3, sub = tid & 7;
  // bias partial sums: mode 1 once per (n-tile, split) [tm == 0, tg == 0]; mode 2 once per (m-tile, tg, split) [tn == 0]
  const bool bias_on = BIAS && ((p.bias_mode == 1 && tmi == 0 && tg == 0) || (p.bias_mode == 2 && tn == 0));
  float bacc = 0.f;
  u32x4 reg[CPT];

  auto load = [&](int ks) {
    const int q = kbeg + ks * BK + krow;
    const bool qok = q < kend;
    int qn = 0, qd = 0, qh = 0, qw = 0;
    if (qok) {
      qw = q % p.QW;
      int r = q / p.QW;
      qh = r % p.QH;
      r /= p.QH;
      qd = r % p.QD;
      qn = r / p.QD;
    }
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int j = sub + 8 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (j < NA && qok) {
        const int tl = j / (BM / 8), col = j % (BM / 8);
        if constexpr (SMALLC) {
          // m = tap*Cin + ci ; a chunk = 8/Cin taps
          const int mm = m0 + col * 8;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if (e * Cin_s >= 8) break;
            const int tap = mm / Cin_s + e;
            if (tap >= KT) continue;
            const int kw = tap % p.KW, kh = (tap / p.KW) % p.KH, kd = tap / (p.KW * p.KH);
            const int ad = qd * p.stride + kd - padd, ah = qh * p.stride + kh - p.pad,
                      aw = qw * p.stride + kw - p.pad;
            if ((unsigned)ad >= (unsigned)p.AD || (unsigned)ah >= (unsigned)p.AH || (unsigned)aw >= (unsigned)p.AW)
              continue;
            const size_t pix = (((size_t)qn * p.AD + ad) * p.AH + ah) * p.AW + aw;
            const bf16* src = (const bf16*)p.a1 + pix * Cin_s;
            if (Cin_s == 8) {
              v = *(const u32x4*)src;
            } else {
              const u32x2 h = *(const u32x2*)src;
              v[2 * e] = h[0];
              v[2 * e + 1] = h[1];
            }
          }
        } else {
          const int tap = tg * NTAP + tl;
          const int kw = tap % p.KW, kh = (tap / p.KW) % p.KH, kd = tap / (p.KW * p.KH);
          const int ad = qd * p.stride + kd - padd, ah = qh * p.stride + kh - p.pad,
                    aw = qw * p.stride + kw - p.pad;
          if ((unsigned)ad < (unsigned)p.AD && (unsigned)ah < (unsigned)p.AH && (unsigned)aw < (unsigned)p.AW) {
            const int m = m0 + col * 8;
            const bf16* src;
            if (m < p.M1) {
              const size_t pix = (((size_t)qn * AD1 + ad / upAd) * AH1 + ah / upA) * AW1 + aw / upA;
              src = (const bf16*)p.a1 + pix * p.M1 + m;
            } else {
              const size_t pix = (((size_t)qn * p.AD + ad) * p.AH + ah) * p.AW + aw;
              src = (const bf16*)p.a2 + pix * p.M2 + (m - p.M1);
            }
            v = *(const u32x4*)src;
          }
        }
      } else if (j >= NA && j < NCH && qok) {
        const int col = j - NA;
        v = *(const u32x4*)((const bf16*)p.b + (size_t)q * p.Nc + n0 + col * 8);
      }
      reg[i] = v;
    }
  };
  auto store = [&](int buf) {
    char* S = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int j = sub + 8 * i;
      if (j < NA) {
        const int tl = j / (BM / 8), col = j % (BM / 8);
        *(u32x4*)(S + tl * A_IMG + tr_off<BM>(krow, col * 8)) = reg[i];
      } else if (j < NCH) {
        const int col = j - NA;
        *(u32x4*)(S + NTAP * A_IMG + tr_off<BN>(krow, col * 8)) = reg[i];
      }
    }
  };

  f32x4 acc[NTAP][TM][TN];
#pragma unroll
  for (int a = 0; a < NTAP; ++a)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[a][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nks > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
    const char* S = smem + buf * STAGE;
    bf16x8 bfr[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = tr_frag<BN>(S + NTAP * A_IMG, lane, wn * WN + j * 16);
#pragma unroll
    for (int a = 0; a < NTAP; ++a) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 af = tr_frag<BM>(S + a * A_IMG, lane, wm * WM + i * 16);
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[a][i][j] = mfma16(bfr[j], af, acc[a][i][j]);
      }
    }
    if constexpr (BIAS) {
      // column sums of the staged B image (mode 1) or of the WG's A images (mode 2)
      if (bias_on) {
        if (p.bias_mode == 1) {
          const int c = tid % BN;
          for (int k = tid / BN; k < BK; k += NTHR / BN)
            bacc += (float)*(const bf16*)(S + NTAP * A_IMG + tr_off<BN>(k, c));
        } else {
          const int c = tid % BM;
#pragma unroll
          for (int a = 0; a < NTAP; ++a)
            for (int k = tid / BM; k < BK; k += NTHR / BM) bacc += (float)*(const bf16*)(S + a * A_IMG + tr_off<BM>(k, c));
        }
      }
    }
    if (ks + 1 < nks) store(buf ^ 1);
    __syncthreads();
  }

  if constexpr (BIAS) {
    if (bias_on) {
      // reduce bacc over the threads sharing a column (deterministic order through LDS)
      float* red = (float*)smem;
      red[tid] = bacc;
      __syncthreads();
      const int W = p.bias_mode == 1 ? BN : BM;
      if (tid < W) {
        float s = 0.f;
        for (int k = tid; k < NTHR; k += W) s += red[k];
        const int base = p.bias_mode == 1 ? n0 : m0;
        const int Wtot = p.bias_mode == 1 ? p.Nc : Mtot;
        const int tgi = p.bias_mode == 1 ? 0 : tg;
        const int tgn = p.bias_mode == 1 ? 1 : p.tap_groups;
        p.bias_slab[((size_t)split * tgn + tgi) * Wtot + base + tid] = s;
      }
    }
  }

  // epilogue: C[n][m] orientation -> lane holds 4 consecutive n of one m
  const int KTs = SMALLC ? 1 : KT;
#pragma unroll
  for (int a = 0; a < NTAP; ++a) {
    const int tap = SMALLC ? 0 : tg * NTAP + a;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WM + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * WN + j * 16 + (lane >> 4) * 4;
        float* dst = p.slab + (((size_t)split * KTs + tap) * Mtot + m) * p.Nc + n;
        *(f32x4*)dst = acc[a][i][j];
      }
    }
  }
}

// out[t][m][n] (m < Mout) = scale * sum_s slab[s][t][m][n]   (Mtot >= Mout rows in the slab)
// Deterministic two-level reduction of the split-K slabs.
// Stage 1 (grid x = float4 chunks of a slab row, grid y = groups of G splits):
//   stage[y][i] = sum_{s in group y} slab[s][i]          (8 loads in flight per thread)
// Stage 2: out[o] = scale * sum_y stage[y][row_map(o)]   (rows remapped for the padded
//   first-layer input: output row o = grp*rkeep + j reads slab row grp*rg + j).
// With a single group, stage 1 writes the output directly (identity row map only).
constexpr int RED_G = 16;

__global__ void __launch_bounds__(256) slab_partial_kernel(const float* __restrict__ slab, int splits, size_t n4,
                                                           float* __restrict__ stage, float scale) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const int s0 = blockIdx.y * RED_G, s1 = min(splits, s0 + RED_G);
  const f32x4* src = (const f32x4*)slab + i;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int s = s0;
  for (; s + 4 <= s1; s += 4) {
    const f32x4 a = src[(size_t)s * n4], b = src[(size_t)(s + 1) * n4];
    const f32x4 c = src[(size_t)(s + 2) * n4], d = src[(size_t)(s + 3) * n4];
    acc += (a + b) + (c + d);
  }
  for (; s < s1; ++s) acc += src[(size_t)s * n4];
  ((f32x4*)stage)[(size_t)blockIdx.y * n4 + i] = acc * scale;
}

__global__ void __launch_bounds__(256) slab_final_kernel(const float* __restrict__ stage, int groups, int taps, int Mtot,
                                                         int Mout, int Nc, int rg, int rkeep,
                                                         float* __restrict__ out) {
  const size_t n4o = (size_t)taps * Mout * Nc / 4;
  const size_t n4 = (size_t)taps * Mtot * Nc / 4;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n4o) return;
  const size_t e = i * 4;
  const int n = e % Nc;
  const size_t r = e / Nc;
  const int mo = r % Mout;
  const int t = r / Mout;
  const int m = (mo / rkeep) * rg + (mo % rkeep);
  const size_t src = (((size_t)t * Mtot + m) * Nc + n) / 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int y = 0; y < groups; ++y) acc += ((const f32x4*)stage)[(size_t)y * n4 + src];
  ((f32x4*)out)[i] = acc;
}

// partial[b][c] = sum over rows r of block b of x[r][c]   (bf16 [rows][C], C % 8 == 0, C <= 1024)
__global__ void __launch_bounds__(256) colsum_kernel(const bf16* __restrict__ x, int rows, int C, int rows_per_block,
                                                     float* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) float red[];
  const int cpr = C / 8;                        // chunks per row
  const int rpi = 256 / cpr;                    // rows per iteration (C <= 2048)
  const int tid = threadIdx.x;
  const int cc = tid % cpr, rr = tid / cpr;
  float a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(rows, r0 + rows_per_block);
  if (rr < rpi) {
    for (int r = r0 + rr; r < r1; r += rpi) {
      const u32x4 v = *(const u32x4*)(x + (size_t)r * C + cc * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += f[e];
    }
  }
  // reduce across rr (deterministic tree in LDS)
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = (rr < rpi) ? a[e] : 0.f;
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    const int ch = c / 8, e = c % 8;
    float s = 0.f;
    for (int k = 0; k < rpi; ++k) s += red[(k * cpr + ch) * 8 + e];
    partial[(size_t)blockIdx.x * C + c] = s;
  }
}

template <int BM, int BN, int NTAP, int WAVES_M, int WAVES_N, bool SMALLC = false>
hipError_t launch_wg(WgradParams p, hipStream_t s) {
  const int KT = p.KD * p.KH * p.KW;
  const int Mtot = SMALLC ? (((KT * p.M1 + BM - 1) / BM) * BM) : (p.M1 + p.M2);
  p.tap_groups = SMALLC ? 1 : KT / NTAP;
  const int ntile = (Mtot / BM) * (p.Nc / BN) * p.tap_groups;
  const int grid = ntile * p.splits;
  if (p.bias_mode)
    hipLaunchKernelGGL((wgrad_kernel<BM, BN, NTAP, WAVES_M, WAVES_N, SMALLC, true>), dim3(grid), dim3(NTHR), 0, s, p);
  else
    hipLaunchKernelGGL((wgrad_kernel<BM, BN, NTAP, WAVES_M, WAVES_N, SMALLC, false>), dim3(grid), dim3(NTHR), 0, s, p);
  return hipGetLastError();
}

}  // namespace

WgradCfg wgrad_pick(const WgradParams& p) {
  const int KT = p.KD * p.KH * p.KW;
  const int M = p.M1 + p.M2;
  if ((p.M1 == 4 || p.M1 == 8) && p.M2 == 0) return {64, 32, 1, 1};
  if (M <= 64 && p.Nc <= 64 && KT % 9 == 0) return {32, 32, 9, 0};
  if (M <= 64 && p.Nc <= 64 && KT % 4 == 0) return {32, 32, 4, 0};
  if (M % 128 == 0 && p.Nc % 128 == 0) return {128, 128, 1, 0};
  if (KT % 3 == 0) return {64, 64, 3, 0};
  return {64, 64, 1, 0};
}

const char* wgrad_check(const WgradParams& p) {
  const int KT = p.KD * p.KH * p.KW;
  const WgradCfg c = wgrad_pick(p);
  const int M = p.M1 + p.M2;
  if (c.smallc) {
    if (p.upA != 1 || p.M2 != 0) return "wgrad: small-Cin mode supports plain convs";
    if (p.Nc % c.BN) return "wgrad: Nc must be a multiple of 32";
  } else {
    if (M % c.BM || p.Nc % c.BN) return "wgrad: channel counts not divisible by the tile";
    if (p.M1 % 8 || p.M2 % 8) return "wgrad: channel split must be a multiple of 8";
    if (KT % c.NTAP) return "wgrad: taps not divisible by the tap group";
  }
  if (p.upA != 1 && p.upA != 2) return "wgrad: upA must be 1 or 2";
  if (p.splits < 1) return "wgrad: splits must be >= 1";
  return nullptr;
}

hipError_t wgrad_launch(const WgradParams& p, hipStream_t s) {
  const WgradCfg c = wgrad_pick(p);
  if (c.smallc) return launch_wg<64, 32, 1, 2, 2, true>(p, s);
  if (c.BM == 32 && c.NTAP == 9) return launch_wg<32, 32, 9, 2, 2>(p, s);
  if (c.BM == 32 && c.NTAP == 4) return launch_wg<32, 32, 4, 2, 2>(p, s);
  if (c.BM == 128) return launch_wg<128, 128, 1, 2, 2>(p, s);
  if (c.NTAP == 3) return launch_wg<64, 64, 3, 2, 2>(p, s);
  return launch_wg<64, 64, 1, 2, 2>(p, s);
}

size_t wgrad_reduce_stage_floats(int splits, int taps, int Mtot, int Nc) {
  const int groups = (splits + RED_G - 1) / RED_G;
  return (size_t)groups * taps * Mtot * Nc;
}

hipError_t wgrad_reduce_launch(const float* slab, int splits, int taps, int Mtot, int Mout, int Nc, int rg, int rkeep,
                               float scale, float* out, float* stage, hipStream_t s) {
  if (rg <= 0) rg = Mout;
  if (rkeep <= 0) rkeep = rg;
  const bool identity = (Mout == Mtot) && (rg == rkeep);
  const int groups = (splits + RED_G - 1) / RED_G;
  const size_t n4 = (size_t)taps * Mtot * Nc / 4;
  const dim3 g1((unsigned)((n4 + 255) / 256), (unsigned)groups);
  if (groups == 1 && identity) {
    hipLaunchKernelGGL(slab_partial_kernel, g1, dim3(256), 0, s, slab, splits, n4, out, scale);
    return hipGetLastError();
  }
  if (!stage) return hipErrorInvalidValue;
  hipLaunchKernelGGL(slab_partial_kernel, g1, dim3(256), 0, s, slab, splits, n4, stage, scale);
  const size_t n4o = (size_t)taps * Mout * Nc / 4;
  hipLaunchKernelGGL(slab_final_kernel, dim3((unsigned)((n4o + 255) / 256)), dim3(256), 0, s, stage, groups, taps,
                     Mtot, Mout, Nc, rg, rkeep, out);
  return hipGetLastError();
}

hipError_t colsum_launch(const void* x, int rows, int C, int blocks, float* partial, hipStream_t s) {
  const int rpb = (rows + blocks - 1) / blocks;
  hipLaunchKernelGGL(colsum_kernel, dim3(blocks), dim3(256), 256 * 8 * sizeof(float), s, (const bf16*)x, rows, C,
                     rpb, partial);
  return hipGetLastError();
}

}  // namespace unet
