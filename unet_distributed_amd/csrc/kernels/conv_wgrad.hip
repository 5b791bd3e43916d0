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
#include "head_grad.h"
#include "conv_params.h"

namespace unet {

// splits handled by one launch: [split_lo, split_lo + split_n) of p.splits (0 = all)
static inline int launch_splits(const WgradParams& p) { return p.split_n > 0 ? p.split_n : p.splits - p.split_lo; }

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
__device__ __forceinline__ h16x8 tr_frag(const char* img, int lane, int cbase) {
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
  return __builtin_bit_cast(h16x8, v);
}

// BK = 64 pixels per K step; 4 threads per pixel row (tid >> 2 = row, tid & 3 = sub).
// With BM/8 a multiple of 4, the tap of chunk j = sub + 4i is j / (BM/8) = wave-uniform,
// so tap deltas come from SGPRs.  Pixel coordinates use shifts when the grid is a
// power of two (POW2), divisions otherwise.
template <int BM, int BN, int NTAP, int WAVES_M, int WAVES_N, bool SMALLC, bool BIAS, bool POW2>
__global__ void __launch_bounds__(NTHR) wgrad_kernel(const WgradParams p) {
  constexpr int BKW = 64;
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_IMG = BKW * BM * 2, B_IMG = BKW * BN * 2;
  constexpr int STAGE = NTAP * A_IMG + B_IMG;
  constexpr int NA = NTAP * BM / 8;          // A chunks per pixel row
  constexpr int NCH = NA + BN / 8;           // chunks per pixel row
  constexpr int CPT = NCH / 4;               // chunks per thread (4 threads per row)
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  static_assert((BM / 8) % 4 == 0 && NCH % 4 == 0, "chunk split");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int KT = p.KD * p.KH * p.KW;
  const int Mtot = SMALLC ? (((KT * p.M1 + BM - 1) / BM) * BM) : (p.M1 + p.M2);
  const int tiles_m = Mtot / BM, tiles_n = p.Nc / BN;
  const int ntile = tiles_m * tiles_n * p.tap_groups;
  // blockIdx.x = split * ntile + tile   (splits of one tile spread over XCDs)
  const int bid = (p.xcd & 2) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int lsplit = bid / ntile;
  const int split = p.split_lo + lsplit;
  int t = bid - lsplit * ntile;
  const int tg = t % p.tap_groups;
  t /= p.tap_groups;
  const int tn = t % tiles_n, tmi = t / tiles_n;
  const int m0 = tmi * BM, n0 = tn * BN;
  const int Q = p.N * p.QD * p.QH * p.QW;
  const int per = ((Q + p.splits - 1) / p.splits + BKW - 1) / BKW * BKW;
  const int kbeg = split * per;
  const int kend = min(Q, kbeg + per);
  const int nks = kend > kbeg ? (kend - kbeg + BKW - 1) / BKW : 0;
  const int padd = p.KD > 1 ? p.pad : 0;     // 2D: depth is not padded
  const int Cin_s = p.M1;                    // SMALLC: channels of the first-layer input

  const int krow = tid >> 2, sub = tid & 3;
  // SWP: odd pixel rows take their chunk groups in pair-swapped order (group c <-> c ^ 1,
  // same in load and store).  Rows are whole multiples of 128 bytes and the transposed-read
  // swizzle moves rows 2r, 2r + 1 by only one 32-byte block, so the 8 lanes of a 16-byte
  // store group (two rows x four chunks) otherwise land in one 64-byte half: 2-way
  // conflicted stores, 33 % conflict cycles on wgrad_kernel<128, 128> (r5 PMC pass).
  constexpr bool SWP = !SMALLC && (BM / 32) % 2 == 0 && (BN / 32) % 2 == 0;
  const int rsw = SWP ? (krow & 1) : 0;
  // bias partial sums: mode 1 once per (n-tile, split) [tm == 0, tg == 0]; mode 2 once per (m-tile, tg, split) [tn == 0]
  const bool bias_on = BIAS && ((p.bias_mode == 1 && tmi == 0 && tg == 0) || (p.bias_mode == 2 && tn == 0));

  constexpr int OOB = 0x7fffffff;
  const __amdgpu_buffer_rsrc_t ra1 = __builtin_amdgcn_make_buffer_rsrc((void*)p.a1, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t ra2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.a2 ? p.a2 : p.a1), (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rbb = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, (short)0, OOB, 0x00020000);

  u32x4 reg[CPT];

  auto load = [&](int ks) {
    const int q = kbeg + ks * BKW + krow;
    const bool qok = q < kend;
    int qn, qd, qh, qw;
    if (POW2) {
      qw = q & (p.QW - 1);
      int r = q >> p.lqw;
      qh = r & (p.QH - 1);
      r >>= p.lqh;
      qd = r & (p.QD - 1);
      qn = r >> p.lqd;
    } else {
      qw = q % p.QW;
      int r = q / p.QW;
      qh = r % p.QH;
      r /= p.QH;
      qd = r % p.QD;
      qn = r / p.QD;
    }
    const int bd = qd * p.stride - padd, bh = qh * p.stride - p.pad, bw = qw * p.stride - p.pad;
    const int pix0 = ((qn * p.AD + bd) * p.AH + bh) * p.AW + bw;     // window origin (full res)
    if constexpr (SMALLC) {
#pragma unroll
      for (int i = 0; i < NA / 4; ++i) {
        const int col = sub + 4 * i;
        u32x4 v = {0u, 0u, 0u, 0u};
        // m = tap*Cin + ci ; a chunk = 8/Cin taps (Cin in {4, 8})
        const int mm = m0 + col * 8;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          if (e * Cin_s >= 8) break;
          const int tap = mm / Cin_s + e;
          const int tt = tap < KT ? tap : 0;
          const int kw = tt % p.KW, kh = (tt / p.KW) % p.KH, kd = tt / (p.KW * p.KH);
          const bool ok = qok && tap < KT && (unsigned)(bd + kd) < (unsigned)p.AD &&
                          (unsigned)(bh + kh) < (unsigned)p.AH && (unsigned)(bw + kw) < (unsigned)p.AW;
          const int off = ((pix0 + (kd * p.AH + kh) * p.AW + kw) * Cin_s) * 2;
          if (Cin_s == 8) {
            v = __builtin_amdgcn_raw_buffer_load_b128(ra1, ok ? off : OOB, 0, 0);
          } else {
            const u32x2 h = __builtin_amdgcn_raw_buffer_load_b64(ra1, ok ? off : OOB, 0, 0);
            v[2 * e] = h[0];
            v[2 * e + 1] = h[1];
          }
        }
        reg[i] = v;
      }
    } else {
      constexpr int CPS = BM / 32;                  // chunks per thread per tap slot
#pragma unroll
      for (int tl = 0; tl < NTAP; ++tl) {
        // per (K step, tap slot): scalar tap offsets, one validity test, one base offset
        const int tap = tg * NTAP + tl;
        const int kw = __builtin_amdgcn_readfirstlane(p.tap_w[tap]);
        const int kh = __builtin_amdgcn_readfirstlane(p.tap_h[tap]);
        const int kd = __builtin_amdgcn_readfirstlane(p.tap_d[tap]);
        const bool ok = qok && (unsigned)(bd + kd) < (unsigned)p.AD && (unsigned)(bh + kh) < (unsigned)p.AH &&
                        (unsigned)(bw + kw) < (unsigned)p.AW;
        const int fpix = pix0 + (kd * p.AH + kh) * p.AW + kw;
        const int base1 = fpix * p.M1 * 2;
        const int base2 = (fpix * p.M2 - p.M1) * 2;
#pragma unroll
        for (int ci = 0; ci < CPS; ++ci) {
          const int m = m0 + (sub + 4 * (ci ^ rsw)) * 8;
          const int i = tl * CPS + ci;
          if (p.M2 == 0) {
            reg[i] = __builtin_amdgcn_raw_buffer_load_b128(ra1, ok ? base1 + m * 2 : OOB, 0, 0);
          } else {
            const bool f1 = m < p.M1;
            reg[i] = __builtin_amdgcn_raw_buffer_load_b128(ra1, (ok && f1) ? base1 + m * 2 : OOB, 0, 0) |
                     __builtin_amdgcn_raw_buffer_load_b128(ra2, (ok && !f1) ? base2 + m * 2 : OOB, 0, 0);
          }
        }
      }
    }
    const int bbase = q * p.Nc * 2 + n0 * 2;
#pragma unroll
    for (int i = NA / 4; i < CPT; ++i) {
      const int col = sub + 4 * ((i - NA / 4) ^ rsw);
      reg[i] = __builtin_amdgcn_raw_buffer_load_b128(rbb, qok ? bbase + col * 16 : OOB, 0, 0);
    }
  };
  auto store = [&](int buf) {
    char* S = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int j = sub + 4 * i;
      if (j < NA) {
        const int tl = (4 * i) / (BM / 8), col = sub + 4 * ((i - tl * (BM / 32)) ^ rsw);
        *(u32x4*)(S + tl * A_IMG + tr_off<BM>(krow, col * 8)) = reg[i];
      } else {
        const int col = sub + 4 * ((i - NA / 4) ^ rsw);
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
  // bias column sums ride on the MFMA pipe: one extra MFMA per fragment against a
  // constant all-ones operand (C[n][*] = sum_k B[k][n], or C[*][m] = sum_k A[k][m])
  constexpr int NF = BIAS ? (TN > TM ? TN : TM) : 1;
  f32x4 bacc[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) bacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  // wave-uniform scalar branches (readfirstlane) so the compiler does not predicate
  // the extra MFMAs with exec masks
  const bool do_b1 = BIAS && __builtin_amdgcn_readfirstlane((int)(bias_on && p.bias_mode == 1 && wm == 0));
  const bool do_b2 = BIAS && __builtin_amdgcn_readfirstlane((int)(bias_on && p.bias_mode == 2 && wn == 0));
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);

  if (nks > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int ks = 0; ks < nks; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nks) load(ks + 1);
    const char* S = smem + buf * STAGE;
#pragma unroll
    for (int h = 0; h < 2; ++h) {      // two k32 halves of the 64-pixel step
      h16x8 bfr[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tr_frag<BN>(S + NTAP * A_IMG + h * 32 * BN * 2, lane, wn * WN + j * 16);
      if constexpr (BIAS) {
        if (do_b1) {
#pragma unroll
          for (int j = 0; j < TN; ++j) bacc[j] = mfma16(bfr[j], ones, bacc[j]);
        }
      }
#pragma unroll
      for (int a = 0; a < NTAP; ++a) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const h16x8 af = tr_frag<BM>(S + a * A_IMG + h * 32 * BM * 2, lane, wm * WM + i * 16);
          if constexpr (BIAS) {
            if (do_b2) bacc[i] = mfma16(ones, af, bacc[i]);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[a][i][j] = mfma16(bfr[j], af, acc[a][i][j]);
        }
      }
    }
    if (ks + 1 < nks) store(buf ^ 1);
    __syncthreads();
  }

  if constexpr (BIAS) {
    if (bias_on) {
      // mode 1: bacc[j] = C[n = 4g + r][*], g = lane >> 4 -> lanes 0,16,32,48 hold 4 columns each
      // mode 2: bacc[i] = C[*][m = lane & 15]          -> lanes 0..15, register 0
      const int Wtot = p.bias_mode == 1 ? p.Nc : Mtot;
      const int tgi = p.bias_mode == 1 ? 0 : tg;
      const int tgn = p.bias_mode == 1 ? 1 : p.tap_groups;
      float* bs = p.bias_slab + ((size_t)split * tgn + tgi) * Wtot;
      if (p.bias_mode == 1 && wm == 0 && (lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j) *(f32x4*)(bs + n0 + wn * WN + j * 16 + (lane >> 4) * 4) = bacc[j];
      }
      if (p.bias_mode == 2 && wn == 0 && lane < 16) {
#pragma unroll
        for (int i = 0; i < TM; ++i) bs[m0 + wm * WM + i * 16 + lane] = bacc[i][0];
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


// Batched deterministic slab reduction: one launch per phase for a whole list of
// weight / bias gradients (a backward segment's worth), instead of two tiny launches
// per gradient.  Phase 1: stage[g][i] = sum of the splits of group g (groups of
// RED_G); jobs with a single group and an identity row map write the output directly.
// Phase 2: out[o] = sum_g stage[g][row_map(o)].  Threads find their job by a scan of
// the (few dozen) prefix offsets.
__global__ void __launch_bounds__(256) multi_reduce1_kernel(const ReduceJob* __restrict__ jobs, int njobs,
                                                            long long total) {
  // job ranges start on 256-thread boundaries (native_engine flush): the job is
  // block-uniform, so the scan and the job fields are scalar loads
  const long long b0 = blockIdx.x * 256LL, gi = b0 + threadIdx.x;
  if (gi >= total) return;
  int j = 0;
  while (j + 1 < njobs && jobs[j + 1].p1_begin <= b0) ++j;
  const ReduceJob& J = jobs[j];
  const long long local = gi - J.p1_begin;
  if (local >= (long long)J.groups * J.n4) return;   // the job range's padding
  const int g = (int)(local / J.n4);
  const long long i = local - (long long)g * J.n4;
  const int s0 = g * RED_G, s1 = min(J.splits, s0 + RED_G);
  const f32x4* src = (const f32x4*)J.slab + i;
  // all RED_G loads issued before the first add (one memory round trip; the kernel is
  // latency-bound), then a fixed pairwise tree (deterministic)
  f32x4 v[RED_G];
#pragma unroll
  for (int k = 0; k < RED_G; ++k)
    v[k] = s0 + k < s1 ? src[(size_t)(s0 + k) * J.n4] : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int w = 1; w < RED_G; w <<= 1)
#pragma unroll
    for (int k = 0; k + w < RED_G; k += 2 * w) v[k] += v[k + w];
  ((f32x4*)(J.direct ? J.out : J.stage))[(size_t)g * J.n4 + i] = v[0];
}

__global__ void __launch_bounds__(256) multi_reduce2_kernel(const ReduceJob* __restrict__ jobs, int njobs,
                                                            long long total) {
  const long long b0 = blockIdx.x * 256LL, gi = b0 + threadIdx.x;
  if (gi >= total) return;
  int j = 0;
  while (j + 1 < njobs && jobs[j + 1].p2_begin <= b0) ++j;
  const ReduceJob& J = jobs[j];
  const long long i = gi - J.p2_begin;
  if (J.direct || i >= J.n4o) return;
  const size_t e = i * 4;
  const int n = e % J.Nc;
  const size_t r = e / J.Nc;
  const int mo = r % J.Mout;
  const int t = r / J.Mout;
  const int m = (mo / J.rkeep) * J.rg + (mo % J.rkeep);
  const size_t src = (((size_t)t * J.Mtot + m) * J.Nc + n) / 4;
  const f32x4* st = (const f32x4*)J.stage + src;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int y = 0;
  for (; y + 8 <= J.groups; y += 8) {                 // 8 loads in flight per round trip
    f32x4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = st[(size_t)(y + k) * J.n4];
    acc += ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
  }
  for (; y < J.groups; ++y) acc += st[(size_t)y * J.n4];
  ((f32x4*)J.out)[i] = acc;
}

// partial[b][c] = sum over rows r of block b of x[r][c]   (bf16 [rows][C], C % 8 == 0, C <= 1024)
__global__ void __launch_bounds__(256) colsum_kernel(const h16* __restrict__ x, int rows, int C, int rows_per_block,
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
    // (unrolled: 8 row loads in flight per thread instead of one dependent load per add;
    // the adds keep their row order)
#pragma unroll 8
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
  for (int t = 0; t < 27; ++t) p.tap_d[t] = p.tap_h[t] = p.tap_w[t] = 0;
  for (int t = 0; t < KT && t < 27; ++t) {
    p.tap_w[t] = (signed char)(t % p.KW);
    p.tap_h[t] = (signed char)((t / p.KW) % p.KH);
    p.tap_d[t] = (signed char)(t / (p.KW * p.KH));
  }
  const int Mtot = SMALLC ? (((KT * p.M1 + BM - 1) / BM) * BM) : (p.M1 + p.M2);
  p.tap_groups = SMALLC ? 1 : KT / NTAP;
  const int ntile = (Mtot / BM) * (p.Nc / BN) * p.tap_groups;
  const int grid = ntile * launch_splits(p);
  auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  auto lg = [](int v) { int l = 0; while ((1 << l) < v) ++l; return l; };
  const bool p2 = pow2(p.QW) && pow2(p.QH) && pow2(p.QD);
  p.lqw = lg(p.QW);
  p.lqh = lg(p.QH);
  p.lqd = lg(p.QD);
  if (p.bias_mode) {
    if (p2)
      UNET_LAUNCH((wgrad_kernel<BM, BN, NTAP, WAVES_M, WAVES_N, SMALLC, true, true>), dim3(grid), dim3(NTHR), 0, s, p);
    else
      UNET_LAUNCH((wgrad_kernel<BM, BN, NTAP, WAVES_M, WAVES_N, SMALLC, true, false>), dim3(grid), dim3(NTHR), 0, s, p);
  } else {
    if (p2)
      UNET_LAUNCH((wgrad_kernel<BM, BN, NTAP, WAVES_M, WAVES_N, SMALLC, false, true>), dim3(grid), dim3(NTHR), 0, s, p);
    else
      UNET_LAUNCH((wgrad_kernel<BM, BN, NTAP, WAVES_M, WAVES_N, SMALLC, false, false>), dim3(grid), dim3(NTHR), 0, s, p);
  }
  return launch_status();
}


// ---------------------------------------------------------------------------------
// Row-window weight gradient (2D 3x3 stride 1 'same', full rows of W in {8,16,32,64,128}).
//
// The tiled kernel above stages one A image per tap (9 copies of the input tile):
// at the fine levels, where Cin and Cout are 32..64, that LDS traffic bounds it at
// ~160 TF.  Here a workgroup walks a contiguous range of 256-pixel windows (R = 256/W
// whole rows of the flattened (n, h) row space) and, per window, LDS-DMAs ONE halo
// image of the input rows (32 channels) plus the dY rows of its 32*QO output
// channels.  Every tap then reads its shifted A fragments from that single image
// with the hardware transpose read (ds_read_b64_tr_b16 -> 8 pixels of one channel
// per lane), the dY fragments are read once per 32-pixel step and reused by all nine
// taps, and the partial dW (9 x 32 x 32 per wave) stays in registers across windows.
// Waves split output channels (QO) and pixel steps (4 / QO); pixel-split partials are
// summed through LDS and each workgroup writes one fp32 slab (deterministic reduce).
// Images: 64-byte pixel slots; 16-byte chunk c of the slot in column col is stored at
// c ^ (((col >> 3) & 1) << 1), which makes the transposed fragment reads conflict free
// (tools/lds_bank_model.py) and depends only on col mod 16 (DMA lane roles fixed).
// GEO: 0 = 2D full rows, 1 = 2D segmented rows (Wf = p.QW > W), 2 = 3D (tap group =
// depth tap); compile-time so the 2D full-row kernel carries no segment / depth state.
enum { WGEO_2D = 0, WGEO_SEG = 1, WGEO_3D = 2 };
// HG: head-on-load (conv_params.h HeadGrad): the B operand (dY of the head input, 32
// channels, 2D full rows) is formed per window from the head's per-pixel probability,
// target and ReLU bits instead of being read from memory.
// PAIR (round 6, column-unit path): wave w owns the 16-channel half jh = w & 1 of its
// 32-channel output block, so its dW partial is 9 x 32 x 16 (72 registers instead of 144)
// and the kernel fits three workgroups per CU (the 3D level-1 weight gradients were half
// waits at two); the pixel splits halve and each x fragment feeds two waves.
// DZ (xform 2, 2D single source, rows 16..64 wide): the B operand is the layer's norm
// backward dz = ca g + cb z + cc formed on load -- p.b = g is DMA'd as usual, each thread's
// z granules are loaded with it and the staged g image is rewritten in place (the
// norm_bwd_apply formula and rounding; coefficients of the window's sample in LDS, Ks).
template <int W, int QO, bool CONCAT, int GEO, bool HG = false, bool PAIR = false, bool DZ = false>
__global__ void __launch_bounds__(NTHR, PAIR ? 3 : 2) wgrad_win_kernel(const WgradParams p) {
  constexpr int BMW = 256, R = BMW / W, HR = R + 2;
  constexpr int HWP = ((W + 2 + 15) / 16) * 16, IPR = HWP / 16, ROWB = HWP * 64;
  constexpr int XI = HR * IPR, YI = QO * BMW / 16;
  constexpr int XB = XI * 1024, YB = YI * 1024;
  constexpr int PS = 4 / QO, KS = BMW / 32;
  constexpr int REDB = 4 * 64 * 16 * 4;                 // one tap of every wave's partials
  constexpr int KB = DZ ? 3 * 32 * QO * 4 : 0;         // DZ: ca / cb / cc of the block's channels
  constexpr int LDS_BYTES = (XB + YB + KB > REDB) ? XB + YB + KB : REDB;
  static_assert(W >= 8 && W <= 128 && (QO == 1 || QO == 2), "window wgrad shape");
  static_assert(!DZ || (GEO == WGEO_2D && !HG && !PAIR && !CONCAT && W >= 16 && W <= 64 && QO == 1),
                "dz on load: 2D single-source full rows 16..64 wide");
  static_assert(!HG || (QO == 1 && !CONCAT && (GEO == WGEO_2D || GEO == WGEO_3D) && BMW == NTHR),
                "head-on-load B: one 32-channel image (2D rows or 3D slices)");
  static_assert(!PAIR || (W >= 32 && !HG), "wave-pair partials: column-unit path");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ys = smem + XB;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // PAIR: wave = (ps, qo, jh) from the top bit down; pixel splits PSP = 2 / QO
  constexpr int PSP = PAIR ? 2 / QO : PS;
  const int jh = PAIR ? wave & 1 : 0;
  const int qo = PAIR ? (wave >> 1) % QO : wave % QO, ps = PAIR ? (wave >> 1) / QO : wave / QO;
  // Row space g = (n, d, h), rows of Wf pixels cut into nseg W-wide segments (Wf > 128);
  // a window is R rows x one segment.  3D: tap group kd (grid dimension) computes the
  // nine (dh, dw) taps of depth tap kd from the halo rows of slice d + kd - 1.
  constexpr int KD = GEO == WGEO_3D ? 3 : 1;
  const int H = p.QH;
  const int D = GEO == WGEO_3D ? p.QD : 1;
  const int Wf = GEO == WGEO_SEG ? p.QW : W;
  const int nseg = GEO == WGEO_SEG ? p.QW / W : 1;
  const int rows_total = p.N * D * H;
  const int Mq = rows_total * Wf;
  const int nwin = ((rows_total + R - 1) / R) * nseg;
  const int Mtot = p.M1 + p.M2;
  const int cob = p.Nc / (32 * QO);
  const int ntile = (Mtot / 32) * cob * KD;
  // (p.xcd bit 0: the tiles of one split -- which read the same dY / input windows --
  // run on one XCD and share its L2)
  const int bid = (p.xcd & 1) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int lsplit = bid / ntile;
  const int split = p.split_lo + lsplit;
  int tile = bid - lsplit * ntile;
  const int kd = tile % KD;
  tile /= KD;
  const int ci_blk = tile / cob, co_blk = tile - ci_blk * cob;
  const int ci0 = ci_blk * 32, co0 = co_blk * 32 * QO;
  const bool from1 = !CONCAT || ci0 < p.M1;
  const int CA = from1 ? p.M1 : p.M2, ca0 = from1 ? ci0 : ci0 - p.M1;
  constexpr int OOB = 0x7fffffff;
  // window-relative buffer bases (rebuilt per window, scalar): 32-bit DMA offsets count
  // from the window's first halo row, so the tensors may exceed 2 GiB
  const char* abase = (const char*)(from1 ? p.a1 : p.a2);
  const char* bbase = (const char*)p.b;
  const int w_begin = (int)((long long)split * nwin / p.splits);
  const int w_end = (int)((long long)(split + 1) * nwin / p.splits);
  // bias: once per output-channel block, by the centre depth tap (it sees every window)
  const bool do_bias = p.bias_mode == 1 && ci_blk == 0 && kd == (KD >> 1);
  const int gsh = (kd - (KD >> 1)) * H;

  constexpr int NJ = PAIR ? 1 : 2;                      // 16-channel output halves per wave
  f32x4 acc[9][2][NJ];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) bacc[j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);

  // LDS-DMA lane roles (slot 16k + lslot, physical chunk lane & 3)
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ (((lslot >> 3) & 1) << 1);
  const int xl = ((lslot - 1) * CA + ca0 + lchunk * 8) * 2;
  // 8-wide rows: a 32-pixel step spans 4 halo rows whose slots sit 1 KB apart (same
  // banks), so odd halo rows additionally flip chunk bit 1 -- the transposed A reads of
  // lanes in rows r and r + 1 then hit disjoint banks (was 2-way, 49 % conflict cycles)
  constexpr bool ROWSWZ = W == 8;
  const int xl_odd = ((lslot - 1) * CA + ca0 + (lchunk ^ 2) * 8) * 2;
  const int yl = (lslot * p.Nc + co0 + lchunk * 8) * 2;
  // transposed-read lane roles: group G = lane >> 4 covers pixels 8G .. 8G + 7 of a
  // 32-pixel step; lane 4q + pp addresses pixel 8G + 4hh + q, channels 4pp .. 4pp + 3
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;

  auto tr_addr = [&](int slot, int col, int ch, int row = 0) -> int {   // ch: channel within the 32-ch slot
    const int swz = (((col >> 3) & 1) ^ (ROWSWZ ? (row & 1) : 0)) << 1;
    return slot * 64 + (((ch >> 3) ^ swz) << 4) + ((ch & 7) << 1);
  };
  auto tr8 = [&](const char* base0, const char* base1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };

  // column-unit path (below): the window never spans two images (H % R == 0,
  // wgrad_win_eligible), so halo rows of a neighbouring image are DMA'd as zeros and
  // its tap loop needs no image-edge branches
  constexpr bool UNITS_PATH = W >= 32 && W / 32 <= PS;
  // 16-wide rows (row-pair path): a 32-pixel K step is a pair of rows, and each wave
  // owns R / PS consecutive output rows.  The A fragment of halo rows (hr, hr + 1) at
  // shift dw feeds every output pair y = hr - dh with y even: rows of even hr serve
  // dh = 0 and 2, odd hr dh = 1, so per window a wave reads (2 NP + 1) x 6 A
  // fragments instead of NP x 18 (25 % fewer LDS reads; this kernel is LDS-read
  // bound at W = 16).  Needs windows inside one image (halo rows of the neighbour
  // image are then DMA'd as zeros, as on the column-unit path).
  constexpr bool PAIR_PATH = W == 16 && GEO == WGEO_2D;
  constexpr bool pair_ok = PAIR_PATH;   // wgrad_win_eligible: QH % 16 == 0 for 16-wide rows
  HeadGradCtx hctx{};
  if constexpr (HG) hctx = head_grad_ctx(p.hg);
  // DZ: thread t rewrites granules u = t + 256 c of the B image: image o = c / 4, slot
  // (t >> 2) + 64 (c & 3), physical chunk t & 3 = logical chunk dzl (the slot swizzle bit
  // (slot >> 3) & 1 is (t >> 5) & 1 for every c): channels co0 + 32 o + 8 dzl ..
  float* Ks = (float*)(smem + XB + YB);
  const int dzl = (tid & 3) ^ (((tid >> 5) & 1) << 1);
  int ks_n = -1;                                        // sample whose coefficients Ks holds
  // CARRY (128-wide rows, 2D / 3D: two-row windows, four halo rows): consecutive windows of
  // one image share two halo rows -- the previous window's logical rows 2, 3 are the next
  // one's 0, 1 -- so only two new rows are DMA'd (18 of 36 KB) and logical row r lives at
  // physical row r ^ 2 fl, fl flipping with every carry (conv_dw.hip's halo-row carry)
  constexpr bool CARRY = UNITS_PATH && W == 128 && (GEO == WGEO_2D || GEO == WGEO_3D);
  int fl = 0, prev = -2;
  for (int win = w_begin; win < w_end; ++win) {
    const int g0 = (GEO == WGEO_SEG ? win / nseg : win) * R;
    const int col0 = GEO == WGEO_SEG ? (win % nseg) * W : 0;
    // 3D: a window lies in one (n, d) slice (H % R == 0); its depth-shifted input slice
    // is padding -> the window contributes nothing to this tap group (uniform skip)
    if (GEO == WGEO_3D && (unsigned)((g0 / H) % D + kd - 1) >= (unsigned)D) continue;
    const bool zero_halo = UNITS_PATH || pair_ok;
    const bool top_in = !zero_halo || (g0 % H) != 0, bot_in = !zero_halo || ((g0 + R) % H) != 0;
    // (top_in: the previous window's bottom halo rows are this image's rows, not zeros)
    const bool carry = CARRY && prev == win - 1 && top_in;
    if constexpr (CARRY) {
      fl = carry ? fl ^ 1 : 0;
      prev = win;
    }
    const int kb = carry ? 2 * IPR : 0;                 // first halo piece to load
    const int rb = max(g0 - 1 + gsh, 0);             // first halo row held by rsa
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(abase + (size_t)rb * Wf * CA * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(bbase + (size_t)g0 * Wf * p.Nc * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsz = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((DZ ? (const char*)p.xz : bbase) + (size_t)g0 * Wf * p.Nc * 2), (short)0, OOB, 0x00020000);
    __syncthreads();   // the previous window's fragment reads are done
#pragma unroll
    for (int qq = 0; qq < (XI + 3) / 4; ++qq) {
      const int k = kb + wave + 4 * qq;
      if (k < XI) {
        const int hr = k / IPR, j = k - hr * IPR;
        const int gr = g0 - 1 + hr + gsh;
        const int col = col0 + 16 * j + lslot - 1;
        const bool row_in = (hr > 0 || top_in) && (hr < R + 1 || bot_in);
        const bool ok = row_in && (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)Wf &&
                        (GEO != WGEO_SEG || 16 * j + lslot <= W + 1);
        const int off = ok ? ((gr - rb) * Wf + col0 + 16 * j) * CA * 2 + ((ROWSWZ && (hr & 1)) ? xl_odd : xl) : OOB;
        const int pk = CARRY && fl ? k + (hr < 2 ? 2 * IPR : -2 * IPR) : k;   // (CARRY: physical row hr ^ 2 fl)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (__attribute__((address_space(3))) void*)(Xs + pk * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    if constexpr (HG) {
      // thread t forms window pixel t (slot t; logical chunk k at physical k ^ swizzle)
      const int pix = g0 * W + tid;
      u32x4 v[4] = {{0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}, {0u, 0u, 0u, 0u}};
      if (pix < Mq) head_grad_pixel(p.hg, hctx, pix, v);
      const int sw = ((tid >> 3) & 1) << 1;
      // store order rotated by (t / 2) mod 4: the 8 lanes of a store group then write 8
      // different 16-byte bank groups (same order in every lane: 2-way conflicted, 41 %
      // LDS conflict cycles on this kernel, r3_pmc_table.md); values picked by selects, not
      // a dynamically indexed register array
      const int rot = (tid >> 1) & 3;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int kk = (k + rot) & 3;
        const u32x4 w = kk == 0 ? v[0] : (kk == 1 ? v[1] : (kk == 2 ? v[2] : v[3]));
        *(u32x4*)(Ys + tid * 64 + 16 * (kk ^ sw)) = w;
      }
    }
#pragma unroll
    for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (!HG && k < YI) {
        const int o = k / (BMW / 16), sb = (k - o * (BMW / 16)) * 16;   // image o, first slot
        // window slot sb -> row g0 + sb / W, column col0 + sb % W (W = 8: one segment,
        // the 16-slot run covers two consecutive rows contiguous in memory)
        const int pix = GEO == WGEO_SEG ? (g0 + sb / W) * Wf + col0 + sb % W : g0 * W + sb;
        const int off = (pix + lslot < Mq) ? ((pix - g0 * Wf) * p.Nc + 32 * o) * 2 + yl : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (__attribute__((address_space(3))) void*)(Ys + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    u32x4 zq[DZ ? 4 * QO : 1];
    if constexpr (DZ) {
      const int n = p.xcs ? g0 / H : 0;                 // (windows never span two images: rows_ok)
      if (n != ks_n) {                                  // (the loop-top barrier ordered the old reads)
        ks_n = n;
        if (tid < 3 * 32 * QO) {
          const int m = tid / (32 * QO), c = tid - m * 32 * QO;
          Ks[tid] = (m == 0 ? p.xa : m == 1 ? p.xb : p.xc)[(size_t)n * p.xcs + co0 + c];
        }
      }
#pragma unroll
      for (int c = 0; c < 4 * QO; ++c) {
        const int pix = g0 * W + (tid >> 2) + 64 * (c & 3);
        zq[c] = __builtin_amdgcn_raw_buffer_load_b128(
            rsz, pix < Mq ? ((pix - g0 * W) * p.Nc + co0 + 32 * (c >> 2) + 8 * dzl) * 2 : OOB, 0, 0);
      }
    }
    __syncthreads();
    if constexpr (DZ) {
#pragma unroll
      for (int o = 0; o < QO; ++o) {
        float ka[8], kz[8], kk[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int ch = 32 * o + 8 * dzl + e;
          ka[e] = Ks[ch];
          kz[e] = Ks[32 * QO + ch];
          kk[e] = Ks[64 * QO + ch];
        }
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const int c = 4 * o + c4;
          if (g0 * W + (tid >> 2) + 64 * c4 >= Mq) continue;   // past the tensor: stays zero
          u32x4* a = (u32x4*)(Ys + (tid + NTHR * c) * 16);
          float gv[8], zv[8];
          unpack8(*a, gv);
          unpack8(zq[c], zv);
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = fmaf(ka[e], gv[e], fmaf(kz[e], zv[e], kk[e]));
          *a = pack8(gv);
        }
      }
      __syncthreads();
    }
    const char* Yq = Ys + qo * (BMW * 64);
    // (one column unit per wave: with two, the 128-wide QO = 2 case spills)
    if constexpr (UNITS_PATH) {
      // Column units: 32 pixels wide x RWG rows.  The dY fragments of the unit's rows
      // stay in registers; each halo-row A fragment (row hr, shift dw) is read once
      // and feeds the output rows hr - dh of all three vertical taps, so a unit reads
      // 3 (RWG + 2) A fragment pairs instead of 9 RWG.
      constexpr int NCOL = W / 32;
      constexpr int RG = PSP > NCOL ? PSP / NCOL : 1;
      constexpr int RWG = R / RG;
      constexpr int UNITS = NCOL * RG;
      static_assert(R % RG == 0 && RWG >= 1, "wgrad column units");
      static_assert(!CARRY || (RWG == R && R == 2), "halo-row carry: one two-row unit per column");
      // CARRY: logical halo row hr at physical hr ^ 2 fl -- rows 0, 1 shifted by +xsh, 2, 3 by -xsh
      const int xsh = (CARRY && fl) ? 2 * ROWB : 0;
      const int lp = 8 * G + q;
#pragma unroll 1
      for (int u = ps; u < UNITS; u += PSP) {
        const int cu = u % NCOL, rr0 = (u / NCOL) * RWG;
        const int c0 = cu * 32;
        // Per-lane LDS byte bases (the swizzle depends only on lp + dw because c0 and
        // the row pitches are multiples of 32 slots): halo row hr and dY row y are
        // compile-time immediates on top of these 16 registers.
        int ab[3][2][2], yb[NJ][2];
#pragma unroll
        for (int dw = 0; dw < 3; ++dw)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              const int col = c0 + dw + lp + 4 * hh;
              ab[dw][i][hh] = tr_addr(rr0 * HWP + col, col, 16 * i + 4 * pp);
            }
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int sl = rr0 * W + c0 + lp + 4 * hh;
            yb[j][hh] = tr_addr(sl, sl, 16 * (PAIR ? jh : j) + 4 * pp);
          }
        // dY fragments of the unit's rows, loaded when first needed (halo row hr = y
        // feeds output row y through dh = 0) and live for three halo rows; pixels past
        // the tensor were DMA'd as zeros
        h16x8 bf[RWG][NJ];
#pragma unroll
        for (int hr = 0; hr < RWG + 2; ++hr) {
          if (hr < RWG) {
#pragma unroll
            for (int j = 0; j < NJ; ++j) bf[hr][j] = tr8(Yq + yb[j][0] + hr * W * 64, Yq + yb[j][1] + hr * W * 64);
            if (do_bias) {
#pragma unroll
              for (int j = 0; j < NJ; ++j) bacc[j] = mfma16(ones, bf[hr][j], bacc[j]);
            }
          }
#pragma unroll
          for (int dw = 0; dw < 3; ++dw) {
            h16x8 af[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
              const int ro = hr * ROWB + (CARRY ? (hr < 2 ? xsh : -xsh) : 0);
              af[i] = tr8(Xs + ab[dw][i][0] + ro, Xs + ab[dw][i][1] + ro);
            }
#pragma unroll
            for (int dh = 0; dh < 3; ++dh) {
              const int y = hr - dh;
              if (y < 0 || y >= RWG) continue;
#pragma unroll
              for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[3 * dh + dw][i][j] = mfma16(af[i], bf[y][j], acc[3 * dh + dw][i][j]);
            }
          }
          // keep the scheduler from hoisting every row's fragment reads to the top
          // (144 accumulator registers leave room for about one row of fragments)
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      continue;
    }
    if constexpr (PAIR_PATH) {
      {
        constexpr int NP = R / 2 / PS;             // output row pairs per wave
        const int y0 = ps * 2 * NP;                // first output row (window-relative)
        const int lp = 8 * G + q;                  // lane pixel of a 32-pixel step
        const int lr = lp >> 4, lc = lp & 15;      // its row in the pair, its column
        // halo row of output row y, tap dh is y + dh (halo row 0 = window row -1)
        int ab[3][2][2];
#pragma unroll
        for (int dw = 0; dw < 3; ++dw)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
              const int col = lc + dw + 4 * hh;
              ab[dw][i][hh] = tr_addr((y0 + lr) * HWP + col, col, 16 * i + 4 * pp);
            }
        // dY fragments of output pair k: loaded at hr = 2k (first use, dh = 0), last
        // used at hr = 2k + 2 (dh = 2) -- at most two pairs live
        h16x8 bf[NP][NJ];
#pragma unroll
        for (int hr = 0; hr <= 2 * NP; ++hr) {
          if (!(hr & 1) && hr < 2 * NP) {
            const int s0 = (y0 + hr) * W + lp, s1 = s0 + 4;
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              bf[hr >> 1][j] = tr8(Yq + tr_addr(s0, s0, 16 * j + 4 * pp), Yq + tr_addr(s1, s1, 16 * j + 4 * pp));
            if (do_bias) {
#pragma unroll
              for (int j = 0; j < NJ; ++j) bacc[j] = mfma16(ones, bf[hr >> 1][j], bacc[j]);
            }
          }
#pragma unroll
          for (int dw = 0; dw < 3; ++dw) {
            h16x8 af[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) af[i] = tr8(Xs + ab[dw][i][0] + hr * ROWB, Xs + ab[dw][i][1] + hr * ROWB);
#pragma unroll
            for (int dh = 0; dh < 3; ++dh) {
              const int y = hr - dh;
              if (y < 0 || y >= 2 * NP || (y & 1)) continue;
#pragma unroll
              for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j)
                  acc[3 * dh + dw][i][j] = mfma16(af[i], bf[y >> 1][j], acc[3 * dh + dw][i][j]);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        continue;
      }
    }
#pragma unroll 1
    for (int kk = ps; kk < KS; kk += PS) {
      const int px0 = kk * 32;
      const int rr = px0 / W, c0 = px0 - rr * W;
      const int g = g0 + rr;
      if (g >= rows_total) break;
      const int h = g % H;
      // dY fragments (B operand: k = pixels, n = output channels)
      h16x8 bf[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int s0 = px0 + 8 * G + q, s1 = s0 + 4;
        bf[j] = tr8(Yq + tr_addr(s0, s0, 16 * j + 4 * pp), Yq + tr_addr(s1, s1, 16 * j + 4 * pp));
      }
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < NJ; ++j) bacc[j] = mfma16(ones, bf[j], bacc[j]);
      }
      // lane pixel 8G + q (+4 for the second transposed read): for rows narrower than
      // a 32-pixel step it lies lr rows below the step's first row, at column lc
      const int lp = 8 * G + q;
      const int lr = W >= 32 ? 0 : lp / W, lc = W >= 32 ? lp : lp - (lp / W) * W;
      const int hl = W >= 32 ? h : (g + lr) % H;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dh = t / 3, dw = t % 3;
        if (W >= 32 && ((dh == 0 && h == 0) || (dh == 2 && h == H - 1))) continue;   // zero-padding rows
        const bool lane_ok = W >= 32 || !((dh == 0 && hl == 0) || (dh == 2 && hl == H - 1));
        const int colA = c0 + dw + lc;              // halo column of this lane's first pixel
        const int slotA = (rr + lr + dh) * HWP + colA;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int rowA = rr + lr + dh;            // halo row (row swizzle of 8-wide rows)
          h16x8 af = tr8(Xs + tr_addr(slotA, colA, 16 * i + 4 * pp, rowA),
                          Xs + tr_addr(slotA + 4, colA + 4, 16 * i + 4 * pp, rowA));
          if (W < 32 && !lane_ok) af = __builtin_bit_cast(h16x8, (u32x4){0u, 0u, 0u, 0u});
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[t][i][j] = mfma16(af, bf[j], acc[t][i][j]);
        }
      }
    }
  }

  // ---- reduce the pixel-split partials (waves with the same qo) and write the slab
  // acc[t][i][j][r] = dW[t][ci0 + 16i + 4(lane>>4) + r][co0 + 32qo + 16j + (lane&15)]
  float* red = (float*)smem;
  const int n_base = co0 + 32 * qo + (lane & 15) + 16 * jh;
  const int m_base = ci0 + 4 * (lane >> 4);
  // (PAIR: the partner waves of (qo, jh) are ((o QO + qo) 2 + jh), o < PSP)
  auto partner = [&](const int o) { return PAIR ? (o * QO + qo) * 2 + jh : qo + QO * o; };
  auto reduce_store = [&](const f32x4 (&v4)[2][NJ], const int t) {
    __syncthreads();
    // red[fragment (i, j)][wave * 64 + lane]: consecutive lanes 16 bytes apart (a lane-major
    // [lane][4 fragments] layout puts the 8 lanes of a 16-byte store group 64 bytes apart,
    // two 64-byte positions per 128-byte bank window: 4-way conflicted stores and loads)
    if (PSP > 1 && ps > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) *(f32x4*)(red + ((i * 2 + j) * NTHR + wave * 64 + lane) * 4) = v4[i][j];
    }
    __syncthreads();
    if (ps == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          f32x4 v = v4[i][j];
#pragma unroll
          for (int o = 1; o < PSP; ++o) v += *(const f32x4*)(red + ((i * 2 + j) * NTHR + partner(o) * 64 + lane) * 4);
          if (t < 9) {
            float* dst = p.slab + (((size_t)split * 9 * KD + 9 * kd + t) * Mtot + m_base + 16 * i) * p.Nc + n_base + 16 * j;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)r * p.Nc] = v[r];
          } else if (i == 0 && lane < 16) {
            p.bias_slab[(size_t)split * p.Nc + n_base + 16 * j] = v[0];
          }
        }
    }
  };
#pragma unroll
  for (int t = 0; t < 9; ++t) reduce_store(acc[t], t);
  if (do_bias) {
    const f32x4 z = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 bv[2][NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      bv[0][j] = bacc[j];
      bv[1][j] = z;
    }
    reduce_store(bv, 9);
  }
}


// ---------------------------------------------------------------------------------
// Prefetching 128-wide window weight gradient (option wg_pf; 2D / 3D, 32-channel output
// block).  wgrad_win_kernel<128, 1> stages each window by LDS-DMA and waits for it: at two
// workgroups per CU the 3D level-1 weight gradients ran ~4.5 us per window against ~0.5 us
// of MFMA work -- one HBM round trip per window, exposed.  Here the halo-row carry leaves
// two new input rows (18 KB) + the dY image (16 KB) per window, 9 x 16 bytes per thread:
// they are loaded into registers right after the current window's data is in LDS, fly under
// its MFMAs, and are written to LDS after them (one barrier pair per window, as before).  A
// window that cannot carry (the first of a workgroup or of an image) loads synchronously.
// Same LDS images, swizzles, fragment reads, MFMA order and reduction as wgrad_win_kernel
// with CARRY: bit-identical slabs.  xform 1 (BatchNorm, single source): the A operand is the
// pre-norm z of a normalised activation, relu(xa z + xb) formed in registers before the LDS
// store (padding stays zero) -- the activation itself need not be stored (norm_pool's y);
// coefficients [C] (BatchNorm) or [N][C] (GroupNorm, xcs = C: refreshed per image).
template <bool CONCAT, int GEO, bool AXF = false>
__global__ void __launch_bounds__(NTHR, 2) wgrad_pf128_kernel(const WgradParams p) {
  constexpr int W = 128, BMW = 256, R = 2, HWP = 144, IPR = 9, ROWB = HWP * 64;
  constexpr int XI = (R + 2) * IPR, YI = BMW / 16, XB = XI * 1024, YB = YI * 1024;
  constexpr int REDB = 4 * 64 * 16 * 4;
  constexpr int LDS_BYTES = (XB + YB + 256 > REDB) ? XB + YB + 256 : REDB;
  static_assert(!AXF || (!CONCAT && GEO == WGEO_2D), "A on load: 2D single source");
  constexpr int NX = (2 * IPR + 3) / 4, NY = YI / 4;    // pieces per wave: new rows, dY
  static_assert(GEO == WGEO_2D || GEO == WGEO_3D, "2D / 3D full rows");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ys = smem + XB;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ps = wave;                                  // pixel split = column unit (QO = 1)
  constexpr int KD = GEO == WGEO_3D ? 3 : 1;
  const int H = p.QH;
  const int D = GEO == WGEO_3D ? p.QD : 1;
  const int rows_total = p.N * D * H;
  const int Mq = rows_total * W;
  const int nwin = rows_total / R;
  const int Mtot = p.M1 + p.M2;
  const int cob = p.Nc / 32;
  const int ntile = (Mtot / 32) * cob * KD;
  const int bid = (p.xcd & 1) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int lsplit = bid / ntile;
  const int split = p.split_lo + lsplit;
  int tile = bid - lsplit * ntile;
  const int kd = tile % KD;
  tile /= KD;
  const int ci_blk = tile / cob, co_blk = tile - ci_blk * cob;
  const int ci0 = ci_blk * 32, co0 = co_blk * 32;
  const bool from1 = !CONCAT || ci0 < p.M1;
  const int CA = from1 ? p.M1 : p.M2, ca0 = from1 ? ci0 : ci0 - p.M1;
  constexpr int OOB = 0x7fffffff;
  const char* abase = (const char*)(from1 ? p.a1 : p.a2);
  const char* bbase = (const char*)p.b;
  const int w_begin = (int)((long long)split * nwin / p.splits);
  const int w_end = (int)((long long)(split + 1) * nwin / p.splits);
  const bool do_bias = p.bias_mode == 1 && ci_blk == 0 && kd == (KD >> 1);
  const int gsh = (kd - (KD >> 1)) * H;

  f32x4 acc[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);

  // lane roles of wgrad_win_kernel's LDS-DMA (slot 16k + lslot, physical chunk lane & 3)
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ (((lslot >> 3) & 1) << 1);
  const int xl = ((lslot - 1) * CA + ca0 + lchunk * 8) * 2;
  const int yl = (lslot * p.Nc + co0 + lchunk * 8) * 2;
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto tr_addr = [&](int slot, int col, int ch) -> int {
    const int swz = ((col >> 3) & 1) << 1;
    return slot * 64 + (((ch >> 3) ^ swz) << 4) + ((ch & 7) << 1);
  };
  auto tr8 = [&](const char* base0, const char* base1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };

  // xform 1: the block's 32 channels' xa / xb in LDS (BatchNorm: one set for the launch)
  float* Kx = (float*)(smem + XB + YB);
  constexpr bool axf = AXF;
  if (axf && tid < 64 && !p.xcs) Kx[tid] = (tid < 32 ? p.xa : p.xb)[ca0 + (tid & 31)];
  // halo pieces k = kb + wave + 4 i (i < NX) of window `win` (input rows g0 - 1 + hr + gsh)
  u32x4 xr[NX], yr[NY];
  uint32_t xokm = 0;
  auto load_x = [&](const int win, const int kb) {
    const int g0 = win * R;
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const int rb = max(g0 - 1 + gsh, 0);
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(abase + (size_t)rb * W * CA * 2), (short)0, OOB, 0x00020000);
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int k = kb + wave + 4 * i;
      const int hr = k / IPR, j = k - hr * IPR;
      const int gr = g0 - 1 + hr + gsh;
      const int col = 16 * j + lslot - 1;
      const bool ok = k < kb + 2 * IPR && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                      (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
      xokm = i ? (xokm | ((ok ? 1u : 0u) << i)) : (ok ? 1u : 0u);
      xr[i] = __builtin_amdgcn_raw_buffer_load_b128(rsa, ok ? ((gr - rb) * W + 16 * j) * CA * 2 + xl : OOB, 0, 0);
    }
  };
  auto load_y = [&](const int win) {
    const int g0 = win * R;
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(bbase + (size_t)g0 * W * p.Nc * 2), (short)0, OOB, 0x00020000);
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const int sb = (wave + 4 * i) * 16;
      const int pix = g0 * W + sb;
      yr[i] = __builtin_amdgcn_raw_buffer_load_b128(rsb, pix + lslot < Mq ? sb * p.Nc * 2 + yl : OOB, 0, 0);
    }
  };
  // (logical halo row hr at physical row hr ^ 2 fl; every slot of the row pieces is written:
  // out-of-range loads return zeros, as the DMA leaves them)
  auto store_x = [&](const int kb, const int fl) {
    if (axf) {
      const float* ka = Kx + lchunk * 8;
#pragma unroll
      for (int i = 0; i < NX; ++i) {
        if (!((xokm >> i) & 1u)) continue;
        float f[8];
        unpack8(xr[i], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(ka[e], f[e], ka[32 + e]), 0.f);
        xr[i] = pack8(f);
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int k = kb + wave + 4 * i;
      if (k < kb + 2 * IPR) {
        const int hr = k / IPR;
        const int pk = fl ? k + (hr < 2 ? 2 * IPR : -2 * IPR) : k;
        *(u32x4*)(Xs + pk * 1024 + lane * 16) = xr[i];
      }
    }
  };
  auto store_y = [&]() {
#pragma unroll
    for (int i = 0; i < NY; ++i) *(u32x4*)(Ys + (wave + 4 * i) * 1024 + lane * 16) = yr[i];
  };

  int fl = 0, prev = -2, pwin = -1;
  for (int win = w_begin; win < w_end; ++win) {
    const int g0 = win * R;
    if (GEO == WGEO_3D && (unsigned)((g0 / H) % D + kd - 1) >= (unsigned)D) continue;
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const bool carry = prev == win - 1 && top_in;
    fl = carry ? fl ^ 1 : 0;
    prev = win;
    __syncthreads();                                   // the previous window's fragment reads are done
    if (!(carry && pwin == win)) {
      // not prefetched: this window's rows (all four unless it carries) and dY, synchronously
      if (!carry) {
        load_x(win, 0);
        if constexpr (AXF) {
          if (p.xcs) {
            // GroupNorm: the coefficients of this image's sample (a carried window never
            // changes image, so only these windows refresh them)
            if (tid < 64) Kx[tid] = (tid < 32 ? p.xa : p.xb)[(size_t)(g0 / H) * p.xcs + ca0 + (tid & 31)];
            __syncthreads();
          }
        }
        store_x(0, fl);
      }
      load_x(win, 2 * IPR);
      load_y(win);
    }
    store_x(2 * IPR, fl);
    store_y();
    pwin = -1;
    if (win + 1 < w_end && bot_in) {
      // the next window carries (same image, not a depth-padding window: same slice): its
      // two new rows and dY fly under this window's MFMAs
      load_x(win + 1, 2 * IPR);
      load_y(win + 1);
      pwin = win + 1;
    }
    __syncthreads();
    {
      const int c0 = ps * 32;
      const int lp = 8 * G + q;
      const int xsh = fl ? 2 * ROWB : 0;
      int ab[3][2][2], yb[2][2];
#pragma unroll
      for (int dw = 0; dw < 3; ++dw)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int col = c0 + dw + lp + 4 * hh;
            ab[dw][i][hh] = tr_addr(col, col, 16 * i + 4 * pp);
          }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int sl = c0 + lp + 4 * hh;
          yb[j][hh] = tr_addr(sl, sl, 16 * j + 4 * pp);
        }
      h16x8 bf[R][2];
#pragma unroll
      for (int hr = 0; hr < R + 2; ++hr) {
        if (hr < R) {
#pragma unroll
          for (int j = 0; j < 2; ++j) bf[hr][j] = tr8(Ys + yb[j][0] + hr * W * 64, Ys + yb[j][1] + hr * W * 64);
          if (do_bias) {
#pragma unroll
            for (int j = 0; j < 2; ++j) bacc[j] = mfma16(ones, bf[hr][j], bacc[j]);
          }
        }
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          h16x8 af[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const int ro = hr * ROWB + (hr < 2 ? xsh : -xsh);
            af[i] = tr8(Xs + ab[dw][i][0] + ro, Xs + ab[dw][i][1] + ro);
          }
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int y = hr - dh;
            if (y < 0 || y >= R) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int j = 0; j < 2; ++j) acc[3 * dh + dw][i][j] = mfma16(af[i], bf[y][j], acc[3 * dh + dw][i][j]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }

  // ---- reduce the pixel-split partials of the four waves and write the slab (as wgrad_win_kernel)
  float* red = (float*)smem;
  const int n_base = co0 + (lane & 15);
  const int m_base = ci0 + 4 * (lane >> 4);
  auto reduce_store = [&](const f32x4 (&v4)[2][2], const int t) {
    __syncthreads();
    if (ps > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) *(f32x4*)(red + ((i * 2 + j) * NTHR + wave * 64 + lane) * 4) = v4[i][j];
    }
    __syncthreads();
    if (ps == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 v = v4[i][j];
#pragma unroll
          for (int o = 1; o < 4; ++o) v += *(const f32x4*)(red + ((i * 2 + j) * NTHR + o * 64 + lane) * 4);
          if (t < 9) {
            float* dst = p.slab + (((size_t)split * 9 * KD + 9 * kd + t) * Mtot + m_base + 16 * i) * p.Nc + n_base + 16 * j;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)r * p.Nc] = v[r];
          } else if (i == 0 && lane < 16) {
            p.bias_slab[(size_t)split * p.Nc + n_base + 16 * j] = v[0];
          }
        }
    }
  };
#pragma unroll
  for (int t = 0; t < 9; ++t) reduce_store(acc[t], t);
  if (do_bias) {
    const f32x4 z = (f32x4){0.f, 0.f, 0.f, 0.f};
    f32x4 bv[2][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bv[0][j] = bacc[j];
      bv[1][j] = z;
    }
    reduce_store(bv, 9);
  }
}


// ---------------------------------------------------------------------------------
// First-layer row-window weight gradient (CIN = 4 or 8 padded input channels).
// GEMM rows m = (tap, channel) (36 or 72, padded to MT x 16), columns = 32 output
// channels, K = pixels.  The halo image uses the first-layer forward's slot layout
// (8- or 16-byte slots, row pitch W + 4, slot 0 always zero).  A fragments come from
// the transposed LDS read with per-lane addresses: lane 4q + pp of a 16-lane group
// supplies pixel q's slot for tap 4mt + pp (CIN 4) or tap 2mt + pp/2 and channel half
// pp & 1 (CIN 8), so the transpose hands lane i the (tap, channel) row 16 mt + i; taps
// past the ninth and taps whose input row leaves the pixel's image address slot 0.
// D3 (3x3x3, CIN 4): the halos of the three depth slices d - 1, d, d + 1 of the window are
// staged together (zeros past the volume), GEMM rows m = (9 kd + t) CIN + c over the 27 taps
// (MT = 7 row tiles); a row tile may span two depth slices, its lanes just address their own
// slice's halo.
template <int W, int CIN, bool XF = false, bool D3 = false>
__global__ void __launch_bounds__(NTHR) wgrad_win_first_kernel(const WgradParams p) {
  // Row pitch in slots: CIN 4 (8-byte slots) pads it to == 16 (mod 32) -- the four taps of
  // an A fragment (4 mt .. 4 mt + 3) then read slot sets that never share banks (a vertical
  // neighbour RS slots on lands 64 bytes x 2 away from the row's own slots), and GEMM rows
  // past the ninth tap (discarded) read 16 slots on instead of the broadcast zero slot
  // (round 4: W + 4 = 132 -- 37.5 % of the kernel's LDS cycles were conflicts).
  // (256-pixel windows; a window is one row on rows 512 wide -- the 512^2 model)
  constexpr int BMW = W > 256 ? W : 256, R = BMW / W, HR = R + 2, SB = 2 * CIN;
  constexpr int RS = CIN == 4 ? ((W + 4 + 15) / 32) * 32 + 16 : W + 4, ROWB = RS * SB;
  constexpr int CPR = ROWB / 16;
  constexpr int NS = D3 ? 3 : 1;                      // staged depth slices
  constexpr int XI = (NS * HR * CPR + 63) / 64, YI = BMW / 16;
  constexpr int XB = XI * 1024, YB = YI * 1024;
  constexpr int NT = D3 ? 27 : 9;                     // taps
  constexpr int MT = (NT * CIN + 15) / 16;
  static_assert(!D3 || (CIN == 4 && !XF), "3D first-layer window wgrad: 4 padded channels");
  constexpr int KS = BMW / 32;
  // (cross-wave reduction rows padded to an odd number of 16-byte units: a lane stride of
  // NV = 2 MT + 2 units (128 bytes at MT = 3) put all 8 lanes of a 16-byte store group on
  // the same banks -- 8-way; r5 PMC pass: 14.5 % conflict cycles)
  constexpr int REDB = 4 * 64 * (MT * 2 + 3) * 16;
  constexpr int LDS_BYTES = (XB + YB > REDB) ? XB + YB : REDB;
  static_assert(W >= 16 && W <= 512, "first-layer window wgrad");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ys = smem + XB;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.QH, D = D3 ? p.QD : 1;
  const int rows_total = p.N * D * H;
  const int Mq = rows_total * W;
  const int nwin = (rows_total + R - 1) / R;
  const int Mtot = MT * 16;
  const int cot = p.Nc / 32;
  const int bid = (p.xcd & 1) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int lsplit = bid / cot, co_blk = bid - lsplit * cot;
  const int split = p.split_lo + lsplit;
  const int co0 = co_blk * 32;
  constexpr int OOB = 0x7fffffff;
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.a1, (short)0, OOB, 0x00020000);
  const int w_begin = (int)((long long)split * nwin / p.splits);
  const int w_end = (int)((long long)(split + 1) * nwin / p.splits);
  const bool do_bias = p.bias_mode == 1;

  f32x4 acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ (((lslot >> 3) & 1) << 1);
  const int yl = (lslot * p.Nc + co0 + lchunk * 8) * 2;
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;

  auto tr_addr = [&](int slot, int col, int ch) -> int {
    return slot * 64 + ((((ch >> 3) ^ (((col >> 3) & 1) << 1))) << 4) + ((ch & 7) << 1);
  };
  auto tr8 = [&](const char* base0, const char* base1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };

  // XF: this lane's B-transform coefficients (its logical chunk lchunk is fixed)
  float xa[8], xb[8], xc[8];
  for (int win = w_begin; win < w_end; ++win) {
    const int g0 = win * R;
    // dY window base (scalar): the 32-bit DMA offsets stay window-relative (> 2 GiB dY)
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.b + (size_t)g0 * W * p.Nc * 2), (short)0, OOB, 0x00020000);
    __syncthreads();
    u32x4 xzv[(YI + 3) / 4];
    if constexpr (XF) {
      // the pre-norm z of this lane's dY chunks, loaded beside the DMA
      const size_t crow = p.xcs ? (size_t)(g0 / H) * p.xcs : 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xa[e] = p.xa[crow + co0 + lchunk * 8 + e];
        xb[e] = p.xb[crow + co0 + lchunk * 8 + e];
        xc[e] = p.xc[crow + co0 + lchunk * 8 + e];
      }
#pragma unroll
      for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
        const int k = wave + 4 * qq;
        const int pix = g0 * W + 16 * k + lslot;
        if (k < YI && pix < Mq)
          xzv[qq] = *(const u32x4*)((const h16*)p.xz + (size_t)pix * p.Nc + co0 + lchunk * 8);
      }
    }
#pragma unroll
    for (int qq = 0; qq < (XI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < XI) {
        const int u = 64 * k + lane;
        const int hr3 = u / CPR, c = u - hr3 * CPR;
        const int kd = D3 ? hr3 / HR : 0, hr = hr3 - kd * HR;     // (3D: slice d + kd - 1)
        const int gr = g0 - 1 + hr + (D3 ? (kd - 1) * H : 0);
        const int col = CIN == 4 ? 2 * c - 2 : c - 2;
        const int dd = D3 ? (g0 / H) % D + kd - 1 : 0;
        const bool ok = hr3 < NS * HR && (unsigned)dd < (unsigned)D && (unsigned)gr < (unsigned)rows_total &&
                        (unsigned)col < (unsigned)W;
        const int off = ok ? ((gr * W + col) * CIN) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (__attribute__((address_space(3))) void*)(Xs + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < YI) {
        const int pix = g0 * W + 16 * k;
        const int off = (pix + lslot < Mq) ? 16 * k * p.Nc * 2 + yl : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (__attribute__((address_space(3))) void*)(Ys + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    __syncthreads();
    if constexpr (XF) {
      // B operand dz = xa g + xb z + xc formed in place (each lane rewrites the chunk its
      // own DMA lane role wrote); pixels past the tensor keep the DMA's zeros
#pragma unroll
      for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
        const int k = wave + 4 * qq;
        if (k < YI && g0 * W + 16 * k + lslot < Mq) {
          char* a = Ys + k * 1024 + lslot * 64 + (lane & 3) * 16;
          float gv[8], zv[8];
          unpack8(*(const u32x4*)a, gv);
          unpack8(xzv[qq], zv);
#pragma unroll
          for (int e = 0; e < 8; ++e) gv[e] = fmaf(xa[e], gv[e], fmaf(xb[e], zv[e], xc[e]));
          *(u32x4*)a = pack8(gv);
        }
      }
      __syncthreads();
    }
#pragma unroll 1
    for (int kk = wave; kk < KS; kk += 4) {
      const int px0 = kk * 32;
      if (g0 + px0 / W >= rows_total) break;
      h16x8 bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int s0 = px0 + 8 * G + q, s1 = s0 + 4;
        bf[j] = tr8(Ys + tr_addr(s0, s0, 16 * j + 4 * pp), Ys + tr_addr(s1, s1, 16 * j + 4 * pp));
      }
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 2; ++j) bacc[j] = mfma16(ones, bf[j], bacc[j]);
      }
      // this lane's two pixels (second transposed read: +4)
      int slotp[2], hlp[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int px = px0 + 8 * G + 4 * hh + q;
        const int rr = px / W, cw = px - rr * W;
        slotp[hh] = rr * RS + cw + 1;        // tap (dh, dw) adds dh * RS + dw
        hlp[hh] = (g0 + rr) % H;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int t3 = CIN == 4 ? 4 * mt + pp : 2 * mt + (pp >> 1);
        const int kd = D3 ? t3 / 9 : 0, t = t3 - 9 * kd;
        const int chb = CIN == 4 ? 0 : (pp & 1) * 8;
        const int dh = t / 3, dw = t - 3 * dh;
        int a[2];
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const bool ok = t3 < NT && !(dh == 0 && hlp[hh] == 0) && !(dh == 2 && hlp[hh] == H - 1);
          a[hh] = ok ? (slotp[hh] + (kd * HR + dh) * RS + dw) * SB + chb
                     : (t3 >= NT && CIN == 4 ? (slotp[hh] + 16) * SB : 0);
        }
        const h16x8 af = tr8(Xs + a[0], Xs + a[1]);
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[mt][j] = mfma16(af, bf[j], acc[mt][j]);
      }
    }
  }

  // cross-wave reduce (all four waves split pixels), then one slab per workgroup:
  // acc[mt][j][r] = dW[m = 16 mt + 4 (lane >> 4) + r][co0 + 16 j + (lane & 15)]
  __syncthreads();
  float* red = (float*)smem;
  constexpr int NV = MT * 2 + 2, NVP = NV | 1;
  {
    float* dst = red + (wave * 64 + lane) * NVP * 4;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int j = 0; j < 2; ++j) *(f32x4*)(dst + (mt * 2 + j) * 4) = acc[mt][j];
    *(f32x4*)(dst + (MT * 2) * 4) = bacc[0];
    *(f32x4*)(dst + (MT * 2 + 1) * 4) = bacc[1];
  }
  __syncthreads();
  for (int idx = tid; idx < 64 * NV; idx += NTHR) {
    const int ln = idx / NV, v = idx - ln * NV;
    f32x4 sum = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 4; ++w) sum += *(const f32x4*)(red + ((w * 64 + ln) * NVP + v) * 4);
    const int n = co0 + (ln & 15);
    if (v < MT * 2) {
      const int mt = v >> 1, j = v & 1;
      const int m = 16 * mt + 4 * (ln >> 4);
      float* dst = p.slab + ((size_t)split * Mtot + m) * p.Nc + n + 16 * j;
#pragma unroll
      for (int r = 0; r < 4; ++r) dst[(size_t)r * p.Nc] = sum[r];
    } else if (do_bias && ln < 16) {
      p.bias_slab[(size_t)split * p.Nc + n + 16 * (v - MT * 2)] = sum[0];
    }
  }
}

template <int CIN>
hipError_t launch_wgrad_win_first(const WgradParams& p, hipStream_t s) {
  const int grid = (p.Nc / 32) * launch_splits(p);
  if constexpr (CIN == 4) {
    if (p.KD == 3) {          // (wgrad_win_first3_eligible: the caller checked)
      switch (p.QW) {
        case 16: UNET_LAUNCH((wgrad_win_first_kernel<16, 4, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
        case 32: UNET_LAUNCH((wgrad_win_first_kernel<32, 4, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
        case 64: UNET_LAUNCH((wgrad_win_first_kernel<64, 4, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
        default: UNET_LAUNCH((wgrad_win_first_kernel<128, 4, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      }
      return launch_status();
    }
  }
  if (p.xform == 2) {         // dz formed on load (norm backward of the first layer)
    switch (p.QW) {
      case 16: UNET_LAUNCH((wgrad_win_first_kernel<16, CIN, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 32: UNET_LAUNCH((wgrad_win_first_kernel<32, CIN, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 64: UNET_LAUNCH((wgrad_win_first_kernel<64, CIN, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 256: UNET_LAUNCH((wgrad_win_first_kernel<256, CIN, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 512: UNET_LAUNCH((wgrad_win_first_kernel<512, CIN, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      default: UNET_LAUNCH((wgrad_win_first_kernel<128, CIN, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
    }
    return launch_status();
  }
  switch (p.QW) {
    case 16: UNET_LAUNCH((wgrad_win_first_kernel<16, CIN>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 32: UNET_LAUNCH((wgrad_win_first_kernel<32, CIN>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 64: UNET_LAUNCH((wgrad_win_first_kernel<64, CIN>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 256: UNET_LAUNCH((wgrad_win_first_kernel<256, CIN>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 512: UNET_LAUNCH((wgrad_win_first_kernel<512, CIN>), dim3(grid), dim3(NTHR), 0, s, p); break;
    default: UNET_LAUNCH((wgrad_win_first_kernel<128, CIN>), dim3(grid), dim3(NTHR), 0, s, p); break;
  }
  return launch_status();
}


// ---------------------------------------------------------------------------------
// 2x2 stride-2 transposed-conv weight gradient on windows of whole coarse rows:
//   dW[t][co][ci] = sum_{coarse px} dy[fine(px, t)][co] * x[px][ci],  bias = sum dy.
// Per window the workgroup LDS-DMAs the coarse x rows (32 input channels) and the 2R
// fine dy rows (32 output channels, even / odd columns de-interleaved so a tap's
// pixels are consecutive slots); both operands are read with ds_read_b64_tr_b16.
// Slab contract of the tiled kernel: slab[split][tap][co][ci], bias_slab[split][co].
template <int W, int QN>
__global__ void __launch_bounds__(NTHR) wgrad_tconv_win_kernel(const WgradParams p) {
  // QN 32-channel blocks of x per workgroup (one per wave); PS = 4 / QN waves split pixels.
  // The fine dy slice of the co block is then staged once per window for all of them.
  constexpr int BMc = 128, R = BMc / W, FW = 2 * W;
  constexpr int PS = 4 / QN;
  constexpr int XI = QN * BMc / 16, YI = 2 * R * FW / 16;
  constexpr int XB = XI * 1024, YB = YI * 1024;
  constexpr int KS = BMc / 32;
  constexpr int REDB = 4 * 64 * 16 * 4;
  constexpr int LDS_BYTES = (XB + YB > REDB) ? XB + YB : REDB;
  static_assert(W >= 32 && W <= 64 && (QN == 1 || QN == 2 || QN == 4), "tconv window wgrad");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ys = smem + XB;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qn = wave % QN, ps = wave / QN;
  const int H = p.QH;                       // coarse grid
  const int rows_total = p.N * H;
  const int Mq = rows_total * W;
  const int fine_rows_total = 2 * rows_total;
  const int nwin = (rows_total + R - 1) / R;
  const int Mtot = p.M1;                    // output channels of the transposed conv
  const int cit = p.Nc / (32 * QN);
  const int ntile = (Mtot / 32) * cit;
  const int bid = (p.xcd & 1) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int lsplit = bid / ntile, tile = bid - lsplit * ntile;
  const int split = p.split_lo + lsplit;
  const int co_blk = tile / cit, ci_blk = tile - co_blk * cit;
  const int co0 = co_blk * 32, ci0 = ci_blk * 32 * QN;
  constexpr int OOB = 0x7fffffff;
  const int w_begin = (int)((long long)split * nwin / p.splits);
  const int w_end = (int)((long long)(split + 1) * nwin / p.splits);
  const bool do_bias = p.bias_mode == 2 && ci_blk == 0 && qn == 0;

  f32x4 acc[4][2][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i) acc[t][i][0] = acc[t][i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ (((lslot >> 3) & 1) << 1);
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto tr_addr = [&](int slot, int ch) -> int {   // swizzle keyed on slot mod 16
    return slot * 64 + ((((ch >> 3) ^ (((slot >> 3) & 1) << 1))) << 4) + ((ch & 7) << 1);
  };
  auto tr8 = [&](const char* base0, const char* base1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };
  const char* Xq = Xs + qn * (BMc * 64);

  for (int win = w_begin; win < w_end; ++win) {
    const int g0 = win * R;
    // window-relative bases (scalar): 32-bit DMA offsets, tensors beyond 2 GiB
    const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.b + (size_t)g0 * W * p.Nc * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.a1 + (size_t)2 * g0 * FW * Mtot * 2), (short)0, OOB, 0x00020000);
    __syncthreads();
#pragma unroll
    for (int qq = 0; qq < (XI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < XI) {
        const int o = k / (BMc / 16), sb = (k - o * (BMc / 16)) * 16;   // x image o (channel block)
        const int pix = g0 * W + sb + lslot;
        const int off = pix < Mq ? ((sb + lslot) * p.Nc + ci0 + 32 * o + lchunk * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (__attribute__((address_space(3))) void*)(Xs + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < YI) {
        const int sl = 16 * k + lslot;
        const int frr = sl / FW, s = sl - frr * FW;
        const int col = s < W ? 2 * s : 2 * (s - W) + 1;
        const int gf = 2 * g0 + frr;
        const int off = gf < fine_rows_total ? ((frr * FW + col) * Mtot + co0 + lchunk * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsy, (__attribute__((address_space(3))) void*)(Ys + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int kk = ps; kk < KS; kk += PS) {
      const int px0 = kk * 32;
      const int rr = px0 / W, c0 = px0 - rr * W;
      if (g0 + rr >= rows_total) break;
      h16x8 bf[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int s0 = px0 + 8 * G + q;
        bf[j] = tr8(Xq + tr_addr(s0, 16 * j + 4 * pp), Xq + tr_addr(s0 + 4, 16 * j + 4 * pp));
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int th = t >> 1, tw = t & 1;
        const int s0 = (2 * rr + th) * FW + tw * W + c0 + 8 * G + q;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const h16x8 af = tr8(Ys + tr_addr(s0, 16 * i + 4 * pp), Ys + tr_addr(s0 + 4, 16 * i + 4 * pp));
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[t][i][j] = mfma16(af, bf[j], acc[t][i][j]);
          if (do_bias) bacc[i] = mfma16(af, ones, bacc[i]);
        }
      }
    }
  }

  // reduce the PS pixel-split partials of each channel block through LDS, then write
  // acc[t][i][j][r] = dW[t][co0 + 16i + 4(lane>>4) + r][ci0 + 32 qn + 16j + (lane&15)]
  float* red = (float*)smem;
  auto reduce_store = [&](const f32x4 (&v4)[2][2], const int t) {
    __syncthreads();
    // red[fragment (i, j)][wave * 64 + lane]: consecutive lanes 16 bytes apart (a lane-major
    // [lane][4 fragments] layout puts the 8 lanes of a 16-byte store group 64 bytes apart,
    // two 64-byte positions per 128-byte bank window: 4-way conflicted stores and loads)
    if (PS > 1 && ps > 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) *(f32x4*)(red + ((i * 2 + j) * NTHR + wave * 64 + lane) * 4) = v4[i][j];
    }
    __syncthreads();
    if (ps == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 v = v4[i][j];
#pragma unroll
          for (int o = 1; o < PS; ++o) v += *(const f32x4*)(red + ((i * 2 + j) * NTHR + (qn + QN * o) * 64 + lane) * 4);
          const int m = co0 + 16 * i + 4 * (lane >> 4), n = ci0 + 32 * qn + 16 * j + (lane & 15);
          if (t < 4) {
            float* o = p.slab + (((size_t)split * 4 + t) * Mtot + m) * p.Nc + n;
#pragma unroll
            for (int r = 0; r < 4; ++r) o[(size_t)r * p.Nc] = v[r];
          } else if (qn == 0 && j == 0 && (lane & 15) == 0) {   // bias: channel-block-0 waves only
#pragma unroll
            for (int r = 0; r < 4; ++r) p.bias_slab[(size_t)split * Mtot + m + r] = v[r];
          }
        }
    }
  };
#pragma unroll
  for (int t = 0; t < 4; ++t) reduce_store(acc[t], t);
  if (p.bias_mode == 2 && ci_blk == 0) {     // uniform over the workgroup (qn > 0 waves hold zeros)
    const f32x4 z = (f32x4){0.f, 0.f, 0.f, 0.f};
    const f32x4 bv[2][2] = {{bacc[0], z}, {bacc[1], z}};
    reduce_store(bv, 4);
  }
}

// Composite transposed-conv slab sums (tconv_fused.hip) on windows of whole coarse rows:
//   slab[split][4 sh + sw][o][k] = sum_{coarse px (h, w)} dz[2h + sh - 1][2w + sw - 1][o] * b[h][w][k]
//   bias_slab[split][4 sh + sw][o] = sum_{(h, w)} dz[2h + sh - 1][2w + sw - 1][o]
// (the generic tiled kernel with 4x4 taps re-read the coarse operand once per tap).  Per
// window of R = 128 / W coarse rows the workgroup LDS-DMAs the coarse b rows (QN 32-channel
// blocks, read once for all 16 taps) and the 2R + 2 fine dz rows 2 g0 - 1 .. 2 g0 + 2R with
// even / odd columns de-interleaved (even e = 0..W-1 at slots 0..W-1, zero at W; zero at
// W + 1, odd o = 0..W-1 at W + 2..2W + 1), so every tap's pixels are consecutive slots.
// Wave sh owns the four taps (sh, sw): column shift sw - 1 reads odd column w - 1 (sw 0),
// even w (1), odd w (2), even w + 1 (3).  Both operands go through ds_read_b64_tr_b16.
template <int W, int QN>
__global__ void __launch_bounds__(NTHR) wgrad_s2d_win_kernel(const WgradParams p) {
  constexpr int BMc = 128, R = BMc / W, FP = 2 * W + 2, FR = 2 * R + 2;
  constexpr int XI = QN * BMc / 16, YI = (FR * FP + 15) / 16;
  constexpr int XB = XI * 1024, YB = YI * 1024;
  constexpr int KS = BMc / 32;
  static_assert(W >= 16 && W <= 128, "composite window wgrad");
  __shared__ __attribute__((aligned(1024))) char smem[XB + YB];
  char* Xs = smem;
  char* Ys = smem + XB;

  const int tid = threadIdx.x, lane = tid & 63, sh = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.QH;
  const int rows_total = p.N * H;
  const int Mq = rows_total * W;
  const int nwin = rows_total / R;                 // H % R == 0: windows never span images
  const int O = p.M1, K = p.Nc;
  const int kt = K / (32 * QN);
  const int ntile = (O / 32) * kt;
  const int bid = (p.xcd & 1) ? xcd_remap(blockIdx.x, gridDim.x) : (int)blockIdx.x;
  const int lsplit = bid / ntile, tile = bid - lsplit * ntile;
  const int split = p.split_lo + lsplit;
  const int o_blk = tile / kt, k_blk = tile - o_blk * kt;
  const int o0 = o_blk * 32, k0 = k_blk * 32 * QN;
  constexpr int OOB = 0x7fffffff;
  const int w_begin = (int)((long long)split * nwin / p.splits);
  const int w_end = (int)((long long)(split + 1) * nwin / p.splits);
  const bool do_bias = p.bias_mode == 2 && k_blk == 0;

  f32x4 acc[4][2][2 * QN];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2 * QN; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) bacc[t][0] = bacc[t][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ (((lslot >> 3) & 1) << 1);
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto tr_addr = [&](int slot, int ch) -> int {   // swizzle keyed on slot mod 16
    return slot * 64 + ((((ch >> 3) ^ (((slot >> 3) & 1) << 1))) << 4) + ((ch & 7) << 1);
  };
  auto tr8 = [&](const char* base0, const char* base1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };
  // slot of coarse column w for tap column sw within a staged fine row
  auto col_slot = [&](const int sw, const int w) -> int {
    return sw == 0 ? W + 1 + w : sw == 1 ? w : sw == 2 ? W + 2 + w : w + 1;
  };

  for (int win = w_begin; win < w_end; ++win) {
    const int g0 = win * R;
    const int fimg0 = 2 * (g0 - g0 % H);             // first fine row of the window's image
    // image-relative bases (scalar): 32-bit DMA offsets, tensors beyond 2 GiB
    const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.b + (size_t)g0 * W * K * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.a1 + (size_t)fimg0 * (2 * W) * O * 2), (short)0, OOB, 0x00020000);
    __syncthreads();
#pragma unroll
    for (int qq = 0; qq < (XI + 3) / 4; ++qq) {
      const int k = sh + 4 * qq;
      if (k < XI) {
        const int o = k / (BMc / 16), sb = (k - o * (BMc / 16)) * 16;   // x image o (channel block)
        const int pix = g0 * W + sb + lslot;
        const int off = pix < Mq ? ((sb + lslot) * K + k0 + 32 * o + lchunk * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (__attribute__((address_space(3))) void*)(Xs + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
      const int k = sh + 4 * qq;
      if (k < YI) {
        const int sl = 16 * k + lslot;
        const int fr = sl / FP, ps = sl - fr * FP;
        const int gf = 2 * g0 - 1 + fr;                 // fine row
        const bool odd = ps > W;
        const int cc = odd ? ps - (W + 2) : ps;          // column index in its parity class
        const bool ok = fr < FR && gf >= fimg0 && gf < fimg0 + 2 * H && (unsigned)cc < (unsigned)W;
        const int col = odd ? 2 * cc + 1 : 2 * cc;
        const int off = ok ? (((gf - fimg0) * (2 * W) + col) * O + o0 + lchunk * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsy, (__attribute__((address_space(3))) void*)(Ys + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int kk = 0; kk < KS; ++kk) {
      const int px0 = kk * 32;
      // this lane group's 8 coarse pixels px0 + 8 G .. + 7 lie in one coarse row (W % 8 == 0;
      // at W = 16 a 32-pixel step spans two rows)
      const int pg = px0 + 8 * G;
      const int rr = pg / W, cg = pg - rr * W;
      h16x8 bf[2 * QN];
#pragma unroll
      for (int qn = 0; qn < QN; ++qn)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const char* Xq = Xs + qn * (BMc * 64);
          const int s0 = px0 + 8 * G + q;
          bf[2 * qn + j] = tr8(Xq + tr_addr(s0, 16 * j + 4 * pp), Xq + tr_addr(s0 + 4, 16 * j + 4 * pp));
        }
      const int rowb = (2 * rr + sh) * FP;              // staged row of fine row 2(g0 + rr) + sh - 1
#pragma unroll
      for (int sw = 0; sw < 4; ++sw) {
        const int s0 = rowb + col_slot(sw, cg + q);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const h16x8 af = tr8(Ys + tr_addr(s0, 16 * i + 4 * pp), Ys + tr_addr(s0 + 4, 16 * i + 4 * pp));
#pragma unroll
          for (int j = 0; j < 2 * QN; ++j) acc[sw][i][j] = mfma16(af, bf[j], acc[sw][i][j]);
          if (do_bias) bacc[sw][i] = mfma16(af, ones, bacc[sw][i]);
        }
      }
    }
  }

  // acc[sw][i][j][r] = slab[tap][o0 + 16i + 4(lane >> 4) + r][k0 + 16j + (lane & 15)]
#pragma unroll
  for (int sw = 0; sw < 4; ++sw) {
    const int tap = sh * 4 + sw;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = o0 + 16 * i + 4 * (lane >> 4);
#pragma unroll
      for (int j = 0; j < 2 * QN; ++j) {
        float* o = p.slab + (((size_t)split * 16 + tap) * O + m) * K + k0 + 16 * j + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(size_t)r * K] = acc[sw][i][j][r];
      }
      if (do_bias && (lane & 15) == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) p.bias_slab[((size_t)split * 16 + tap) * O + m + r] = bacc[sw][i][r];
      }
    }
  }
}

template <int W, int QO, int GEO>
hipError_t launch_wgrad_win_g(const WgradParams& p, hipStream_t s) {
  const int grid = ((p.M1 + p.M2) / 32) * (p.Nc / (32 * QO)) * p.KD * launch_splits(p);
  if constexpr ((GEO == WGEO_2D || GEO == WGEO_3D) && QO == 1) {
    if (p.hg.prob) {
      UNET_LAUNCH((wgrad_win_kernel<W, QO, false, GEO, true>), dim3(grid), dim3(NTHR), 0, s, p);
      return launch_status();
    }
  }
  if (p.hg.prob) return hipErrorInvalidValue;
  if constexpr (W == 128 && QO == 1 && (GEO == WGEO_2D || GEO == WGEO_3D)) {
    if (p.pf && p.xform != 2 && !p.pair) {              // prefetching window (option wg_pf; xform 1: A on load)
      if (p.xform == 1) {
        if constexpr (GEO == WGEO_2D) {
          UNET_LAUNCH((wgrad_pf128_kernel<false, GEO, true>), dim3(grid), dim3(NTHR), 0, s, p);
          return launch_status();
        }
        return hipErrorInvalidValue;
      }
      if (p.M2 > 0)
        UNET_LAUNCH((wgrad_pf128_kernel<true, GEO>), dim3(grid), dim3(NTHR), 0, s, p);
      else
        UNET_LAUNCH((wgrad_pf128_kernel<false, GEO>), dim3(grid), dim3(NTHR), 0, s, p);
      return launch_status();
    }
  }
  if (p.xform == 2) {                                   // dz on load (wgrad_check: 2D single source)
    if constexpr (GEO == WGEO_2D && W >= 16 && W <= 64 && QO == 1) {
      if (p.M2 > 0) return hipErrorInvalidValue;
      UNET_LAUNCH((wgrad_win_kernel<W, QO, false, GEO, false, false, true>), dim3(grid), dim3(NTHR), 0, s, p);
      return launch_status();
    }
    return hipErrorInvalidValue;
  }
  if constexpr (QO == 1 && W >= 32 && W <= 64) {      // (128-wide rows: 61 VGPRs spilled, 2x slower)
    if (p.pair) {
      if (p.M2 > 0)
        UNET_LAUNCH((wgrad_win_kernel<W, QO, true, GEO, false, true>), dim3(grid), dim3(NTHR), 0, s, p);
      else
        UNET_LAUNCH((wgrad_win_kernel<W, QO, false, GEO, false, true>), dim3(grid), dim3(NTHR), 0, s, p);
      return launch_status();
    }
  }
  if (p.M2 > 0)
    UNET_LAUNCH((wgrad_win_kernel<W, QO, true, GEO>), dim3(grid), dim3(NTHR), 0, s, p);
  else
    UNET_LAUNCH((wgrad_win_kernel<W, QO, false, GEO>), dim3(grid), dim3(NTHR), 0, s, p);
  return launch_status();
}

template <int W, int QO>
hipError_t launch_wgrad_win(const WgradParams& p, hipStream_t s) {
  if (p.KD == 3) {
    if constexpr (W >= 32) return launch_wgrad_win_g<W, QO, WGEO_3D>(p, s);
    return hipErrorInvalidValue;          // (not eligible: 3D needs the column-unit rows)
  }
  if (p.QW > W) {
    if constexpr (W == 128) return launch_wgrad_win_g<W, QO, WGEO_SEG>(p, s);
    return hipErrorInvalidValue;
  }
  return launch_wgrad_win_g<W, QO, WGEO_2D>(p, s);
}

}  // namespace

// Row-window wgrad applies to 2D 3x3 stride-1 'same' convs on full rows 8..128 wide
// (p.win < 0 disables it for A/B tests).
// Rows wider than 128 (a multiple of 128) are cut into 128-wide segments; 3D 3x3x3 runs
// one tap group per depth tap on rows >= 32 wide (column-unit path: windows never span
// two (n, d) slices, so the depth padding is a per-window skip).
static bool wgrad_win_eligible(const WgradParams& p) {
  const bool w_ok = p.QW == 8 || p.QW == 16 || p.QW == 32 || p.QW == 64 ||
                    (p.QW % 128 == 0 && p.QW > 0 && p.QW <= 8192);
  const int W = p.QW > 128 ? 128 : (p.QW > 0 ? p.QW : 1);
  // the column-unit (W >= 32) and row-pair (W = 16) paths need windows (256 / W rows)
  // that never span two images
  const bool rows_ok = W < 16 || p.QH % (256 / W) == 0;
  const bool dims_ok = (p.QD == 1 && p.KD == 1) || (p.KD == 3 && p.QD == p.AD && p.QD > 1 && W >= 32);
  return p.win >= 0 && w_ok && rows_ok && dims_ok && p.KH == 3 && p.KW == 3 && p.stride == 1 &&
         p.pad == 1 && p.upA == 1 && p.AW == p.QW && p.AH == p.QH && (p.M1 % 32) == 0 && (p.M2 % 32) == 0 &&
         p.M1 > 0 && (p.Nc % 32) == 0 && p.bias_mode != 2;
}

// First layer (CIN 4/8, padded channels) on full rows 16..128 wide.
static bool wgrad_win_first3_eligible(const WgradParams& p) {
  const bool w_ok = p.QW == 16 || p.QW == 32 || p.QW == 64 || p.QW == 128;
  return p.win >= 0 && w_ok && p.KD == 3 && p.QD > 1 && p.AD == p.QD && p.KH == 3 && p.KW == 3 && p.stride == 1 &&
         p.pad == 1 && p.upA == 1 && p.AW == p.QW && p.AH == p.QH && p.QH % (256 / p.QW) == 0 && p.M1 == 4 &&
         p.M2 == 0 && (p.Nc % 32) == 0 && p.bias_mode != 2 && p.xform == 0;
}

static bool wgrad_win_first_eligible(const WgradParams& p) {
  if (wgrad_win_first3_eligible(p)) return true;
  const bool w_ok = p.QW == 16 || p.QW == 32 || p.QW == 64 || p.QW == 128 || p.QW == 256 || p.QW == 512;
  return p.win >= 0 && w_ok && p.QD == 1 && p.KD == 1 && p.KH == 3 && p.KW == 3 && p.stride == 1 && p.pad == 1 &&
         p.upA == 1 && p.AW == p.QW && p.AH == p.QH && (p.M1 == 4 || p.M1 == 8) && p.M2 == 0 &&
         (p.Nc % 32) == 0 && p.bias_mode != 2;
}

// 2D transposed conv (2x2 stride 2) on coarse rows 32 / 64 wide.
static bool wgrad_tconv_win_eligible(const WgradParams& p) {
  return p.win >= 0 && (p.QW == 32 || p.QW == 64) && p.QD == 1 && p.KD == 1 && p.KH == 2 && p.KW == 2 &&
         p.stride == 2 && p.pad == 0 && p.upA == 1 && p.AW == 2 * p.QW && p.AH == 2 * p.QH && p.M2 == 0 &&
         (p.M1 % 32) == 0 && (p.Nc % 32) == 0 && p.bias_mode != 1;
}

// Composite transposed-conv slab sums (4x4 taps, stride 2, pad 1) on coarse rows 16..128
// wide (128: the 512^2 model's level-3 -> 2 transposed conv; there the generic one-tap tile
// ran at 38 TF/s, 0.89 ms of a 14.5 ms step -- r5 layer times).
static bool wgrad_s2d_win_eligible(const WgradParams& p) {
  const int R = p.QW > 0 ? 128 / p.QW : 1;
  return p.win >= 0 && (p.QW == 16 || p.QW == 32 || p.QW == 64 || p.QW == 128) && p.QD == 1 && p.KD == 1 && p.KH == 4 && p.KW == 4 &&
         p.stride == 2 && p.pad == 1 && p.upA == 1 && p.AW == 2 * p.QW && p.AH == 2 * p.QH && p.QH % R == 0 &&
         p.M2 == 0 && (p.M1 % 32) == 0 && (p.Nc % 32) == 0 && p.bias_mode != 1;
}

WgradCfg wgrad_pick(const WgradParams& p) {
  const int KT = p.KD * p.KH * p.KW;
  const int M = p.M1 + p.M2;
  // row-window tile (dz on load: the 32-channel output block -- with two, the z granules in
  // flight pushed the 64-channel block past 256 VGPRs, 11-17 spilled)
  if (wgrad_win_eligible(p)) return {32, (p.Nc % 64 == 0 && p.xform != 2) ? 64 : 32, 9, 0};
  if (wgrad_win_first3_eligible(p)) return {112, 32, 1, 1};                     // 3D first-layer window
  if (wgrad_win_first_eligible(p)) return {p.M1 == 4 ? 48 : 80, 32, 1, 1};      // first-layer window
  if (wgrad_tconv_win_eligible(p))                                                 // transposed-conv window
    return {32, p.Nc % 128 == 0 ? 128 : (p.Nc % 64 == 0 ? 64 : 32), 4, 0};
  // composite window (128-wide coarse rows: one 32-channel block per workgroup -- the four
  // staged fine rows of 258 slots + a 64-channel coarse block would exceed two workgroups' LDS)
  if (wgrad_s2d_win_eligible(p)) return {32, (p.Nc % 64 == 0 && p.QW <= 64) ? 64 : 32, 16, 0};
  if ((p.M1 == 4 || p.M1 == 8) && p.M2 == 0) return {64, 32, 1, 1};
  // composite transposed-conv slab (tconv_fused.hip): 4x4 taps, stride 2, pad 1, one tap
  // per tile so bias mode 2 yields the per-tap sums
  if (p.KH == 4 && p.KW == 4 && p.KD == 1 && p.stride == 2 && p.pad == 1 && p.M1 % 32 == 0 && p.M2 == 0)
    return {32, p.Nc % 64 == 0 ? 64 : 32, 1, 0};
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
  if (p.xform != 0 && p.xform != 1 && p.xform != 2) return "wgrad: xform must be 0, 1 or 2";
  if (p.xform == 1 && (!p.pf || !wgrad_win_eligible(p) || p.QW != 128 || p.KD != 1 || p.QD != 1 || p.M2 != 0 ||
                       p.M1 != 32 || (p.xcs != 0 && p.xcs != p.M1) || !p.xa || !p.xb || p.hg.prob || p.pair))
    return "wgrad: A normalised on load needs the prefetching 128-wide window (2D, one 32-channel source)";
  if (p.xform == 2 && (!p.xa || !p.xb || !p.xc || !p.xz || (p.xcs != 0 && p.xcs != p.Nc) ||
                       (wgrad_win_first_eligible(p)
                            ? (p.xcs && p.QH % ((p.QW > 256 ? p.QW : 256) / p.QW)) != 0
                            : (!wgrad_win_eligible(p) || p.KD != 1 || p.QD != 1 || p.QW < 16 || p.QW > 64 ||
                               p.M2 != 0 || p.hg.prob || p.pair))))
    return "wgrad: B transform (dz on load) needs the first-layer window wgrad or a 2D single-source row-window "
           "wgrad on rows 16..64 wide";
  if (p.upA != 1) return "wgrad: upA must be 1 (nearest upsampling is materialised)";
  // (the head-on-load instantiations are the 2D full-row and the 3D windows,
  // launch_wgrad_win_g<W, 1, WGEO_2D / WGEO_3D>, on the rows the executor plans them for)
  if (p.hg.prob && (!p.hg.t || !p.hg.sums || !p.hg.w || !p.hg.bits || !wgrad_win_eligible(p) || p.Nc != 32 ||
                    p.M2 != 0 || (p.KD == 1 && p.QD != 1) || p.QW < 16 || p.QW > 128 || p.xform ||
                    (p.KD == 3 && p.QW < 32)))
    return "wgrad: head-on-load B needs a 2D / 3D single-source row-window wgrad with 32 output channels on rows "
           "16..128 wide (3D: 32..128)";
  // 32-bit buffer offsets: the window kernels count them from each window's rows (one
  // image must stay below 2 GiB), the tiled kernel from the tensor starts
  {
    const bool win = wgrad_win_eligible(p) || wgrad_win_first_eligible(p) || wgrad_tconv_win_eligible(p) ||
                     wgrad_s2d_win_eligible(p);
    const long long ia = (long long)p.AD * p.AH * p.AW * (p.M1 > p.M2 ? p.M1 : p.M2) * 2;
    const long long ib = (long long)p.QD * p.QH * p.QW * p.Nc * 2;
    const long long lim = (1LL << 31) - 64;
    if (win ? (ia >= lim || ib >= lim) : (ia * p.N >= lim || ib * p.N >= lim))
      return win ? "wgrad: one image of an operand exceeds 2 GiB" : "wgrad: operand tensor exceeds 2 GiB (split the batch)";
  }
  if (p.splits < 1) return "wgrad: splits must be >= 1";
  if (p.split_lo < 0 || p.split_n < 0 || p.split_lo + launch_splits(p) > p.splits)
    return "wgrad: split range [split_lo, split_lo + split_n) outside [0, splits)";
  return nullptr;
}

hipError_t wgrad_launch(const WgradParams& p0, hipStream_t s) {
  // workgroup -> XCD map of the window weight gradients: the 64 tiles of a split run on
  // one XCD and share its L2 instead of fetching each dY / input window into several
  // (same-box sweep of the headline step 43.4k -> 44.1k img/s; the tiled kernel's map
  // measured neutral and stays off)
  WgradParams p = p0;
  p.xcd = 1;
  const WgradCfg c = wgrad_pick(p);
  if (wgrad_win_first_eligible(p)) return p.M1 == 4 ? launch_wgrad_win_first<4>(p, s) : launch_wgrad_win_first<8>(p, s);
  if (wgrad_tconv_win_eligible(p)) {
    const int qn = p.Nc % 128 == 0 ? 4 : (p.Nc % 64 == 0 ? 2 : 1);
    const int grid = (p.M1 / 32) * (p.Nc / (32 * qn)) * launch_splits(p);
#define TW_CASE(WW, QQ) UNET_LAUNCH((wgrad_tconv_win_kernel<WW, QQ>), dim3(grid), dim3(NTHR), 0, s, p)
    if (p.QW == 32) {
      if (qn == 4) TW_CASE(32, 4); else if (qn == 2) TW_CASE(32, 2); else TW_CASE(32, 1);
    } else {
      if (qn == 4) TW_CASE(64, 4); else if (qn == 2) TW_CASE(64, 2); else TW_CASE(64, 1);
    }
#undef TW_CASE
    return launch_status();
  }
  if (wgrad_s2d_win_eligible(p)) {
    const int qn = (p.Nc % 64 == 0 && p.QW <= 64) ? 2 : 1;
    const int grid = (p.M1 / 32) * (p.Nc / (32 * qn)) * launch_splits(p);
#define SW_CASE(WW, QQ) UNET_LAUNCH((wgrad_s2d_win_kernel<WW, QQ>), dim3(grid), dim3(NTHR), 0, s, p)
    if (p.QW == 16) {
      if (qn == 2) SW_CASE(16, 2); else SW_CASE(16, 1);
    } else if (p.QW == 32) {
      if (qn == 2) SW_CASE(32, 2); else SW_CASE(32, 1);
    } else if (p.QW == 64) {
      if (qn == 2) SW_CASE(64, 2); else SW_CASE(64, 1);
    } else {
      SW_CASE(128, 1);
    }
#undef SW_CASE
    return launch_status();
  }
  if (wgrad_win_eligible(p)) {
    const bool q2 = c.BN == 64;
    switch (p.QW) {
      case 8: return q2 ? launch_wgrad_win<8, 2>(p, s) : launch_wgrad_win<8, 1>(p, s);
      case 16: return q2 ? launch_wgrad_win<16, 2>(p, s) : launch_wgrad_win<16, 1>(p, s);
      case 32: return q2 ? launch_wgrad_win<32, 2>(p, s) : launch_wgrad_win<32, 1>(p, s);
      case 64: return q2 ? launch_wgrad_win<64, 2>(p, s) : launch_wgrad_win<64, 1>(p, s);
      default: return q2 ? launch_wgrad_win<128, 2>(p, s) : launch_wgrad_win<128, 1>(p, s);
    }
  }
  if (c.smallc) return launch_wg<64, 32, 1, 2, 2, true>(p, s);
  if (c.BM == 32 && c.NTAP == 1) return c.BN == 64 ? launch_wg<32, 64, 1, 2, 2>(p, s) : launch_wg<32, 32, 1, 2, 2>(p, s);
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
    UNET_LAUNCH(slab_partial_kernel, g1, dim3(256), 0, s, slab, splits, n4, out, scale);
    return launch_status();
  }
  if (!stage) return hipErrorInvalidValue;
  UNET_LAUNCH(slab_partial_kernel, g1, dim3(256), 0, s, slab, splits, n4, stage, scale);
  const size_t n4o = (size_t)taps * Mout * Nc / 4;
  UNET_LAUNCH(slab_final_kernel, dim3((unsigned)((n4o + 255) / 256)), dim3(256), 0, s, stage, groups, taps,
                     Mtot, Mout, Nc, rg, rkeep, out);
  return launch_status();
}

int reduce_groups(int splits) { return (splits + RED_G - 1) / RED_G; }

hipError_t multi_reduce_launch(const void* jobs, int njobs, long long total1, long long total2, hipStream_t s) {
  if (total1 > 0)
    UNET_LAUNCH(multi_reduce1_kernel, dim3((unsigned)((total1 + 255) / 256)), dim3(256), 0, s,
                       (const ReduceJob*)jobs, njobs, total1);
  if (total2 > 0)
    UNET_LAUNCH(multi_reduce2_kernel, dim3((unsigned)((total2 + 255) / 256)), dim3(256), 0, s,
                       (const ReduceJob*)jobs, njobs, total2);
  return launch_status();
}

hipError_t colsum_launch(const void* x, int rows, int C, int blocks, float* partial, hipStream_t s) {
  const int rpb = (rows + blocks - 1) / blocks;
  UNET_LAUNCH(colsum_kernel, dim3(blocks), dim3(256), 256 * 8 * sizeof(float), s, (const h16*)x, rows, C,
                     rpb, partial);
  return launch_status();
}

}  // namespace unet
