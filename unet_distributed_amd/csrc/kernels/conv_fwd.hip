// Implicit-GEMM convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16), NHWC/NDHWC bf16.
//
// out[q][n] = epilogue( sum_{k} A[q][k] * W[n][k] ),  k = tap * Cin + c  (linear K, padded to 64)
//
// * GEMM M = output pixels (B*D*H*W), N = Cout, K = taps x Cin; one K-step = 64 k
//   (one tap x 64 channels, two taps x 32 channels, or every tap of a 4/8-channel
//   first layer).
// * Address generation is hoisted out of the K loop: each thread owns BM/32 fixed
//   A rows and one 16-byte chunk column; per row it precomputes the signed pixel
//   index of the window origin and a bitmask of in-bounds taps (the 'same'
//   padding halo).  Per K-step the tap's pixel delta is a wave-uniform value from a
//   host-built table, so an A chunk costs a few VALU (v1 spent ~13 VALU per MFMA on
//   64-bit address math and divisions).
// * A (pixels) and B (weights) tiles are staged global->VGPR->LDS with one register
//   stage in flight while the MFMAs consume the other LDS buffer (T14); 128-byte
//   LDS rows with chunk' = chunk ^ ((row >> 1) & 7), found by exhaustive search in
//   tools/lds_bank_model.py to make ds_read_b128 fragment reads bank-conflict free.
// * The MFMA is issued as W x X^T so each lane's accumulator registers run along
//   Cout (4 consecutive channels of one pixel) -> packed 8-byte LDS staging and a
//   fully coalesced 16 B/lane epilogue store.
// * Fused epilogue: scale, bias, ReLU, inverted dropout (counter hash), per-channel
//   BN statistics, consumer-side ReLU mask (out *= mask > 0), channel split into
//   two destinations (dgrad of a concat input), transposed-conv pixel shuffle.
// * Skip concat (two sources) and nearest-upsample (src1 at half resolution) are
//   folded into the A address generation: neither is ever materialised.
//
// Reference semantics: Conv2D 3x3 'same' + ReLU (`model.py:47-117`),
// Conv2DTranspose 2x2/2 (`model.py:79-113`), concatenate (`model.py:76-113`),
// UpSampling2D (`model.py:76-109`), Dropout(0.2) (`model.py:60,66`).
#include "common.h"
#include "conv_params.h"

namespace unet {

namespace {

constexpr int NTHR = 256;
constexpr int BK = 64;

__device__ __forceinline__ int swz8(int row) { return (row >> 1) & 7; }

struct PixCoord {
  int n, d, h, w;
};

__device__ __forceinline__ PixCoord decompose(int q, int OD, int OH, int OW) {
  PixCoord c;
  c.w = q % OW;
  int t = q / OW;
  c.h = t % OH;
  t /= OH;
  c.d = t % OD;
  c.n = t / OD;
  return c;
}

// MODE 0: plain; MODE 1: src1 nearest-upsampled x2; MODE 2: first layer (Cin 4/8).
// CONCAT: a second source supplies channels [C1, C1 + C2) (decoder skip concat).
template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE, bool CONCAT>
__global__ void __launch_bounds__(NTHR) conv_fwd_kernel(const ConvFwdParams p) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AR = BM / 32;                       // A rows per thread
  constexpr int BR = (BN + 31) / 32;                // B rows per thread
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int EPI_STRIDE = (BN + 4) * 2;          // bytes; 8B-aligned, conflict-free b64 writes
  constexpr int EPI_BYTES = BM * EPI_STRIDE;
  constexpr int LDS_BYTES = (2 * STAGE > EPI_BYTES) ? 2 * STAGE : EPI_BYTES;
  static_assert(WAVES_M * WAVES_N == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int M = p.N * p.OD * p.OH * p.OW;
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int Cin = p.C1 + p.C2;
  const int KT = p.KD * p.KH * p.KW;
  const int Kpad = p.Kpad;
  const int nk = Kpad / BK;
  const int cc = tid & 7;                            // this thread's 16-byte chunk column
  const int padd = p.KD > 1 ? p.pad : 0;
  const int upd = p.ID > 1 ? p.up1 : 1;
  const int ID1 = p.ID / upd, IH1 = p.IH / p.up1, IW1 = p.IW / p.up1;

  // ---- per-row precomputation (hoisted out of the K loop)
  int a_pix[AR];      // full-res pixel index of the window origin (may be negative at the halo)
  int a_pb1[AR], a_pb2[AR];   // the same as byte offsets into src1 / src2
  int a_lo[AR];       // MODE 1: low-res pixel index of the centre; parity bits in a_par
  int a_par[AR];
  uint32_t a_mask[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int q = m0 + r;
    const bool ok = q < M;
    const PixCoord c = decompose(ok ? q : 0, p.OD, p.OH, p.OW);
    const int bd = c.d * p.stride - padd, bh = c.h * p.stride - p.pad, bw = c.w * p.stride - p.pad;
    a_pix[i] = ((c.n * p.ID + bd) * p.IH + bh) * p.IW + bw;
    a_pb1[i] = a_pix[i] * p.C1 * 2;
    a_pb2[i] = a_pix[i] * p.C2 * 2;
    // in-bounds tap mask, taps ordered t = (kd*KH + kh)*KW + kw; kernel extents <= 3
    uint32_t m = 0;
#pragma unroll
    for (int kd = 0; kd < 3; ++kd)
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const bool in = kd < p.KD && kh < p.KH && kw < p.KW && (unsigned)(bd + kd) < (unsigned)p.ID &&
                          (unsigned)(bh + kh) < (unsigned)p.IH && (unsigned)(bw + kw) < (unsigned)p.IW;
          if (in) m |= 1u << ((kd * p.KH + kh) * p.KW + kw);
        }
    a_mask[i] = ok ? m : 0u;
    if (MODE == 1) {
      a_lo[i] = ((c.n * ID1 + c.d / upd) * IH1 + c.h / 2) * IW1 + c.w / 2;
      a_par[i] = ((c.d & 1) << 2) | ((c.h & 1) << 1) | (c.w & 1);
    }
  }
  u32x4 ra[AR], rb[BR];

  // raw buffer resources: an offset past num_records returns zeros in hardware, so
  // halo taps, K padding and the M tail need no branches (cdna_hip_programming.md T8)
  constexpr int OOB = 0x7fffffff;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)p.src1, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 =
      __builtin_amdgcn_make_buffer_rsrc((void*)(p.src2 ? p.src2 : p.src1), (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
  int wofs[BR];
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int r = (tid >> 3) + 32 * i;
    wofs[i] = r < BN ? ((n0 + r) * Kpad + cc * 8) * 2 : OOB;
  }

  int kt_tap = 0, kt_kk = 0;           // (tap, channel) at the start of the K step being loaded
  const bool c32 = Cin == 32;
  const int kk_c = c32 ? (cc & 3) * 8 : cc * 8;
  const int hi_c = (c32 && cc >= 4) ? 1 : 0;
  auto load_stage = [&](int ks) {
    const int k0 = ks * BK;
    if constexpr (MODE == 2) {
      // first layer: chunk cc covers k = k0 + 8cc .. +7 = (8 / Cin) taps x Cin channels
      const int t0 = (k0 + cc * 8) / Cin;   // lane-varying; first layers have 1-2 K steps
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (Cin == 8) {
          const bool ok = t0 < KT && ((a_mask[i] >> t0) & 1u);
          v = __builtin_amdgcn_raw_buffer_load_b128(rs1, ok ? (a_pix[i] + p.tap_delta[t0]) * 16 : OOB, 0, 0);
        } else {
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int t = t0 + e;
            const bool ok = t < KT && ((a_mask[i] >> t) & 1u);
            const u32x2 h = __builtin_amdgcn_raw_buffer_load_b64(rs1, ok ? (a_pix[i] + p.tap_delta[t]) * 8 : OOB, 0, 0);
            v[2 * e] = h[0];
            v[2 * e + 1] = h[1];
          }
        }
        ra[i] = v;
      }
    } else {
      // K step = 64 consecutive k of the (tap, channel) index.  Cin == 32: the upper
      // four chunk columns belong to the next tap (hi_c); Cin % 64 == 0: one tap per
      // step.  hi_c / kk_c / the concat source are per-thread loop invariants, the
      // tap (kt_tap) and channel base (kt_kk) are wave-uniform.
      const int tap = kt_tap + hi_c;
      const int kk = kt_kk + kk_c;
      const bool live = tap < KT;
      const int t_a = kt_tap < KT ? kt_tap : 0, t_b = kt_tap + 1 < KT ? kt_tap + 1 : 0;
      // readfirstlane keeps both table reads scalar (s_load); a lane-indexed select
      // would become a vector load from kernarg memory whose vmcnt(0) wait drains
      // the whole prefetch pipeline every K step.
      const int tdel_a = __builtin_amdgcn_readfirstlane(p.tap_delta[t_a]);
      const int tdel_b = __builtin_amdgcn_readfirstlane(p.tap_delta[t_b]);
      const int tdel = hi_c ? tdel_b : tdel_a;
      const bool from1 = !CONCAT || kk < p.C1;
      int dh = 0, dw = 0, dd = 0;
      if (MODE == 1) {
        const int ha = __builtin_amdgcn_readfirstlane(p.tap_h[t_a]), hb = __builtin_amdgcn_readfirstlane(p.tap_h[t_b]);
        const int wa = __builtin_amdgcn_readfirstlane(p.tap_w[t_a]), wb = __builtin_amdgcn_readfirstlane(p.tap_w[t_b]);
        const int da = __builtin_amdgcn_readfirstlane(p.tap_d[t_a]), db = __builtin_amdgcn_readfirstlane(p.tap_d[t_b]);
        dh = hi_c ? hb : ha;
        dw = hi_c ? wb : wa;
        dd = hi_c ? db : da;
      }
      const int td1 = (tdel * p.C1 + kk) * 2;
      const int td2 = (tdel * p.C2 + kk - p.C1) * 2;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const bool ok = live && ((a_mask[i] >> tap) & 1u);
        int o1;
        if (MODE == 1) {
          const int par = a_par[i];
          const int lh = (dh + ((par >> 1) & 1) - 1) >> 1;
          const int lw = (dw + (par & 1) - 1) >> 1;
          const int ld = p.ID > 1 ? ((dd + ((par >> 2) & 1) - 1) >> 1) : 0;
          o1 = ((a_lo[i] + (ld * IH1 + lh) * IW1 + lw) * p.C1 + kk) * 2;
        } else {
          o1 = a_pb1[i] + td1;
        }
        if constexpr (CONCAT) {
          const int o = from1 ? o1 : a_pb2[i] + td2;
          ra[i] = __builtin_amdgcn_raw_buffer_load_b128(from1 ? rs1 : rs2, ok ? o : OOB, 0, 0);
        } else {
          ra[i] = __builtin_amdgcn_raw_buffer_load_b128(rs1, ok ? o1 : OOB, 0, 0);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) rb[i] = __builtin_amdgcn_raw_buffer_load_b128(rsw, wofs[i] + k0 * 2, 0, 0);
  };
  auto store_stage = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *(u32x4*)(As + r * 128 + 16 * (cc ^ swz8(r))) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int r = (tid >> 3) + 32 * i;
      if (r < BN) *(u32x4*)(Bs + r * 128 + 16 * (cc ^ swz8(r))) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // per-lane fragment byte offsets inside a 16-row slab for the two k32 halves
  const int fr = lane & 15;
  const int frag0 = fr * 128 + 16 * (((lane >> 4) + 0) ^ swz8(fr));
  const int frag1 = fr * 128 + 16 * (((lane >> 4) + 4) ^ swz8(fr));

  auto advance = [&]() {   // Cin == 32 or a multiple of 64 (checked on the host)
    if (c32) {
      kt_tap += 2;
    } else {
      kt_kk += BK;
      if (kt_kk >= Cin) {
        kt_kk -= Cin;
        ++kt_tap;
      }
    }
  };
  load_stage(0);
  advance();
  store_stage(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) {
      load_stage(ks + 1);
      advance();
    }
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int fo = h ? frag1 : frag0;
      bf16x8 xf[TM], wf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) xf[i] = *(const bf16x8*)(As + (wm * WM + i * 16) * 128 + fo);
#pragma unroll
      for (int j = 0; j < TN; ++j) wf[j] = *(const bf16x8*)(Bs + (wn * WN + j * 16) * 128 + fo);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(wf[j], xf[i], acc[i][j]);
    }
    if (ks + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  // register phase: acc[i][j][r] = out[pixel = m0 + wm*WM + i*16 + (lane&15)]
  //                                   [chan  = n0 + wn*WN + j*16 + (lane>>4)*4 + r]
  char* E = smem;
  const float inv_keep = p.drop_rate > 0.f ? 1.f / (1.f - p.drop_rate) : 1.f;
  const uint32_t drop_thr = (uint32_t)(p.drop_rate * 4294967296.0);
  const int Dtb = p.shuffle ? (p.Cout >> p.shuffle) : p.Cout;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WN + j * 16 + (lane >> 4) * 4;
    const int n = n0 + nl;
    float bsv[4], msc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bsv[r] = p.bias ? p.bias[(n + r) % Dtb] : 0.f;
      msc[r] = (n + r < p.D1) ? p.mask_scale1 : p.mask_scale2;
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wm * WM + i * 16 + (lane & 15);
      const int q = m0 + ml;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = acc[i][j][r] * p.out_scale + bsv[r];
        if (p.relu) x = fmaxf(x, 0.f);
        if (p.drop_rate > 0.f) {
          const uint32_t h = drop_hash((uint64_t)q * p.Cout + n + r, p.seed, p.salt);
          x = (h >= drop_thr) ? x * inv_keep : 0.f;
        }
        x *= msc[r];
        v[r] = x;
      }
      if (p.stats && q < M) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float xr = (float)(bf16)v[r];
          s1[r] += xr;
          s2[r] += xr * xr;
        }
      }
      u32x2 pk;
      pk[0] = pack2bf(v[0], v[1]);
      pk[1] = pack2bf(v[2], v[3]);
      *(u32x2*)(E + ml * EPI_STRIDE + nl * 2) = pk;
    }
    if (p.stats) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = s1[r], b = s2[r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          b += __shfl_xor(b, o, 64);
        }
        if ((lane & 15) == 0) {
          atomicAdd(p.stats + n + r, a);
          atomicAdd(p.stats + p.Cout + n + r, b);
        }
      }
    }
  }
  __syncthreads();

  // coalesced phase: 16-byte chunks, consecutive threads -> consecutive channels
  constexpr int CPR = BN / 8;
  constexpr int NCHUNK = BM * CPR;
  const int Dt = p.shuffle ? (p.Cout >> p.shuffle) : 0;
#pragma unroll 2
  for (int c = tid; c < NCHUNK; c += NTHR) {
    const int ml = c / CPR, cb = c % CPR;
    const int q = m0 + ml;
    if (q >= M) continue;
    const int n = n0 + cb * 8;
    const u32x2 lo = *(const u32x2*)(E + ml * EPI_STRIDE + cb * 16);
    const u32x2 hi = *(const u32x2*)(E + ml * EPI_STRIDE + cb * 16 + 8);
    u32x4 v = {lo[0], lo[1], hi[0], hi[1]};
    size_t off;
    bf16* dst;
    const void* mk;
    if (p.shuffle) {
      const int tap = n / Dt, co = n - tap * Dt;
      const PixCoord pc = decompose(q, p.OD, p.OH, p.OW);
      int td = 0, th, tw;
      if (p.shuffle == 3) {
        td = tap >> 2;
        th = (tap >> 1) & 1;
        tw = tap & 1;
      } else {
        th = tap >> 1;
        tw = tap & 1;
      }
      const int dd = p.shuffle == 3 ? 2 : 1;
      const size_t pix = (((size_t)pc.n * (p.OD * dd) + pc.d * dd + td) * (2 * p.OH) + 2 * pc.h + th) *
                             (2 * p.OW) + 2 * pc.w + tw;
      off = pix * Dt + co;
      dst = (bf16*)p.dst1;
      mk = p.mask1;
    } else if (n < p.D1) {
      off = (size_t)q * p.D1 + n;
      dst = (bf16*)p.dst1;
      mk = p.mask1;
    } else {
      off = (size_t)q * (p.Cout - p.D1) + (n - p.D1);
      dst = (bf16*)p.dst2;
      mk = p.mask2;
    }
    if (mk) {
      const u32x4 mv = *(const u32x4*)((const bf16*)mk + off);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // bf16 > 0 <=> sign bit clear and not zero (-0 counts as not positive)
        const uint32_t w = mv[e];
        const uint32_t lo16 = w & 0xffffu, hi16 = w >> 16;
        const uint32_t keep_lo = (lo16 != 0u && !(lo16 & 0x8000u)) ? 0xffffu : 0u;
        const uint32_t keep_hi = (hi16 != 0u && !(hi16 & 0x8000u)) ? 0xffff0000u : 0u;
        v[e] &= (keep_lo | keep_hi);
      }
    }
    *(u32x4*)(dst + off) = v;
  }
}

template <int BM, int BN, int WAVES_M, int WAVES_N>
hipError_t launch_cfg(const ConvFwdParams& p, hipStream_t s) {
  const int M = p.N * p.OD * p.OH * p.OW;
  const int grid = ((M + BM - 1) / BM) * (p.Cout / BN);
  const bool smallc = (p.C1 == 4 || p.C1 == 8) && p.C2 == 0;
  if (smallc)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 2, false>), dim3(grid), dim3(NTHR), 0, s, p);
  else if (p.up1 == 2)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 1, true>), dim3(grid), dim3(NTHR), 0, s, p);
  else if (p.C2 > 0)
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, true>), dim3(grid), dim3(NTHR), 0, s, p);
  else
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, false>), dim3(grid), dim3(NTHR), 0, s, p);
  return hipGetLastError();
}

}  // namespace

// Fills the tap tables and Kpad; returns nullptr on success or a message describing
// why the shape is unsupported.
const char* conv_fwd_prepare(ConvFwdParams& p) {
  const int KT = p.KD * p.KH * p.KW;
  if (KT < 1 || KT > 27 || p.KD > 3 || p.KH > 3 || p.KW > 3) return "conv_fwd: kernel extents 1..3 supported";
  const bool smallc = (p.C1 == 4 || p.C1 == 8) && p.C2 == 0;
  if (smallc) {
    if (p.up1 != 1 || p.shuffle) return "conv_fwd: small-Cin mode supports plain convs only";
  } else if (p.C1 <= 0 || (p.C1 % 32) || (p.C2 % 32)) {
    return "conv_fwd: input channels must be multiples of 32 (or 4/8 for the first layer)";
  }
  const int Cin = p.C1 + p.C2;
  if (!smallc && Cin != 32 && Cin % 64) return "conv_fwd: Cin must be 32 or a multiple of 64";
  // the concat source must be constant per (thread, K step): split on a 64-channel
  // boundary, or the 32 + 32 case where each thread's chunk column fixes the source
  if (p.C2 > 0 && p.C1 % 64 && !(p.C1 == 32 && Cin == 64)) return "conv_fwd: concat split unsupported";
  if (p.Cout % 32) return "conv_fwd: Cout must be a multiple of 32";
  if (p.D1 <= 0 || p.D1 > p.Cout || (p.D1 % 8)) return "conv_fwd: bad channel split D1";
  if (p.D1 < p.Cout && !p.dst2) return "conv_fwd: dst2 missing for channel split";
  if (p.up1 != 1 && p.up1 != 2) return "conv_fwd: up1 must be 1 or 2";
  if (p.up1 == 2 && (p.stride != 1 || p.pad != 1 || p.KH != 3)) return "conv_fwd: upsample fold needs 3x3/s1/p1";
  if (p.up1 == 2 && ((p.ID % 2 && p.ID != 1) || p.IH % 2 || p.IW % 2)) return "conv_fwd: upsample needs even dims";
  if (p.C2 > 0 && !p.src2) return "conv_fwd: src2 missing";
  if (p.shuffle && (p.Cout % (1 << p.shuffle))) return "conv_fwd: shuffle needs Cout % taps == 0";
  if (p.shuffle && ((p.Cout >> p.shuffle) % 8)) return "conv_fwd: shuffle channels must be multiples of 8";
  if (p.shuffle && p.D1 != p.Cout) return "conv_fwd: shuffle with channel split unsupported";
  if (p.stats && p.shuffle) return "conv_fwd: stats with shuffle unsupported";
  if (p.tile < 0 || p.tile > 5) return "conv_fwd: bad tile id";
  {
    const int t = p.tile ? p.tile : 0;
    const int bn = t == 1 ? 128 : (t == 2 || t == 5) ? 64 : 32;
    if (t && p.Cout % bn) return "conv_fwd: forced tile does not divide Cout";
  }
  if ((long long)p.N * p.ID * p.IH * p.IW >= (1LL << 31) || (long long)p.N * p.OD * p.OH * p.OW >= (1LL << 31))
    return "conv_fwd: too many pixels";
  // buffer loads use 32-bit byte offsets: every source tensor must stay below 2 GiB
  if ((long long)p.N * p.ID * p.IH * p.IW * (long long)(p.C1 > p.C2 ? p.C1 : p.C2) * 2 >= (1LL << 31) - 64)
    return "conv_fwd: input tensor exceeds 2 GiB (split the batch)";
  p.Kpad = ((KT * Cin + 63) / 64) * 64;
  for (int t = 0; t < 27; ++t) {
    p.tap_d[t] = p.tap_h[t] = p.tap_w[t] = 0;
    p.tap_delta[t] = 0;
  }
  for (int t = 0; t < KT; ++t) {
    const int kw = t % p.KW, kh = (t / p.KW) % p.KH, kd = t / (p.KW * p.KH);
    p.tap_d[t] = (signed char)kd;
    p.tap_h[t] = (signed char)kh;
    p.tap_w[t] = (signed char)kw;
    p.tap_delta[t] = (kd * p.IH + kh) * p.IW + kw;
  }
  return nullptr;
}

// tile ids: 1 = 128x128, 2 = 128x64, 3 = 256x32, 4 = 128x32, 5 = 256x64 (4 waves each)
int conv_fwd_pick(const ConvFwdParams& p) {
  const int M = p.N * p.OD * p.OH * p.OW;
  if (p.tile) return p.tile;
  if (p.Cout % 128 == 0 && M >= 8192) return 1;
  if (p.Cout % 64 == 0) return 2;
  return 4;
}

hipError_t conv_fwd_launch(const ConvFwdParams& p, hipStream_t s) {
  switch (conv_fwd_pick(p)) {
    case 1: return launch_cfg<128, 128, 2, 2>(p, s);
    case 2: return launch_cfg<128, 64, 2, 2>(p, s);
    case 3: return launch_cfg<256, 32, 4, 1>(p, s);
    case 5: return launch_cfg<256, 64, 4, 1>(p, s);
    default: return launch_cfg<128, 32, 4, 1>(p, s);
  }
}

}  // namespace unet
