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
// * The skip concat (two sources) is folded into the A address generation: it is
//   never materialised.
//
// Reference semantics: Conv2D 3x3 'same' + ReLU (`model.py:47-117`),
// Conv2DTranspose 2x2/2 (`model.py:79-113`), concatenate (`model.py:76-113`),
// UpSampling2D (`model.py:76-109`), Dropout(0.2) (`model.py:60,66`).
#include "common.h"
#include "conv_params.h"
#include "conv_epilogue.h"
#include "conv_win.h"

namespace unet {

namespace {

constexpr int NTHR = 256;
constexpr int BK = 64;

__device__ __forceinline__ int swz8(int row) { return (row >> 1) & 7; }

// MODE 0: plain; MODE 2: first layer (Cin 4/8).
// CONCAT: a second source supplies channels [C1, C1 + C2) (decoder skip concat).
template <int BM, int BN, int WAVES_M, int WAVES_N, int MODE, bool CONCAT, int EPI = EPI_GENERIC>
__global__ void __launch_bounds__(NTHR) conv_fwd_kernel(const ConvFwdParams p) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int AR = BM / 32;                       // A rows per thread
  constexpr int BR = (BN + 31) / 32;                // B rows per thread
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int EPI_BYTES = (EPI == EPI_STATS || EPI == EPI_DGRAD_NORM) ? epi_lds_bytes<BM, BN>() : BM * (BN + 4) * 2;
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

  // image-relative 32-bit offsets: the tile's rows start in image n_base (a tile spans at
  // most BM / (OD OH OW) + 2 images, conv_fwd_prepare bounds their bytes), so a tensor may
  // exceed 2 GiB
  const int n_base = m0 / (p.OD * p.OH * p.OW);
  const size_t base_px = (size_t)n_base * p.ID * p.IH * p.IW;
  // ---- per-row precomputation (hoisted out of the K loop)
  int a_pix[AR];      // full-res pixel index of the window origin (may be negative at the halo)
  int a_pb1[AR], a_pb2[AR];   // the same as byte offsets into src1 / src2
  uint32_t a_mask[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int r = (tid >> 3) + 32 * i;
    const int q = m0 + r;
    const bool ok = q < M;
    const PixCoord c = decompose(ok ? q : 0, p.OD, p.OH, p.OW);
    const int bd = c.d * p.stride - padd, bh = c.h * p.stride - p.pad, bw = c.w * p.stride - p.pad;
    a_pix[i] = (((c.n - n_base) * p.ID + bd) * p.IH + bh) * p.IW + bw;
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
  }
  u32x4 ra[AR], rb[BR];

  // raw buffer resources: an offset past num_records returns zeros in hardware, so
  // halo taps, K padding and the M tail need no branches (cdna_hip_programming.md T8)
  constexpr int OOB = 0x7fffffff;
  const char* s1b = (const char*)p.src1 + base_px * 2 * p.C1;
  const char* s2b = p.src2 ? (const char*)p.src2 + base_px * 2 * p.C2 : s1b;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)s1b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)s2b, (short)0, OOB, 0x00020000);
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
      const int td1 = (tdel * p.C1 + kk) * 2;
      const int td2 = (tdel * p.C2 + kk - p.C1) * 2;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const bool ok = live && ((a_mask[i] >> tap) & 1u);
        const int o1 = a_pb1[i] + td1;
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
      h16x8 xf[TM], wf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) xf[i] = *(const h16x8*)(As + (wm * WM + i * 16) * 128 + fo);
#pragma unroll
      for (int j = 0; j < TN; ++j) wf[j] = *(const h16x8*)(Bs + (wn * WN + j * 16) * 128 + fo);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(wf[j], xf[i], acc[i][j]);
    }
    if (ks + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  conv_epilogue<BM, BN, WM, WN, TM, TN, NTHR, EPI>(p, acc, smem, m0, n0, M, wm, wn, lane, tid, 0, 0, tm);
}

template <int BM, int BN, int WAVES_M, int WAVES_N>
hipError_t launch_cfg(const ConvFwdParams& p, hipStream_t s) {
  const int M = p.N * p.OD * p.OH * p.OW;
  const int grid = ((M + BM - 1) / BM) * (p.Cout / BN);
  const bool smallc = (p.C1 == 4 || p.C1 == 8) && p.C2 == 0;
  const int epi = conv_epi_mode(p);
  if (epi == EPI_STATS || epi == EPI_DGRAD_NORM) {
    // fused-normalisation epilogues: plain (MODE 0) or first-layer (MODE 2) sources
    if (epi == EPI_DGRAD_NORM && !smallc && p.C2 == 0)
      UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, false, EPI_DGRAD_NORM>), dim3(grid), dim3(NTHR),
                         0, s, p);
    else if (epi == EPI_STATS && smallc)
      UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 2, false, EPI_STATS>), dim3(grid), dim3(NTHR), 0,
                         s, p);
    else if (epi == EPI_STATS && p.C2 > 0)
      UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, true, EPI_STATS>), dim3(grid), dim3(NTHR), 0, s,
                         p);
    else if (epi == EPI_STATS)
      UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, false, EPI_STATS>), dim3(grid), dim3(NTHR), 0,
                         s, p);
    else
      return hipErrorInvalidValue;
    return launch_status();
  }
  if (smallc)
    UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 2, false>), dim3(grid), dim3(NTHR), 0, s, p);
  else if (p.C2 > 0)
    UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, true>), dim3(grid), dim3(NTHR), 0, s, p);
  else
    UNET_LAUNCH((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, 0, false>), dim3(grid), dim3(NTHR), 0, s, p);
  return launch_status();
}


// ---------------------------------------------------------------------------------
// Image-window conv for 8 x 8 images (the deepest UNet level at 128^2 inputs: 2D 3x3
// 'same', Cin / Cout multiples of 32 / 64).  The row-window kernel needs 16-pixel rows;
// the implicit GEMM above re-gathers the input once per tap (9x the L2->LDS traffic)
// through one register stage, which leaves these MFMA-bound layers latency-bound at
// ~35 % MFMA utilisation.  Here a workgroup owns IMG8 = 4 whole images (256 pixels, one
// per wave) x 64 output channels.  Per 32-channel chunk it LDS-DMAs each image with its
// zero ring (10 x 10 slots at a 12-slot row pitch, OOB loads supply the zeros) plus the
// chunk's 9 x 64 weight rows, and runs the nine taps on shifted LDS addresses: an MFMA
// A fragment is 2 rows x 8 columns, lane fr reading slot (2 rp + fr / 8 + dh) x 12 +
// fr % 8 + dw.  Chunk c of a slot sits at c ^ (((column >> 2) & 1) << 1): conflict-free
// for every tap shift (tools/lds_bank_model.py search) and row independent, so a lane
// needs one address per horizontal tap plus immediates.  A fragment of halo row k feeds
// every (row pair rp, tap dh) with 2 rp + dh = k.
constexpr int IMG8 = 4;

template <int EPI>
__global__ void __launch_bounds__(NTHR) conv_img8_kernel(const ConvFwdParams p) {
  constexpr int BM = IMG8 * 64, BN = 64, PITCH = 12, ISL = 10 * PITCH;
  constexpr int XI = IMG8 * ISL / 16, WI = 9 * BN / 16;
  constexpr int XB = XI * 1024, WB = WI * 1024;
  constexpr int EPIB = (EPI == EPI_STATS || EPI == EPI_DGRAD_NORM) ? epi_lds_bytes<BM, BN>() : BM * (BN + 4) * 2;
  constexpr int LDS_BYTES = (XB + WB > EPIB) ? XB + WB : EPIB;
  constexpr int TM = 4, TN = BN / 16;
  static_assert(IMG8 * ISL % 16 == 0, "DMA runs");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ws = smem + XB;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int img0 = tm * IMG8, n0 = tn * BN;
  const int M = p.N * 64;
  const int Cin = p.C1 + p.C2;
  const int nchunks = Cin >> 5;
  constexpr int OOB = 0x7fffffff;
  // workgroup-relative buffer bases (32-bit DMA offsets count from the tile's first image)
  const char* s1b = (const char*)p.src1 + (size_t)img0 * 64 * p.C1 * 2;
  const char* s2b = p.src2 ? (const char*)p.src2 + (size_t)img0 * 64 * p.C2 * 2 : s1b;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)s1b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)s2b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fsub = lane >> 4, fr = lane & 15;
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int col = (fr & 7) + dw;
    xbase[dw] = (wave * ISL + (fr >> 3) * PITCH + col) * 64 + 16 * (fsub ^ (((col >> 2) & 1) << 1));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
  for (int kc = 0; kc < nchunks; ++kc) {
    const bool from1 = p.C2 == 0 || (kc << 5) < p.C1;
    const int C = from1 ? p.C1 : p.C2;
    const int cb = from1 ? (kc << 5) : (kc << 5) - p.C1;
    if (kc) __syncthreads();                      // the previous chunk's fragment reads are done
    const __amdgpu_buffer_rsrc_t rs = from1 ? rs1 : rs2;
#pragma unroll
    for (int q = 0; q < (XI + 3) / 4; ++q) {
      const int k = wave + 4 * q;
      if (k < XI) {
        const int sl = 16 * k + lslot;
        const int im = sl / ISL, rem = sl - im * ISL;
        const int hr = rem / PITCH, hc = rem - hr * PITCH;
        const int h = hr - 1, w = hc - 1;
        const bool ok = (unsigned)h < 8u && (unsigned)w < 8u && img0 + im < p.N;
        const int lch = (lane & 3) ^ (((hc >> 2) & 1) << 1);
        const int off = ok ? (((im * 64 + h * 8 + w) * C) + cb + lch * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(Xs + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    const int wl = (lslot * p.Kpad + (kc << 5) + lchunk * 8) * 2;
#pragma unroll
    for (int q = 0; q < (WI + 3) / 4; ++q) {
      const int k = wave + 4 * q;
      if (k < WI) {
        const int tap = k / (BN / 16), nb = (k % (BN / 16)) * 16;
        const int off = ((n0 + nb) * p.Kpad + tap * Cin) * 2 + wl;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      h16x8 wf[3][TN];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[dh][j] = *(const h16x8*)(Ws + ((3 * dh + dw) * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int hr = 0; hr < 2 * TM + 2; ++hr) {      // halo rows 0 .. 9 of the image
        if (hr == 2 * TM + 1) continue;             // (row 9 only feeds pair 4 -- none)
        const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * PITCH * 64);
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) {
          const int r2 = hr - dh;
          if (r2 < 0 || (r2 & 1) || r2 / 2 >= TM) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[r2 / 2][j] = mfma16(wf[dh][j], xf, acc[r2 / 2][j]);
        }
      }
    }
  }
  __syncthreads();
  conv_epilogue<BM, BN, 64, BN, TM, TN, NTHR, EPI>(p, acc, smem, img0 * 64, n0, M, wave, 0, lane, tid, 0, 0, tm);
}

hipError_t launch_img8(const ConvFwdParams& p, hipStream_t s) {
  const int grid = ((p.N + IMG8 - 1) / IMG8) * (p.Cout / 64);
  switch (conv_epi_mode(p)) {
    case EPI_FWD: UNET_LAUNCH((conv_img8_kernel<EPI_FWD>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case EPI_DGRAD: UNET_LAUNCH((conv_img8_kernel<EPI_DGRAD>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case EPI_GENERIC: UNET_LAUNCH((conv_img8_kernel<EPI_GENERIC>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case EPI_STATS: UNET_LAUNCH((conv_img8_kernel<EPI_STATS>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case EPI_DGRAD_NORM:
      UNET_LAUNCH((conv_img8_kernel<EPI_DGRAD_NORM>), dim3(grid), dim3(NTHR), 0, s, p);
      break;
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

// ---------------------------------------------------------------------------------
// First-layer row-window conv (Cin = 4 or 8 after channel padding, 2D 3x3 'same').
//
// K = 9 taps x CIN is tiny, so the implicit GEMM above spends its time on per-tap
// address generation and 64-wide K padding.  Here the workgroup stages the (R+2)-row
// halo of its 512 output pixels once (8- or 16-byte pixel slots, LDS-DMA), keeps the
// 32 x K weight fragments in registers, and builds each MFMA A fragment straight from
// the halo: lane group G of K-step s covers k = 32 s + 8 G .. + 7, i.e. two taps x 4
// channels (CIN 4: two 8-byte reads) or one tap x 8 channels (CIN 8: one 16-byte read).
// Taps past the ninth and taps whose input row leaves the output row's image read the
// always-zero slot 0.  Halo slot layout per row: [0] zero, [1] column -1 (zero),
// [2 .. W+1] columns 0 .. W-1, [W+2] column W (zero), [W+3] pad.
//
// A workgroup runs FWPW consecutive windows: the next window's halo (6 KB) is loaded into
// registers while the current one's MFMAs and epilogue run, and written to LDS after the
// epilogue -- the load latency a one-window workgroup exposes before its few MFMAs is
// hidden, and the epilogue's stores stream back to back.  (Register staging, not LDS-DMA:
// the compiler then counts the loads past the epilogue's stores itself.)
constexpr int FWPW = 8;
// D3: 3D (3x3x3 'same'): rows of the flattened (n, d, h) space; each depth tap kd stages the
// window's halo from the depth slice d + kd - 1 (zeros past the volume) and runs the 2D tap
// set with that depth tap's weights, accumulating into the same tile.  The next (window,
// depth tap)'s halo is in registers under the current one's MFMAs.
// (3D holds three depth taps' weight fragments: two waves per SIMD, no spills)
template <int W, int CIN, int EPI, bool D3 = false>
__global__ void __launch_bounds__(NTHR) __attribute__((amdgpu_waves_per_eu(D3 ? 2 : 3)))
conv_win_first_kernel(const ConvFwdParams p) {
  // Row pitch in slots.  CIN 4 (8-byte slots): a half-wave's two 16-lane groups read 128
  // consecutive bytes each, at taps whose slots differ by Delta; they share no bank iff
  // 8 Delta == 128 (mod 256).  With the pitch == 16 (mod 32) slots and the K order below
  // pairing vertically adjacent taps (Delta = RS) in every half-wave, the halo reads are
  // conflict-free (round 4: W + 4 = 132 slots and taps t, t + 2 paired -- 34.6 % of the
  // kernel's LDS cycles were bank conflicts, r4_pmc_table.md).
  constexpr int BM = 512, R = BM / W, HR = R + 2;
  constexpr int RS = CIN == 4 ? ((W + 4 + 15) / 32) * 32 + 16 : W + 4;
  constexpr int SB = 2 * CIN;                                  // slot bytes
  constexpr int ROWB = RS * SB;
  constexpr int CPR = ROWB / 16;                               // 16-byte chunks per halo row
  constexpr int NCH = HR * CPR;                                // halo chunks
  // + a zeroed tail of 16 chunks: a zero tap reads its partner's slot ^ 16, which for the
  // last halo row's columns W - 1, W lies up to 2 slots past the image (RS = W + 16 at
  // W >= 128) -- never-written LDS there could hold a NaN pattern (0 x NaN).  (Found at
  // W = 512: relative error 0.65.)
  constexpr int NCHZ = NCH + 16;
  constexpr int CPT = (NCHZ + NTHR - 1) / NTHR;                // chunks per thread
  constexpr int XB = (NCHZ * 16 + 1023) / 1024 * 1024;
  constexpr int BN = 32, TM = 8, TN = 2;
  constexpr int KS = (9 * CIN + 31) / 32;                      // MFMA K-steps
  constexpr int EPIB = (EPI == EPI_STATS) ? epi_lds_bytes<BM, BN>() : BM * (BN + 4) * 2;
  constexpr int TPR = W / 16;
  static_assert((CIN == 4 || CIN == 8) && W >= 16 && W <= 512 && BM % W == 0, "first-layer window");
  __shared__ __attribute__((aligned(1024))) char smem[XB + EPIB];
  char* Xs = smem;
  char* Es = smem + XB;                                        // epilogue staging

  constexpr int NKD = D3 ? 3 : 1;                              // depth taps
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH, D = D3 ? p.OD : 1;
  const int rows_total = p.N * D * H;
  const int M = rows_total * W;
  const int tiles_n = p.Cout / BN;
  const int nwin = ((rows_total + R - 1) / R) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int w_lo = bid * FWPW, w_hi = w_lo + FWPW < nwin ? w_lo + FWPW : nwin;
  constexpr int OOB = 0x7fffffff;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)p.src1, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);

  // halo chunk u = row u / CPR, 16 bytes = slots covering columns (CIN 4) 2c - 2, 2c - 1
  // or (CIN 8) c - 2, c = u % CPR; out-of-range chunks load zeros
  u32x4 hv[CPT];
  // a window never spans two depth slices (host check: H % R == 0)
  auto slice_ok = [&](const int w, const int kd) -> bool {
    if constexpr (!D3) return true;
    const int dd = ((w / tiles_n) * R / H) % D + kd - 1;
    return (unsigned)dd < (unsigned)D;
  };
  auto load_halo = [&](const int w, const int kd) {
    const int g0 = (w / tiles_n) * R;
    const bool sok = slice_ok(w, kd);
    const int shift = D3 ? (kd - 1) * H : 0;                  // rows of the depth-shifted slice
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int u = tid + NTHR * c;
      const int hr = u / CPR, cc = u - hr * CPR;
      const int gr = g0 - 1 + hr;
      const int col = CIN == 4 ? 2 * cc - 2 : cc - 2;
      // (the SHIFTED row is range-checked: a halo row of the window's last slice row plus the
      // depth shift lies in the next volume -- past the tensor for the last one, where the
      // 2 GiB buffer range would not stop the load; run P faulted on exactly that)
      const bool ok = sok && u < NCH && (unsigned)gr < (unsigned)rows_total &&
                      (unsigned)(gr + shift) < (unsigned)rows_total && (unsigned)col < (unsigned)W;
      hv[c] = __builtin_amdgcn_raw_buffer_load_b128(rs1, ok ? (((gr + shift) * W + col) * CIN) * 2 : OOB, 0, 0);
    }
  };
  auto store_halo = [&]() {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int u = tid + NTHR * c;
      if (u < NCHZ) *(u32x4*)(Xs + u * 16) = hv[c];
    }
  };
  // weight fragments (A operand: k = 32 s + 8 (lane >> 4) .. + 7, m = lane & 15), from global.
  // CIN 4: k slot i = 8 s + 2 (lane >> 4) + hh holds tap KPERM[i] (4 bits each; 9..15 are
  // zero taps): the half-wave pairs (KPERM[i], KPERM[i + 2]) are the vertical neighbours
  // (0, 3), (1, 4), (2, 5), then 6, 7, 8 with zero taps -- see RS above.  A zero tap (zero
  // weights) reads its partner's slots + 16 (the other half of the banks) instead of the
  // broadcast zero slot, which would share banks with the partner's 128 bytes.
  constexpr unsigned long long KPERM = 0xFEDCBA87'95624310ull;
  auto ktap = [](const int i) -> int { return CIN == 4 ? (int)((KPERM >> (4 * i)) & 15ull) : i; };
  const int fsub = lane >> 4, fr = lane & 15;
  h16x8 wf[NKD][KS][TN];
  auto load_w = [&](const int n0) {
#pragma unroll
    for (int kd = 0; kd < NKD; ++kd)
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (CIN == 4) {
          u32x4 v;
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int t = ktap(8 * s + 2 * fsub + hh);
            const u32x2 h2 = __builtin_bit_cast(
                u32x2, __builtin_amdgcn_raw_buffer_load_b64(
                           rsw, t < 9 ? ((n0 + 16 * j + fr) * p.Kpad + 4 * (9 * kd + t)) * 2 : OOB, 0, 0));
            v[2 * hh] = h2[0];
            v[2 * hh + 1] = h2[1];
          }
          wf[kd][s][j] = __builtin_bit_cast(h16x8, v);
        } else {
          // (taps 9..11 of the last K step read the next depth tap's weights: their halo
          // operand is the zero slot)
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(
              rsw, ((n0 + 16 * j + fr) * p.Kpad + 72 * kd + 32 * s + 8 * fsub) * 2, 0, 0);
          wf[kd][s][j] = __builtin_bit_cast(h16x8, v);
        }
      }
  };
  if (w_lo >= w_hi) return;
  load_halo(w_lo, 0);
  load_w((w_lo % tiles_n) * BN);
  store_halo();
  __syncthreads();
  const int rw0 = (128 * wave) / W;
  for (int w = w_lo; w < w_hi; ++w) {
    const int tm = w / tiles_n, tn = w - tm * tiles_n;
    const int g0 = tm * R, m0 = g0 * W, n0 = tn * BN;
    if (w > w_lo && tiles_n > 1) load_w(n0);
    uint32_t top_ok = 0, bot_ok = 0, live = 0;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int g = g0 + rw0 + (i / TPR);
      const int h = g % H;
      if (g < rows_total) live |= 1u << i;
      if (h > 0) top_ok |= 1u << i;
      if (h < H - 1) bot_ok |= 1u << i;
    }
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kd = 0; kd < NKD; ++kd) {
      // the next (window, depth tap)'s halo lands under this one's MFMAs
      if (kd + 1 < NKD) load_halo(w, kd + 1);
      else if (w + 1 < w_hi) load_halo(w + 1, 0);
      if (slice_ok(w, kd)) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if (!((live >> i) & 1u)) continue;
          const int rr = rw0 + i / TPR;                       // window row of this 16-pixel tile
          const int cw = ((128 * wave) % W) + (i % TPR) * 16 + fr;   // this lane's output column
          const bool tok = (top_ok >> i) & 1u, bok = (bot_ok >> i) & 1u;
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            u32x4 v;
            if constexpr (CIN == 4) {
#pragma unroll
              for (int hh = 0; hh < 2; ++hh) {
                int t = ktap(8 * s + 2 * fsub + hh);            // tap of this 4-channel half
                const bool zt = t >= 9;                         // zero tap: the partner's tap, other banks
                if (zt) t = ktap(8 * s + 2 * (fsub ^ 1) + hh);
                const int dh = t / 3, dw = t - 3 * dh;
                const bool ok = t < 9 && (dh != 0 || tok) && (dh != 2 || bok);
                const int slot = ((rr + dh) * RS + cw + dw + 1) ^ (zt ? 16 : 0);
                const u32x2 h2 = *(const u32x2*)(Xs + (ok ? slot * SB : 0));
                v[2 * hh] = h2[0];
                v[2 * hh + 1] = h2[1];
              }
            } else {
              const int t = 4 * s + fsub;
              const int dh = t / 3, dw = t - 3 * dh;
              const bool ok = t < 9 && (dh != 0 || tok) && (dh != 2 || bok);
              const int slot = (rr + dh) * RS + cw + dw + 1;
              v = *(const u32x4*)(Xs + (ok ? slot * SB : 0));
            }
            const h16x8 xf = __builtin_bit_cast(h16x8, v);
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(wf[kd][s][j], xf, acc[i][j]);
          }
        }
      }
      if (kd + 1 < NKD) {                                  // next depth tap's halo
        __syncthreads();
        store_halo();
        __syncthreads();
      }
    }
    __syncthreads();                                     // halo reads done; previous epilogue's staging reads done
    conv_epilogue<BM, BN, 128, BN, TM, TN, NTHR, EPI>(p, acc, Es, m0, n0, M, wave, 0, lane, tid, 0, 0, tm);
    if (w + 1 < w_hi) store_halo();
    __syncthreads();
  }
}

template <int CIN>
hipError_t launch_win_first(const ConvFwdParams& p, hipStream_t s) {
  const int W = p.OW;
  const int R = 512 / W;
  const bool d3 = p.KD == 3;
  const int grid = (((p.N * p.OD * p.OH + R - 1) / R) * (p.Cout / 32) + FWPW - 1) / FWPW;
  const int epi = conv_epi_mode(p);
  const bool fwd = epi == EPI_FWD;
#define WF_GEO(WW, G3)                                                                                        \
    if (fwd)                                                                                                  \
      UNET_LAUNCH((conv_win_first_kernel<WW, CIN, EPI_FWD, G3>), dim3(grid), dim3(NTHR), 0, s, p);    \
    else if (epi == EPI_STATS)                                                                                \
      UNET_LAUNCH((conv_win_first_kernel<WW, CIN, EPI_STATS, G3>), dim3(grid), dim3(NTHR), 0, s, p);  \
    else                                                                                                      \
      UNET_LAUNCH((conv_win_first_kernel<WW, CIN, EPI_GENERIC, G3>), dim3(grid), dim3(NTHR), 0, s, p);
#define WF_CASE(WW)                                                                                        \
  case WW:                                                                                                 \
    if (d3) {                                                                                              \
      if constexpr (WW <= 128) { WF_GEO(WW, true) } else { return hipErrorInvalidValue; }                  \
    } else {                                                                                               \
      WF_GEO(WW, false)                                                                                    \
    }                                                                                                      \
    break;
  switch (W) {
    WF_CASE(16)
    WF_CASE(32)
    WF_CASE(64)
    WF_CASE(128)
    WF_CASE(256)
    WF_CASE(512)
    default:
      return hipErrorInvalidValue;
  }
#undef WF_CASE
#undef WF_GEO
  return launch_status();
}


// ---------------------------------------------------------------------------------
// 2x2 stride-2 transposed convolution (2D), forward and data gradient, on windows of
// whole coarse rows.  Coarse grid H x W (the transposed conv's input), fine grid 2H x 2W.
//
// Forward  out[2h+th][2w+tw][co] = b[co] + sum_ci x[h][w][ci] W[(th,tw)][co][ci]:
//   a workgroup owns 128 coarse pixels (R = 128 / W coarse rows) and 32 output
//   channels; wave t computes tap t for all 128 pixels (shared x image, per-tap weight
//   rows), and the epilogue assembles the 2R x 2W fine tile in LDS so the stores are
//   whole contiguous fine rows (the pixel shuffle costs nothing).
// Data gradient dx[h][w][ci] = sum_{t,co} dy[2h+th][2w+tw][co] W[(th,tw)][co][ci]:
//   256 coarse pixels x 32 input channels per workgroup; per 32-channel chunk of dy the
//   2R fine rows are LDS-DMA'd once with even / odd columns de-interleaved, so the
//   four taps' A fragments are 16 consecutive slots (conflict free) of the same image.
// SEG (coarse rows wider than 128, the 512^2 model's transConv9: 256-wide): a window is a
// 128-pixel segment of one coarse row, its fine tile two 256-pixel segments of fine rows.
// D3 (2x2x2 stride-2, the 3D model): eight taps -- wave w computes taps w (td = 0) and
// w + 4 (td = 1) from the same x image; a window's R coarse rows lie in one depth slice
// (OH % R == 0), so per td its 2R fine rows are one contiguous run of fine slice 2 sd + td.
template <int W, int EPI, bool SEG = false, bool D3 = false>
__global__ void __launch_bounds__(NTHR) tconv_fwd_kernel(const ConvFwdParams p) {
  constexpr int BMc = 128, R = BMc / W;
  static_assert(!SEG || W == 128, "segmented coarse rows: 128-pixel windows");
  static_assert(!(SEG && D3), "3D: rows <= 128 wide");
  constexpr int NTD = D3 ? 2 : 1;                  // depth taps
  constexpr int XI = BMc / 16, WI = 4 * NTD * 32 / 16;   // 1 KB DMA instructions per chunk
  constexpr int XB = XI * 1024, WB = WI * 1024;
  constexpr int EPIB = 4 * BMc * 64;                // fine staging: 64-byte pixel rows
  constexpr int LDS_BYTES = (XB + WB > EPIB) ? XB + WB : EPIB;
  constexpr int TM = BMc / 16, TN = 2;
  static_assert(BMc % W == 0 && W >= 8 && W <= 128, "tconv window");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ws = smem + XB;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int rows_total = p.N * (D3 ? p.OD : 1) * H;    // coarse rows (n, d, h)
  const int Wc = SEG ? p.OW : W;                 // coarse row width
  const int nseg = SEG ? p.OW / W : 1;
  const int Mc = rows_total * Wc;
  const int cof = p.Cout >> (D3 ? 3 : 2);        // fine output channels
  const int tiles_n = cof / 32;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int g0 = (tm / nseg) * R, seg = tm - (tm / nseg) * nseg;
  const int m0 = g0 * Wc + seg * W, n0 = tn * 32;
  const int Cin = p.C1;
  constexpr int OOB = 0x7fffffff;
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc((void*)p.src1, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
  const int fsub = lane >> 4, fr = lane & 15;
  const int fbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));

  f32x4 acc[NTD][TM][TN];
#pragma unroll
  for (int td = 0; td < NTD; ++td)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[td][i][0] = acc[td][i][1] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < (Cin >> 5); ++kc) {
    if (kc) __syncthreads();
#pragma unroll
    for (int qq = 0; qq < (XI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < XI) {
        const int pix = m0 + 16 * k + lslot;
        const int off = pix < Mc ? (pix * Cin + (kc << 5) + lchunk * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (__attribute__((address_space(3))) void*)(Xs + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
#pragma unroll
    for (int qq = 0; qq < (WI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < WI) {
        const int t = k >> 1, nb = (k & 1) * 16;        // weight image row = t * 32 + co
        const int row = t * cof + n0 + nb + lslot;
        const int off = (row * p.Kpad + (kc << 5) + lchunk * 8) * 2;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    __syncthreads();
    h16x8 wf[NTD][TN];
#pragma unroll
    for (int td = 0; td < NTD; ++td)
#pragma unroll
      for (int j = 0; j < TN; ++j) wf[td][j] = *(const h16x8*)(Ws + ((wave + 4 * td) * 32 + 16 * j) * 64 + fbase);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const h16x8 xf = *(const h16x8*)(Xs + (16 * i) * 64 + fbase);
#pragma unroll
      for (int td = 0; td < NTD; ++td)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[td][i][j] = mfma16(wf[td][j], xf, acc[td][i][j]);
    }
  }
  // register phase: acc[td][i][j][r] = out(coarse px 16i + (lane&15), tap = (td, wave))[co = 16j + 4(lane>>4) + r]
  // Staging: fine pixel fp in 64-byte row fp ^ ((fp >> 1) & 1), 16-byte chunk c at
  // c ^ ((fp >> 2) & 3), its 8-byte halves swapped when ((fp >> 4) ^ (fp >> 5)) & 1.  A
  // register-phase store group (16 lanes, fine pixels 2 apart: fp bits 1-4 = the lane, bit 0
  // the tap column, fixed) then maps its lanes one-to-one onto the 16 8-byte slots of the 32
  // banks (row parity x chunk x half), and the coalesced phase's 16-byte reads of 4
  // consecutive pixels fill 4 distinct 64-byte bank segments: both conflict-free
  // (tools/lds_bank_model.py check_tconv_epi).  The 72-byte padded rows this replaces needed
  // two 8-byte reads per chunk, 2-way conflicted (30.8 % conflict cycles, r5 PMC pass).
  char* E = smem;
  auto tc_off = [](const int fp, const int c) { return (fp ^ ((fp >> 1) & 1)) * 64 + 16 * (c ^ ((fp >> 2) & 3)); };
  auto tc_half = [](const int fp) { return ((fp >> 4) ^ (fp >> 5)) & 1; };
  const int th = wave >> 1, tw = wave & 1;
  const size_t fine_total = (size_t)(2 * rows_total) * (2 * Wc) * (D3 ? 2 : 1);
#pragma unroll
  for (int td = 0; td < NTD; ++td) {
    __syncthreads();        // (td 0: the MFMAs' LDS reads; td 1: the previous tile's stores)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int nl = 16 * j + 4 * (lane >> 4);
      float bs[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) bs[r] = p.bias ? p.bias[n0 + nl + r] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pl = 16 * i + (lane & 15);
        const int rr = pl / W, w = pl - rr * W;
        const int fp = (2 * rr + th) * (2 * W) + 2 * w + tw;
        u32x2 pk;
        pk[0] = pack2h(acc[td][i][j][0] + bs[0], acc[td][i][j][1] + bs[1]);
        pk[1] = pack2h(acc[td][i][j][2] + bs[2], acc[td][i][j][3] + bs[3]);
        *(u32x2*)(E + tc_off(fp, nl >> 3) + 8 * (((nl >> 2) & 1) ^ tc_half(fp))) = pk;
      }
    }
    __syncthreads();
    // coalesced phase: the window's 2R fine rows (SEG: two 2W-pixel segments of fine rows
    // 2 Wc wide; D3: rows of fine slice 2 sd + td) are contiguous runs of the output
    const int sd = D3 ? g0 / H : 0, h0 = D3 ? g0 - sd * H : 0;
    const size_t frow0 = D3 ? (size_t)(2 * sd + td) * (2 * H) + 2 * h0 : (size_t)(2 * g0);
#pragma unroll
    for (int it = 0; it < (4 * BMc * 4) / NTHR; ++it) {
      const int c = tid + it * NTHR;
      const int fp = c >> 2, q = c & 3;
      const int frow = fp / (2 * W), fcol = fp - frow * (2 * W);
      const size_t gp = (frow0 + frow) * (2 * Wc) + 2 * seg * W + fcol;
      if (gp >= fine_total) continue;
      u32x4 v = *(const u32x4*)(E + tc_off(fp, q));
      if (tc_half(fp)) v = (u32x4){v[2], v[3], v[0], v[1]};
      *(u32x4*)((h16*)p.dst1 + gp * cof + n0 + q * 8) = v;
    }
  }
}

template <int W, int BN, int EPI>
__global__ void __launch_bounds__(NTHR) tconv_dgrad_kernel(const ConvFwdParams p) {
  constexpr int BMc = 256, R = BMc / W, FW = 2 * W;     // coarse window; fine row width
  constexpr int YI = (2 * R * FW) / 16;                 // dy image DMA instructions per chunk
  constexpr int WI = 4 * BN / 16;
  constexpr int YB = YI * 1024, WB = WI * 1024;
  constexpr int EPIB = (EPI == EPI_DGRAD_NORM) ? epi_lds_bytes<BMc, BN>() : BMc * (BN + 4) * 2;
  constexpr int LDS_BYTES = (YB + WB > EPIB) ? YB + WB : EPIB;
  constexpr int TM = BMc / 4 / 16, TN = BN / 16;
  static_assert(BMc % W == 0 && W >= 8 && W <= 256, "tconv window");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Ys = smem;
  char* Ws = smem + YB;

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;                                    // coarse (output) grid
  const int rows_total = p.N * H;
  const int Mc = rows_total * W;
  const int cof = p.C1;                                  // fine channels (dy)
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = bid / tiles_n, tn = bid - tm * tiles_n;
  const int g0 = tm * R, m0 = g0 * W, n0 = tn * BN;
  constexpr int OOB = 0x7fffffff;
  const __amdgpu_buffer_rsrc_t rsy = __builtin_amdgcn_make_buffer_rsrc((void*)p.src1, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
  const int fsub = lane >> 4, fr = lane & 15;
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  const int fine_rows_total = 2 * rows_total;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < (cof >> 5); ++kc) {
    if (kc) __syncthreads();
    // dy image: fine row fr2 (of 2R), slot s in [0, 2W): s < W -> column 2s, else 2(s - W) + 1
#pragma unroll
    for (int qq = 0; qq < (YI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < YI) {
        const int sl = 16 * k + lslot;
        const int frr = sl / FW, s = sl - frr * FW;
        const int col = s < W ? 2 * s : 2 * (s - W) + 1;
        const int gf = 2 * g0 + frr;
        const int off = gf < fine_rows_total ? ((gf * FW + col) * cof + (kc << 5) + lchunk * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsy, (__attribute__((address_space(3))) void*)(Ys + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    // weight image [t][ci BN][co chunk 32]: row t * BN + ci, from the dgrad pack [ci][t*cof + co]
#pragma unroll
    for (int qq = 0; qq < (WI + 3) / 4; ++qq) {
      const int k = wave + 4 * qq;
      if (k < WI) {
        const int t = k / (BN / 16), cb = (k % (BN / 16)) * 16;
        const int off = ((n0 + cb + lslot) * p.Kpad + t * cof + (kc << 5) + lchunk * 8) * 2;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int th = t >> 1, tw = t & 1;
      h16x8 wf[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) wf[j] = *(const h16x8*)(Ws + (t * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pl = wave * (BMc / 4) + 16 * i + fr;     // this lane's coarse pixel
        const int rr = pl / W, w = pl - rr * W;
        const int slot = (2 * rr + th) * FW + tw * W + w;
        const h16x8 xf = *(const h16x8*)(Ys + slot * 64 + 16 * (fsub ^ ((slot >> 1) & 3)));
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(wf[j], xf, acc[i][j]);
      }
    }
  }
  __syncthreads();
  conv_epilogue<BMc, BN, BMc / 4, BN, TM, TN, NTHR, EPI>(p, acc, smem, m0, n0, Mc, wave, 0, lane, tid, 0, 0, tm);
}

hipError_t launch_tconv_fwd(const ConvFwdParams& p, hipStream_t s) {
  const int W = p.OW;
  if (p.shuffle == 3) {
    const int grid = (p.N * p.OD * p.OH / (128 / W)) * ((p.Cout >> 3) / 32);
    switch (W) {
      case 16: UNET_LAUNCH((tconv_fwd_kernel<16, 0, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 32: UNET_LAUNCH((tconv_fwd_kernel<32, 0, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 64: UNET_LAUNCH((tconv_fwd_kernel<64, 0, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case 128: UNET_LAUNCH((tconv_fwd_kernel<128, 0, false, true>), dim3(grid), dim3(NTHR), 0, s, p); break;
      default: return hipErrorInvalidValue;
    }
    return launch_status();
  }
  if (W > 128) {
    const int grid = p.N * p.OH * (W / 128) * ((p.Cout >> 2) / 32);
    UNET_LAUNCH((tconv_fwd_kernel<128, 0, true>), dim3(grid), dim3(NTHR), 0, s, p);
    return launch_status();
  }
  const int R = 128 / W;
  const int grid = ((p.N * p.OH + R - 1) / R) * ((p.Cout >> 2) / 32);
  switch (W) {
    case 8: UNET_LAUNCH((tconv_fwd_kernel<8, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 16: UNET_LAUNCH((tconv_fwd_kernel<16, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 32: UNET_LAUNCH((tconv_fwd_kernel<32, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 64: UNET_LAUNCH((tconv_fwd_kernel<64, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case 128: UNET_LAUNCH((tconv_fwd_kernel<128, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return launch_status();
}

// data gradient: 64 input channels per workgroup (one dy image feeds 4 MFMA columns)
hipError_t launch_tconv_dgrad(const ConvFwdParams& p, hipStream_t s) {
  const int W = p.OW;
  const int R = 256 / W;
  const int grid = ((p.N * p.OH + R - 1) / R) * (p.Cout / 64);
  const int epi = conv_epi_mode(p);
  const bool dg = epi == EPI_DGRAD;
#define TD_CASE(WW)                                                                                          \
  case WW:                                                                                                   \
    if (dg)                                                                                                  \
      UNET_LAUNCH((tconv_dgrad_kernel<WW, 64, EPI_DGRAD>), dim3(grid), dim3(NTHR), 0, s, p);       \
    else if (epi == EPI_DGRAD_NORM)                                                                          \
      UNET_LAUNCH((tconv_dgrad_kernel<WW, 64, EPI_DGRAD_NORM>), dim3(grid), dim3(NTHR), 0, s, p);  \
    else                                                                                                     \
      UNET_LAUNCH((tconv_dgrad_kernel<WW, 64, EPI_GENERIC>), dim3(grid), dim3(NTHR), 0, s, p);     \
    break;
  switch (W) {
    TD_CASE(8)
    TD_CASE(16)
    TD_CASE(32)
    TD_CASE(64)
    TD_CASE(128)
    TD_CASE(256)
    default:
      return hipErrorInvalidValue;
  }
#undef TD_CASE
  return launch_status();
}

}  // namespace

// True when the row-window kernel can run this conv: 3x3 (2D) or 3x3x3 (3D) stride 1
// 'same', plain / concat source at full resolution, rows 16..128 wide or a multiple of
// 128 (cut into 128-wide segments).
static bool win_eligible(const ConvFwdParams& p) {
  const bool w_ok = p.OW == 16 || p.OW == 32 || p.OW == 64 || (p.OW % 128 == 0 && p.OW > 0 && p.OW <= 8192);
  const int W = p.OW > 128 ? 128 : (p.OW > 0 ? p.OW : 1);
  const int R = (W == 16 ? 256 : 512) / W;     // window rows
  const bool dims_ok = (p.KD == 1 && p.OD == 1 && p.ID == 1) || (p.KD == 3 && p.OD == p.ID && p.OD > 1 && p.OW <= 128);
  return w_ok && p.OH % R == 0 && dims_ok && p.KH == 3 && p.KW == 3 && p.stride == 1 && p.pad == 1 &&
         p.up1 == 1 && !p.shuffle && p.IW == p.OW && p.IH == p.OH &&
         (p.C1 % 32) == 0 && (p.C2 % 32) == 0 && p.C1 > 0;
}

// First layer (4/8 padded input channels) on full rows 16..512 wide (256 / 512: a window is
// two rows / one row; the 512^2 model's first layer ran the tiled implicit GEMM at 15 TF/s,
// 0.33 ms per half-batch launch -- r5 layer times).
static bool win_first_eligible(const ConvFwdParams& p) {
  const bool w_ok = p.OW == 16 || p.OW == 32 || p.OW == 64 || p.OW == 128 || p.OW == 256 || p.OW == 512;
  // 3D (3x3x3 'same', rows <= 128 wide, windows inside one depth slice)
  if (p.KD == 3 && p.OD > 1 && p.ID == p.OD && p.OW <= 128 && w_ok && p.OH % (512 / p.OW) == 0 && p.KH == 3 &&
      p.KW == 3 && p.stride == 1 && p.pad == 1 && p.up1 == 1 && !p.shuffle && !p.nz && p.IW == p.OW &&
      p.IH == p.OH && p.C2 == 0 && (p.C1 == 4 || p.C1 == 8) && p.Cout % 32 == 0 && p.D1 == p.Cout)
    return true;
  return p.KD == 1 && p.OD == 1 && p.ID == 1 && p.KH == 3 && p.KW == 3 && p.stride == 1 && p.pad == 1 &&
         p.up1 == 1 && !p.shuffle && !p.nz && w_ok && p.IW == p.OW && p.IH == p.OH && p.C2 == 0 &&
         (p.C1 == 4 || p.C1 == 8) && p.Cout % 32 == 0 && p.D1 == p.Cout;
}

// 2D transposed-conv forward (1x1 GEMM + 2x2 pixel shuffle) on coarse rows 8..128 wide
// (128: a window is one coarse row).
static bool tconv_fwd_eligible(const ConvFwdParams& p) {
  const bool w_ok = p.OW == 8 || p.OW == 16 || p.OW == 32 || p.OW == 64 || p.OW == 128 ||
                    (p.OW % 128 == 0 && p.OW <= 8192);       // (wider: 128-pixel row segments)
  // 3D (2x2x2): rows 16..128 wide, a window's 128 / W coarse rows inside one depth slice
  if (p.shuffle == 3)
    return p.KD == 1 && p.KH == 1 && p.KW == 1 && p.OD == p.ID && p.OD > 1 && p.OW >= 16 && p.OW <= 128 && w_ok &&
           p.OH % (128 / p.OW) == 0 && p.IW == p.OW && p.IH == p.OH && p.C2 == 0 && (p.C1 % 32) == 0 &&
           ((p.Cout >> 3) % 32) == 0 && !p.relu && p.drop_rate == 0.f && !p.mask1 && !p.stats &&
           p.out_scale == 1.f && (long long)p.N * p.ID * p.IH * p.IW * p.C1 * 2 < (1LL << 31) - 64;
  return p.shuffle == 2 && p.KD == 1 && p.KH == 1 && p.KW == 1 && p.OD == 1 && w_ok && p.IW == p.OW &&
         p.IH == p.OH && p.C2 == 0 && (p.C1 % 32) == 0 && ((p.Cout >> 2) % 32) == 0 && !p.relu &&
         p.drop_rate == 0.f && !p.mask1 && !p.stats && p.out_scale == 1.f &&
         (long long)p.N * p.IH * p.IW * p.C1 * 2 < (1LL << 31) - 64;      // (offsets from the tensor start)
}

// 2D transposed-conv data gradient (2x2 stride-2 conv of the fine gradient); coarse rows
// 32 / 64 wide (narrower levels measured faster on the implicit-GEMM kernel).
static bool tconv_dgrad_eligible(const ConvFwdParams& p) {
  // (coarse rows 128 / 256 wide: the 512^2 model; 80 KB of LDS, still two workgroups per CU)
  const bool w_ok = p.OW == 8 || p.OW == 16 || p.OW == 32 || p.OW == 64 || p.OW == 128 || p.OW == 256;
  return !p.shuffle && p.KD == 1 && p.KH == 2 && p.KW == 2 && p.stride == 2 && p.pad == 0 && p.OD == 1 &&
         p.ID == 1 && w_ok && p.IW == 2 * p.OW && p.IH == 2 * p.OH && p.up1 == 1 && p.C2 == 0 &&
         (p.C1 % 32) == 0 && (p.Cout % 64) == 0 && (!p.stats || p.nz) && p.drop_rate == 0.f &&
         // (32-bit offsets from the tensor start: the 512^2 model at batch 128 has a 2.1 GB fine
         // gradient and takes the implicit GEMM, whose offsets count from each tile's images)
         (long long)p.N * p.IH * p.IW * p.C1 * 2 < (1LL << 31) - 64;
}

int conv_fwd_pick(const ConvFwdParams& p);
static bool win_tile(int t) { return t == 6 || t == 12; }

// 2D 8 x 8 images, 3x3 'same', plain / concat source, no fused pool / head / transform
// (the image-window kernel above); normalisation statistics per 4-image tile.
static bool img8_eligible(const ConvFwdParams& p) {
  const int ep = conv_epi_mode(p);
  return p.OW == 8 && p.OH == 8 && p.IW == 8 && p.IH == 8 && p.KD == 1 && p.OD == 1 && p.ID == 1 && p.KH == 3 &&
         p.KW == 3 && p.stride == 1 && p.pad == 1 && p.up1 == 1 && !p.shuffle && p.C1 > 0 && (p.C1 % 32) == 0 &&
         (p.C2 % 32) == 0 && (p.Cout % 64) == 0 && !(p.nz && (p.C2 || p.ncs)) &&
         (ep == EPI_FWD || ep == EPI_DGRAD || ep == EPI_GENERIC || ep == EPI_STATS || ep == EPI_DGRAD_NORM) &&
         !p.route_gy && !p.pool_dst && !p.head_w && !p.xform && !p.hg.prob && !p.s2d && !p.ut.x;
}

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
  // (nearest upsampling is materialised by elementwise.hip::ups_fwd; no folded source)
  if (p.up1 != 1) return "conv_fwd: up1 must be 1";
  if (p.C2 > 0 && !p.src2) return "conv_fwd: src2 missing";
  if (p.shuffle && (p.Cout % (1 << p.shuffle))) return "conv_fwd: shuffle needs Cout % taps == 0";
  if (p.shuffle && ((p.Cout >> p.shuffle) % 8)) return "conv_fwd: shuffle channels must be multiples of 8";
  if (p.shuffle && p.D1 != p.Cout) return "conv_fwd: shuffle with channel split unsupported";
  if (const char* m = conv_norm_epi_check(p)) return m;
  if (p.relu_bits && (!p.relu || p.shuffle || p.D1 != p.Cout || p.mask1 || p.mask2))
    return "conv_fwd: relu_bits needs an unsplit ReLU forward";
  if ((p.mask_bits & ~3) || ((p.mask_bits & 1) && !p.mask1) || ((p.mask_bits & 2) && !p.mask2))
    return "conv_fwd: mask_bits marks a missing mask";
  if (p.xform == 2 && !p.fw.x) {     // data gradient of a normalised layer, dz formed on load
    const int ep = conv_epi_mode(p), t = conv_fwd_pick(p);
    if (p.C2 || !p.xa || !p.xb || !p.xc || !p.xz || p.KD != 1 || p.OD != 1 || p.OW < 16 || p.OW > 64 ||
        !win_eligible(p) || t != 6 || (win_bn(p) != 64 && p.OW != 64) || (p.xcs != 0 && p.xcs != p.C1) ||
        (p.OW == 64 && p.C1 > 128) ||
        p.head_w || p.hg.prob || p.s2d || p.ut.x || p.route_gy || p.pool_dst || (ep != EPI_DGRAD && ep != EPI_DGRAD_NORM))
      return "conv_fwd: dz on load needs a 2D single-source row-window data gradient (rows 16..64 wide; the 32-channel "
             "tile on 64-wide rows only)";
  } else if (p.xform && !p.fw.x) {   // (the fused weight gradient's xform 2: conv_dw_check)
    const int ep = conv_epi_mode(p), t = conv_fwd_pick(p);
    if (p.xform != 1 || p.C2 || !p.xa || !p.xb || p.KD != 1 || p.OD != 1 || p.OW > 128 || !win_eligible(p) ||
        (t != 6 && t != 12) || (p.xcs != 0 && p.xcs != p.C1) || p.head_w || (ep != EPI_STATS && ep != EPI_GENERIC))
      return "conv_fwd: operand transform needs a 2D single-source row-window forward of a normalised input";
  }
  if (p.hg.prob && !p.fw.x && (!p.hg.t || !p.hg.sums || !p.hg.w || !p.hg.bits || p.C1 != 32 || p.C2 || p.xform ||
                    (p.KD != 1 && p.KD != 3) || p.OW > 128 || !win_eligible(p) || conv_epi_mode(p) != EPI_DGRAD ||
                    p.route_gy || !win_tile(conv_fwd_pick(p))))
    return "conv_fwd: head-on-load needs a 2D / 3D 32-channel row-window data gradient";
  if (p.s2d && (p.s2d % 32 || p.C1 != 4 * p.s2d || p.C2 || p.xform || p.hg.prob || p.route_gy || p.KD != 1 ||
                p.OD != 1 || p.OW > 128 || !win_eligible(p) ||
                (conv_epi_mode(p) != EPI_DGRAD && conv_epi_mode(p) != EPI_DGRAD_NORM) ||
                !win_tile(conv_fwd_pick(p))))
    return "conv_fwd: space-to-depth source needs a 2D single-source row-window data gradient (C1 = 4 s2d)";
  if (p.ut.x) {
    const int ep = conv_epi_mode(p);
    if (!p.ut.w || !p.ut.b || (p.ut.C != 32 && p.ut.C != 64 && p.ut.C != 128) || p.ut.kpad < p.ut.C ||
        (p.OW / 32) * (p.ut.C / 32) > 8 ||
        p.C2 <= 0 || p.xform || p.hg.prob || p.s2d || p.route_gy || p.pool_dst || p.head_w || p.KD != 1 ||
        p.OD != 1 || p.OW > 128 || p.OW < 32 || p.OH % 2 || !win_eligible(p) || !win_tile(conv_fwd_pick(p)) ||
        win_rows(p) % 2 || (ep != EPI_FWD && ep != EPI_STATS && ep != EPI_GENERIC))
      return "conv_fwd: transposed-conv source on load needs a 2D concat row-window forward (rows 32..128 wide, "
             "32 / 64 / 128 coarse channels, (W / 32) (C / 32) <= 8)";
  }
  if (p.route_gy && (!p.pool_code || (conv_epi_mode(p) != EPI_DGRAD && conv_epi_mode(p) != EPI_DGRAD_NORM) ||
                     !win_eligible(p) || (p.OD == 1 ? p.KD != 1 : p.OD % 2 != 0) ||
                     p.OH % 2 || p.OW % 2 || p.D1 != p.Cout || p.pool_dst || p.mask_scale1 != 1.f ||
                     !(win_tile(conv_fwd_pick(p)) || conv_fwd_pick(p) == 14)))
    return "conv_fwd: fused pool backward needs a row-window data gradient (even dims, one destination, codes)";
  if (p.pool_dst) {
    const int W = p.OW > 128 ? 128 : p.OW;
    const int R = win_rows(p);
    if (!p.pool_code || conv_epi_mode(p) != EPI_FWD || !win_eligible(p) || p.KD != 1 || p.OD != 1 || R % 2 ||
        p.OH % 2 || p.OW % 2 || p.Cout % 8 || p.head_w)
      return "conv_fwd: fused max-pool needs a 2D row-window ReLU forward (even rows, codes buffer)";
  }
  if (p.fw.x) {
    if (const char* m = conv_dw_check(p)) return m;
  } else if (p.tile == 14) {
    return "conv_fwd: tile 14 (fused weight gradient) needs the fw fields";
  }
  if (p.tile < 0 || p.tile > 14) return "conv_fwd: bad tile id";
  if (p.tile == 12 && (!win_eligible(p) || p.Cout % 64 || p.head_w))
    return "conv_fwd: 64-wide row-window tile not applicable";
  if (p.tile == 10 && !tconv_fwd_eligible(p)) return "conv_fwd: transposed-conv window tile not applicable";
  if (p.tile == 11 && !tconv_dgrad_eligible(p)) return "conv_fwd: transposed-conv dgrad tile not applicable";
  if (p.tile == 9 && !win_first_eligible(p)) return "conv_fwd: first-layer window tile not applicable";
  if (p.tile == 13 && !img8_eligible(p)) return "conv_fwd: 8x8 image-window tile not applicable";
  {
    const int t = p.tile ? p.tile : 0;
    const int bn = t == 1 ? 128 : (t == 2 || t == 5 || t == 7 || t == 12 || t == 13) ? 64 : 32;
    if (t && p.Cout % bn) return "conv_fwd: forced tile does not divide Cout";
    if (t == 7) return "conv_fwd: tile 7 (row-window 512x64: 268 registers, 92 KB LDS, 1 wave/SIMD) is not built";
    if (t == 6 && !win_eligible(p)) return "conv_fwd: row-window tile not applicable";
  }
  if (p.head_w) {
    if (!p.head_b || !p.head_logit) return "conv_fwd: fused head needs head_b / head_logit";
    if (p.Cout != 32 || p.drop_rate > 0.f || !p.relu || p.D1 != p.Cout || p.mask1 || p.out_scale != 1.f ||
        conv_epi_mode(p) != EPI_FWD || conv_fwd_pick(p) != 6)
      return "conv_fwd: fused head needs a 32-channel ReLU row-window forward";
  }
  if ((p.x2a || p.x2b) && (!p.x2a || !p.x2b || !win_pfu_eligible(p) || (p.x2cs != 0 && p.x2cs != p.C2)))
    return "conv_fwd: the skip source normalised on load needs the persistent tconv-on-load window";
  if ((p.head_ws || p.head_nostore) &&
      (!p.head_w || p.OW != 128 || (p.head_ws && !p.head_t) || !p.relu_bits ||
       !(win_pf_eligible(p) || (p.KD == 3 && p.OD > 1 && p.Cout == 32 && win_tile(conv_fwd_pick(p)) &&
                                win_bn(p) == 32 && win_bm(p) == 512 && win_cp128_eligible(p)))))
    return "conv_fwd: Mask weight sums / an unstored head input need the persistent 128-wide fused-head window "
           "(3D: the 128-wide chunk-pipelined window) with ReLU bits";
  if ((long long)p.N * p.ID * p.IH * p.IW >= (1LL << 31) || (long long)p.N * p.OD * p.OH * p.OW >= (1LL << 31))
    return "conv_fwd: too many pixels";
  // buffer loads use 32-bit byte offsets: the row-window kernels count them from the
  // window's image, the tiled kernels from the first image of the tile (a tile spans at
  // most BM / image + 2 images), the transposed-conv / first-layer windows from the
  // tensor start
  {
    const int t = conv_fwd_pick(p);
    const long long img = (long long)p.ID * p.IH * p.IW * (long long)(p.C1 > p.C2 ? p.C1 : p.C2) * 2;
    const long long opx = (long long)p.OD * p.OH * p.OW;
    const long long lim = (1LL << 31) - 64;
    long long span = img * p.N;                       // bytes a launch addresses from one base
    if (win_tile(t) || t == 13 || t == 14) span = img;
    else if (t >= 1 && t <= 5) span = img * (256 / opx + 2 < p.N ? 256 / opx + 2 : p.N);
    if (span >= lim) return "conv_fwd: input exceeds the 2 GiB reach of one buffer base (split the batch)";
  }
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

// tile ids: 1 = 128x128, 2 = 128x64, 3 = 256x32, 4 = 128x32, 5 = 256x64 (4 waves each);
// 6 = row-window (auto tile width); 8 = auto but never row-window (A/B tests); 12 = row
// window, 64-channel tile; 13 = 8x8 image window
int conv_fwd_pick(const ConvFwdParams& p) {
  const int M = p.N * p.OD * p.OH * p.OW;
  if (p.fw.x) return 14;
  if (p.tile && p.tile != 8) return p.tile;
  // row-window 512x32 wins at every level it applies to (16..128 wide), measured
  // 1.1-2.1x over the implicit-GEMM tiles (profiles/r1_conv_tiles.md); the 512x64
  // variant needs 287 registers (1 wave/SIMD) and never wins
  if (p.tile != 8 && win_eligible(p)) return 6;
  if (p.tile != 8 && win_first_eligible(p)) return 9;
  if (p.tile != 8 && img8_eligible(p)) return 13;
  if (p.tile != 8 && tconv_fwd_eligible(p)) return 10;
  if (p.tile != 8 && tconv_dgrad_eligible(p)) return 11;
  if (p.Cout % 128 == 0 && M >= 8192) return 1;
  if (p.Cout % 64 == 0) return 2;
  return 4;
}

int conv_fwd_grid(const ConvFwdParams& p) {
  const int t = conv_fwd_pick(p);
  if (t == 14) return conv_dw_grid(p);
  return win_tile(t) ? win_grid(p) : 0;
}

void conv_stat_tiles(const ConvFwdParams& p, int* rows, int* tile_px) {
  *rows = *tile_px = 0;
  const int M = p.N * p.OD * p.OH * p.OW;
  const int t = conv_fwd_pick(p);
  const bool smallc = (p.C1 == 4 || p.C1 == 8) && p.C2 == 0;
  switch (t) {
    case 6:
    case 12: {       // row window: R rows x (segment) width, tiles in (row group, segment) order
      const int W = p.OW > 128 ? 128 : p.OW;
      const int R = win_pfu_eligible(p) ? 2 : win_rows(p);   // (the persistent tconv-on-load window: 2 rows)
      if (p.nz && p.C2) return;
      *rows = ((p.N * p.OD * p.OH + R - 1) / R) * (p.OW / W);
      *tile_px = R * W;
      return;
    }
    case 9: {
      const int R = 512 / p.OW;
      if (p.nz) return;
      *rows = (p.N * p.OD * p.OH + R - 1) / R;
      *tile_px = 512;
      return;
    }
    case 11: {
      const int R = 256 / p.OW;
      if (!p.nz) return;
      *rows = (p.N * p.OH + R - 1) / R;
      *tile_px = 256;
      return;
    }
    case 14:                 // fused data + weight gradient: one row per 256-pixel window
      if (!p.nz) return;
      *rows = conv_dw_stat_rows(p);
      *tile_px = 256;
      return;
    case 10:
      return;
    case 13:               // 8x8 image window: 4 whole images per tile
      *rows = (p.N + IMG8 - 1) / IMG8;
      *tile_px = IMG8 * 64;
      return;
    default: {
      if (p.nz && (smallc || p.C2)) return;
      const int BM = (t == 3 || t == 5) ? 256 : 128;
      *rows = (M + BM - 1) / BM;
      *tile_px = BM;
      return;
    }
  }
}

hipError_t conv_fwd_launch(const ConvFwdParams& p, hipStream_t s) {
  switch (conv_fwd_pick(p)) {
    case 1: return launch_cfg<128, 128, 2, 2>(p, s);
    case 2: return launch_cfg<128, 64, 2, 2>(p, s);
    case 3: return launch_cfg<256, 32, 4, 1>(p, s);
    case 5: return launch_cfg<256, 64, 4, 1>(p, s);
    case 6:
    case 12:
      if (win_bn(p) == 64) return launch_win<64, 256>(p, s);
      return win_bm(p) == 256 ? launch_win<32, 256>(p, s) : launch_win<32, 512>(p, s);
    case 9: return p.C1 == 4 ? launch_win_first<4>(p, s) : launch_win_first<8>(p, s);
    case 10: return launch_tconv_fwd(p, s);
    case 13: return launch_img8(p, s);
    case 11: return launch_tconv_dgrad(p, s);
    case 14: return launch_conv_dw(p, s);
    default: return launch_cfg<128, 32, 4, 1>(p, s);
  }
}

}  // namespace unet
