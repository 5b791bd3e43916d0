// Pipelined row-window 3x3 conv for the mid UNet levels (2D rows 16..64 wide, 64-channel
// output tiles): the K loop's 32-channel chunks are double-buffered in LDS so chunk k+1's
// halo image and weight rows stream in by LDS-DMA while chunk k's MFMAs run.
//
// Why (profiles/r3_stall_breakdown.md): the 4-wave window kernel (conv_win.h) stages one
// chunk, drains it (vmcnt(0) + barrier) and only then issues its MFMAs, so its two
// workgroups per CU alternate DMA-wait and MFMA phases -- 26-50 % MFMA busy on 16..64-wide
// rows where a window has 2-16 chunks.  Here ONE 8-wave workgroup per CU (2 waves per
// SIMD, as before) owns twice the pixels of the 4-wave window for the same 64 channels:
//   * the chunk loop is a ping-pong over two LDS stages: wait for chunk k (this wave's
//     own DMA pieces: vmcnt(0)), one barrier (every wave's pieces landed and every wave is
//     done reading stage k+1's previous chunk), issue chunk k+1 into the other stage,
//     then chunk k's MFMAs -- the DMA latency hides behind a whole chunk of MFMAs;
//   * the weight rows of a chunk (9 taps x 64 channels x 32 inputs = 36 KB, the larger
//     half of a stage) now feed 512 pixels instead of 256: half the weight DMA per MFMA.
// The per-wave work (64 pixels x 64 channels, or x 32 on 16-wide rows) and the MFMA order
// per output element are those of conv_win_kernel, so the results are bit-identical to it
// (tests/test_gpu_kernels.py::test_conv_pipe_matches_window_kernel).
//
// LDS per stage: the (R + 2) x (W + 4) halo image (64-byte pixel slots, 16-byte chunk c of
// column hc at c ^ ((hc >> 1) & 3), as conv_win.h) + the 9 x 64 weight rows.
//   W = 64: R = 8,  512 px: 44.0 + 36.0 KB, two stages 158 KB
//   W = 32: R = 16, 512 px: 41.0 + 36.0 KB, two stages 154 KB
//   W = 16: R = 16, 256 px (a window never spans two images): 23.0 + 36.0 KB, 118 KB; the
//           8 waves split the 64 channels in two halves of 32 (4 pixel strips x 2)
// XF 4: space-to-depth source (conv_params.h s2d, the composite transposed-conv data
// gradient): the DMA gathers the fine pixels of each coarse slot, zero taps skipped.
// XF 1: operand transform (conv_params.h xform 1, normalised input read as the pre-norm
// z): each landed chunk is normalised in LDS, y = relu(xa z + xb), before its MFMAs
// (a second barrier per chunk), and the window's own rows of y go to xout.
#pragma once
#include "common.h"
#include "conv_params.h"
#include "conv_epilogue.h"

namespace unet {

hipError_t launch_pipe(const ConvFwdParams& p, hipStream_t s);

#ifdef UNET_PIPE_IMPL
namespace {

constexpr int PIPE_NTHR = 512;

template <int W>
struct PipeGeo {
  static constexpr int BN = 64;
  static constexpr int BM = W == 16 ? 256 : 512;
  static constexpr int R = BM / W;                    // output rows per window
  static constexpr int HR = R + 2;                    // halo rows
  static constexpr int HWP = W + 4;                   // halo row pitch (slots)
  static constexpr int ROWB = HWP * 64;
  static constexpr int XI = (HR * HWP + 15) / 16;     // halo DMA pieces (1 KB)
  static constexpr int WI = 9 * BN / 16;              // weight DMA pieces
  static constexpr int XB = XI * 1024, WB = WI * 1024;
  static constexpr int STAGE = XB + WB;
  static constexpr int WNS = W == 16 ? 2 : 1;         // channel groups of waves
  static constexpr int NCS = W / 16;                  // 16-pixel column strips per row
  static constexpr int WPG = 8 / WNS;                 // waves per channel group
  static constexpr int RW = R / (WPG / NCS);          // rows per wave strip
  static constexpr int TM = RW, TN = BN / 16 / WNS;
  static constexpr int WMP = RW * 16;                 // pixels per wave
  static_assert(RW == 4 && WPG % NCS == 0, "pipelined window strip map");
  static_assert(STAGE >= epi_lds_bytes<BM, BN, PIPE_NTHR>(), "epilogue staging fits one stage");
  static_assert(2 * STAGE <= 160 * 1024, "two stages fit the 160 KB LDS");
};

template <int W, bool CONCAT, int EPI, int XF>
__global__ void __launch_bounds__(PIPE_NTHR) conv_pipe_kernel(const ConvFwdParams p) {
  using G = PipeGeo<W>;
  constexpr int BN = G::BN, BM = G::BM, R = G::R, HR = G::HR, HWP = G::HWP, ROWB = G::ROWB;
  constexpr int XI = G::XI, WI = G::WI, XB = G::XB, TM = G::TM, TN = G::TN, NCS = G::NCS, RW = G::RW;
  static_assert(XF == 0 || ((XF == 1 || XF == 4) && !CONCAT),
                "pipelined window: plain / concat / normalised / space-to-depth source");
  // two stages as two LDS objects: their accesses carry distinct alias scopes, so the
  // fragment reads of one stage never wait for the DMA in flight into the other
  __shared__ __attribute__((aligned(1024))) char lds0[G::STAGE];
  __shared__ __attribute__((aligned(1024))) char lds1[G::STAGE];
  // XF 1: the normalisation coefficients {xa, xb} of the window's sample (<= 256 channels),
  // staged once before any DMA -- a global load consumed while an LDS-DMA is in flight
  // would make the compiler drain it (vmcnt(0)) and serialise the pipeline
  __shared__ float xco[XF == 1 ? 2 * 256 : 1];
  static_assert(2 * G::STAGE + (XF == 1 ? 2048 : 0) <= 160 * 1024, "stages + coefficients fit the 160 KB LDS");

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int rows_total = p.N * H;
  const int M = rows_total * W;
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm0 = bid / tiles_n, tn = bid % tiles_n;
  const int tm = p.rev ? (int)(gridDim.x / tiles_n) - 1 - tm0 : tm0;
  const int g0 = tm * R;                              // first output row (n, h) of the window
  const int n0 = tn * BN;
  const int Cin = p.C1 + p.C2;
  const int nchunks = Cin >> 5;
  constexpr int OOB = 0x7fffffff;
  // image-relative buffer bases (H % R == 0: a window's rows never leave its image)
  const int grow0 = (g0 / H) * H;
  const size_t img_px = (size_t)grow0 * W;
  const char* s1b = (const char*)p.src1 + img_px * (XF == 4 ? 4 * p.s2d : p.C1) * 2;
  const char* s2b = p.src2 ? (const char*)p.src2 + img_px * p.C2 * 2 : s1b;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)s1b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)s2b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
  const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;

  // wave -> (channel group wn, pixel strip wm): strip = RW rows x 16 columns
  const int wm = wave % G::WPG, wn = wave / G::WPG;
  const int r0 = (wm / NCS) * RW, c0 = (wm % NCS) * 16;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fsub = lane >> 4, fr = lane & 15;
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = r0 * ROWB + c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = (wn * TN * 16 + fr) * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);

  // stage chunk kc into `st` (LDS-DMA pieces: wave w issues pieces w, w + 8, ...)
  auto stage = [&](const int kc, char* st) {
    const bool from1 = !CONCAT || (kc << 5) < p.C1;
    const int C = XF == 4 ? p.s2d : (from1 ? p.C1 : p.C2);
    const int sgrp = XF == 4 ? kc / (p.s2d >> 5) : 0, sa = sgrp >> 1, sb = sgrp & 1;
    const int cb = XF == 4 ? (kc << 5) - sgrp * p.s2d : (from1 ? (kc << 5) : (kc << 5) - p.C1);
    const __amdgpu_buffer_rsrc_t rs = from1 ? rs1 : rs2;
#pragma unroll
    for (int q = 0; q < (XI + 7) / 8; ++q) {
      const int k = wave + 8 * q;
      if (k < XI) {
        const int sl = 16 * k + lslot;
        const int hr = sl / HWP, hc = sl - hr * HWP;
        const int gr = g0 - 1 + hr;
        const int col = hc - 1;
        const bool row_in = hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in);
        const bool ok = row_in && (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
        const int lch = (lane & 3) ^ ((hc >> 1) & 3);
        const int lr = gr - grow0;
        const int pix = XF == 4 ? (2 * lr + sa) * (2 * W) + 2 * col + sb : lr * W + col;
        const int off = ok ? (pix * C + cb + lch * 8) * 2 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(st + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    char* Ws = st + XB;
    const int wl = (lslot * p.Kpad + (kc << 5) + lchunk * 8) * 2;
#pragma unroll
    for (int q = 0; q < (WI + 7) / 8; ++q) {
      const int k = wave + 8 * q;
      if (k < WI) {
        const int tap = k / (BN / 16), nb = (k % (BN / 16)) * 16;
        const int off = ((n0 + nb) * p.Kpad + tap * Cin) * 2 + wl;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
  };
  // XF 1: normalise chunk kc of stage `st` in place (thread t: logical 16-byte chunk
  // t & 3 of slots (t >> 2) + 128 j; padding slots keep the DMA's zeros)
  const size_t xsample = XF == 1 ? (size_t)(g0 / H) * p.xcs : 0;   // the window's sample (GroupNorm rows)
  auto xform = [&](const int kc, char* st) {
    constexpr int XNJ = (XI * 64 + PIPE_NTHR - 1) / PIPE_NTHR;
    const int xlc = tid & 3, xs0 = tid >> 2;
    const int cb = kc << 5;
    float xa[8], xb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      xa[e] = xco[cb + xlc * 8 + e];
      xb[e] = xco[256 + cb + xlc * 8 + e];
    }
#pragma unroll
    for (int j = 0; j < XNJ; ++j) {
      const int sl = xs0 + (PIPE_NTHR / 4) * j;
      const int hr = sl / HWP, hc = sl - hr * HWP;
      const int gr = g0 - 1 + hr;
      const bool ok = hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)gr < (unsigned)rows_total &&
                      (unsigned)(hc - 1) < (unsigned)W;
      if (!ok) continue;
      char* a = st + sl * 64 + 16 * (xlc ^ ((hc >> 1) & 3));
      float v[8];
      unpack8(*(const u32x4*)a, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(xa[e], v[e], xb[e]), 0.f);
      const u32x4 o = pack8(v);
      *(u32x4*)a = o;
      // the window's own rows (once: output-channel tile 0) -> xout
      if (p.xout && tn == 0 && hr >= 1 && hr <= R)
        *(u32x4*)((h16*)p.xout + (size_t)(gr * W + hc - 1) * p.C1 + cb + xlc * 8) = o;
    }
  };
  // chunk kc's MFMAs from stage `st` (the loop nest of conv_win_kernel's chunk_mfmas)
  auto mfmas = [&](const int kc, const char* st) {
    uint32_t tmask = 0x1ffu;
    if constexpr (XF == 4) {
      const int sgrp = kc / (p.s2d >> 5), sa = sgrp >> 1, sb = sgrp & 1;
      tmask = 0x1bu << (3 * (1 - sa) + (1 - sb));      // the 2 x 2 tap block of this phase
    }
    const char* Xs = st;
    const char* Ws = st + XB;
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      if (!((tmask >> dw) & 0x49u)) continue;
      h16x8 wf[3][TN];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[dh][j] = *(const h16x8*)(Ws + ((3 * dh + dw) * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int hr = 0; hr < RW + 2; ++hr) {
        const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * ROWB);
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) {
          const int ri = hr - dh;
          if (ri < 0 || ri >= RW) continue;
          if (!((tmask >> (3 * dh + dw)) & 1u)) continue;
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[ri][j] = mfma16(wf[dh][j], xf, acc[ri][j]);
        }
      }
    }
  };

  if constexpr (XF == 1) {
    for (int c = tid; c < p.C1; c += PIPE_NTHR) {
      xco[c] = p.xa[xsample + c];
      xco[256 + c] = p.xb[xsample + c];
    }
  }
  stage(0, lds0);
  for (int kc = 0; kc < nchunks; kc += 2) {
    __syncthreads();                 // chunk kc landed (vmcnt(0) + barrier); stage 1 free
    if (kc + 1 < nchunks) stage(kc + 1, lds1);
    if constexpr (XF == 1) {
      xform(kc, lds0);
      __syncthreads();
    }
    mfmas(kc, lds0);
    if (kc + 1 < nchunks) {
      __syncthreads();               // chunk kc + 1 landed; stage 0 free
      if (kc + 2 < nchunks) stage(kc + 2, lds0);
      if constexpr (XF == 1) {
        xform(kc + 1, lds1);
        __syncthreads();
      }
      mfmas(kc + 1, lds1);
    }
  }
  __syncthreads();
  using Map = StripTiles<W, RW, 1, NCS>;
  conv_epilogue<BM, BN, G::WMP, BN / G::WNS, TM, TN, PIPE_NTHR, EPI, Map, 0, W>(p, acc, lds0, g0 * W, n0, M, wm, wn,
                                                                                 lane, tid, 0, 0, tm);
}

template <int W>
hipError_t launch_pipe_w(const ConvFwdParams& p, hipStream_t s) {
  using G = PipeGeo<W>;
  const int grid = ((p.N * p.OH + G::R - 1) / G::R) * (p.Cout / G::BN);
  const bool cc = p.C2 > 0;
  const int epi = conv_epi_mode(p);
#define PIPE_L(CC, E, XX) \
  hipLaunchKernelGGL((conv_pipe_kernel<W, CC, E, XX>), dim3(grid), dim3(PIPE_NTHR), 0, s, p)
  if (p.xform) {                      // (conv_fwd_prepare: xform 1, single source, STATS / GENERIC)
    if (cc || p.xform != 1 || p.C1 > 256) return hipErrorInvalidValue;
    if (epi == EPI_STATS) PIPE_L(false, EPI_STATS, 1);
    else if (epi == EPI_GENERIC) PIPE_L(false, EPI_GENERIC, 1);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
  if (p.s2d) {
    if (cc) return hipErrorInvalidValue;
    if (epi == EPI_DGRAD) PIPE_L(false, EPI_DGRAD, 4);
    else if (epi == EPI_DGRAD_NORM) PIPE_L(false, EPI_DGRAD_NORM, 4);
    else return hipErrorInvalidValue;
    return hipGetLastError();
  }
#define PIPE_E(CC)                                                         \
  if (epi == EPI_FWD) PIPE_L(CC, EPI_FWD, 0);                              \
  else if (epi == EPI_DGRAD) PIPE_L(CC, EPI_DGRAD, 0);                     \
  else if (epi == EPI_STATS) PIPE_L(CC, EPI_STATS, 0);                     \
  else if (epi == EPI_GENERIC) PIPE_L(CC, EPI_GENERIC, 0);
  if (cc) {
    PIPE_E(true)
    else return hipErrorInvalidValue;        // (the dgrad-norm epilogue has one destination)
  } else {
    PIPE_E(false)
    else PIPE_L(false, EPI_DGRAD_NORM, 0);
  }
#undef PIPE_E
#undef PIPE_L
  return hipGetLastError();
}

}  // namespace

hipError_t launch_pipe(const ConvFwdParams& p, hipStream_t s) {
  switch (p.OW) {
    case 16: return launch_pipe_w<16>(p, s);
    case 32: return launch_pipe_w<32>(p, s);
    case 64: return launch_pipe_w<64>(p, s);
    default: return hipErrorInvalidValue;
  }
}
#endif  // UNET_PIPE_IMPL

}  // namespace unet
