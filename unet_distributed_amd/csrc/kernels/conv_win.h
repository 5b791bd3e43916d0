// Row-window 3x3 conv kernels (fine UNet levels), shared by the instantiation units
// conv_win_b32.hip (32-channel tiles) and conv_win_b64.hip (64-channel tiles): each
// builds one launch_win<BN, BM> so the ~150 kernel variants compile in parallel.
// conv_fwd.hip picks the tile (win_bn / win_bm) and dispatches.
#pragma once
#include "common.h"
#include "conv_params.h"
#include "conv_epilogue.h"
#include "head_grad.h"
#include <type_traits>

namespace unet {

// GEO: 0 = 2D full rows (Wf = W), 1 = 2D segmented rows (Wf = p.OW, a multiple of W),
// 2 = 3D full rows (three depth taps).  Compile-time so the common 2D case carries no
// segment / depth state (extra SGPR state spilled to VGPR lanes inside the chunk loop).
enum { GEO_2D = 0, GEO_SEG = 1, GEO_3D = 2 };

// Output-channel tile of the row-window conv: 64 on rows 16..64 wide where Cout allows
// it (same-box sweep of the headline step: +2.8 % at W = 16, +0.5 % at 32, +0.4 % at 64,
// -0.3 % at 128 -> 32 there), else 32; a fused head needs the 32-channel tile.  64
// halves the halo image's LDS-DMA and fragment reads per MFMA and doubles the MFMA work
// per synchronisation.  tile 12 / 6 force 64 / 32 (tests).
inline int win_bn(const ConvFwdParams& p) {
  if (p.tile == 12) return 64;
  if (p.tile == 6) return 32;
  const int W = p.OW > 128 ? 128 : p.OW;
  return (p.Cout % 64 == 0 && W <= 64 && !p.head_w) ? 64 : 32;
}
// Window pixels: 256 for 16-wide rows and for the 64-channel tile (its accumulators,
// 4 x 4 fragments per wave, and LDS then still fit two workgroups per CU), else 512.
// (A 256-pixel 32-channel window on 32..128-wide rows -- three workgroups per CU --
// measured -0.4 % at W = 64 and -1 % at 128 and was dropped; a pipelined 8-wave window
// with double-buffered chunks, one workgroup per CU, measured -2..-21 % per launch at
// levels 2-4 in round 4: two independent workgroups per CU already overlap one's DMA
// wait with the other's MFMAs, AND its prologue / epilogue, which one workgroup cannot.)
inline int win_bm(const ConvFwdParams& p) {
  const int W = p.OW > 128 ? 128 : p.OW;
  return (W == 16 || win_bn(p) == 64) ? 256 : 512;
}
inline int win_rows(const ConvFwdParams& p) {
  const int W = p.OW > 128 ? 128 : p.OW;
  return win_bm(p) / W;
}
// Persistent prefetching window (conv_win_pf_kernel): 2D, 128-wide rows, one 32-channel
// input chunk, 32 output channels, bias + ReLU forward or data-gradient epilogue (level 1
// of the 128^2 UNet: the forward of conv1b / conv9b, the skip data gradient of conv9a).
// (every epilogue mode; the head-on-load data gradient of the head input too)
// (rows wider than 128 -- the 512^2 / 256^2 models' level 1 -- as 128-wide segments)
inline bool win_pf_eligible(const ConvFwdParams& p) {
  const bool w_ok = p.OW == 128 || (p.OW % 128 == 0 && p.OW > 128 && p.OW <= 8192 && !p.hg.prob);
  return p.win_pf > 0 && w_ok && p.KD == 1 && p.OD == 1 && p.C1 == 32 && p.C2 == 0 && p.Cout == 32 &&
         p.tile != 12 && !p.s2d && !p.ut.x && !p.fw.x && p.OH % 4 == 0 &&
         (!p.hg.prob || conv_epi_mode(p) == EPI_DGRAD) &&
         (!p.xform || (p.xform == 1 && p.OW == 128 && !p.hg.prob && !(p.xd_rate > 0.f)));
}
constexpr int CP_DZ_MAXC = 128;      // conv_win_cp_kernel DZ: input channels in LDS coefficients
// Chunk-pipelined window (conv_win_cp_kernel): 2D 64-wide full rows, the 64-channel tile,
// plain or concat source, no operand transform, two or more 32-channel input chunks (level 2
// of the 128^2 UNet).  (At levels 3-4 -- 32 / 16-wide rows, 4..16 chunks -- the per-launch
// times rose 0.016-0.034 ms against the DMA chunk loop, run V: not used there.)
inline bool win_cp_eligible(const ConvFwdParams& p) {
  return p.win_cp > 0 && p.OW == 64 && p.KD == 1 && p.OD == 1 &&
         p.C1 + p.C2 >= 64 && p.Cout % 64 == 0 && !p.head_w && p.tile != 6 &&
         (!p.xform || (p.xform == 2 && !p.C2 && p.C1 <= CP_DZ_MAXC)) && !p.hg.prob &&
         !p.s2d && !p.ut.x && !p.fw.x;
}
// Chunk-pipelined window on 128-wide rows (conv_win_cp128_kernel): 2D with two or more input
// chunks, or 3D (3x3x3: depth taps x chunks), the 32-channel tile, no operand transform
// (the 3D level 1 of the 128^3 UNet, the 512^2 model's 128-wide level).
inline bool win_cp128_eligible(const ConvFwdParams& p) {
  const bool d3 = p.KD == 3 && p.OD > 1;
  return p.win_cp > 1 && p.OW == 128 && (d3 || (p.KD == 1 && p.OD == 1 && p.C1 + p.C2 >= 64)) && p.tile != 12 &&
         !p.xform && !p.hg.prob && !p.s2d && !p.ut.x && !p.fw.x && !win_pf_eligible(p);
}
// Persistent prefetching tconv-on-load window (conv_win_pfu_kernel): conv9a of the 128^2 UNet --
// 2D 128-wide rows, u (32 channels) = tconv2x2s2 of a 32 / 64-channel coarse input formed on
// load + a 32-channel skip source, 32 output channels, bias + ReLU epilogue or the
// normalised configs' statistics epilogue (pre-norm z + one {sum z, sum z^2} row per
// 256-pixel window: conv_stat_tiles).
inline bool win_pfu_eligible(const ConvFwdParams& p) {
  return p.win_pf > 0 && p.ut.x && p.OW == 128 && p.KD == 1 && p.OD == 1 && p.C1 == 32 && p.C2 == 32 &&
         p.Cout == 32 && (p.ut.C == 32 || p.ut.C == 64) && p.tile != 12 &&
         (conv_epi_mode(p) == EPI_FWD || conv_epi_mode(p) == EPI_STATS) && !p.pool_dst && !p.head_w &&
         p.OH % 2 == 0;
}
inline int win_grid(const ConvFwdParams& p) {
  const int W = p.OW > 128 ? 128 : p.OW;          // window segment width
  const int rows = p.N * p.OD * p.OH;
  const int R = win_rows(p);
  if (win_pf_eligible(p)) return (rows / 4 * (p.OW / 128) + p.win_pf - 1) / p.win_pf;
  if (win_pfu_eligible(p)) return (rows / 2 + p.win_pf - 1) / p.win_pf;
  return ((rows + R - 1) / R) * (p.OW / W) * (p.Cout / win_bn(p));
}
// (BN, BM, row width) combinations win_bn / win_bm can select (the 64-channel tile also
// on 128-wide rows: tile 12 forces it there for tests)
template <int BN, int BM>
constexpr bool win_tile_built(int W) {
  return BN == 64 ? BM == 256 : (BM == 256 ? W == 16 : W != 16);
}

template <int BN, int BM>
hipError_t launch_win(const ConvFwdParams& p, hipStream_t s);

// fused data + weight gradient window (conv_dw.hip, tile 14; conv_params.h FusedWgrad)
const char* conv_dw_check(const ConvFwdParams& p);
int conv_dw_grid(const ConvFwdParams& p);
int conv_dw_stat_rows(const ConvFwdParams& p);
hipError_t launch_conv_dw(const ConvFwdParams& p, hipStream_t s);

#ifdef UNET_WIN_IMPL
namespace {

constexpr int NTHR = 256;

// ---------------------------------------------------------------------------------
// Row-window conv (fine UNet levels): 2D, 3x3, stride 1, 'same' padding, full-width rows.
//
// The implicit GEMM above re-gathers the input once per tap: at the 128^2 / 64^2
// levels (Cin, Cout <= 64) that 9x L2->LDS traffic, not the MFMA, bounds it.  Here a
// workgroup owns BM = 512 output pixels = R = 512/W whole rows of the flattened
// (n, h) row space and BN output channels.  Per 32-channel input chunk it stages the
// (R+2) x (W+2) halo image of those rows ONCE in LDS (zero columns at the left/right
// border come free from out-of-range buffer loads), plus the chunk's 9 x BN weight
// rows, and then runs all nine taps as MFMAs on shifted LDS addresses.  Rows that
// cross an image boundary inside the window are handled by skipping the (wave-uniform)
// MFMAs of taps whose input row falls outside the output row's image.
//
// LDS images: 64-byte pixel slots (32 bf16); the halo image has rows of HWP = W + 4
// slots (a multiple of 4: every row starts on a 256-byte bank row) and stores 16-byte
// chunk c of the pixel in column hc at c ^ ((hc >> 1) & 3).  Fragment reads are 16
// consecutive columns from any start (any tap shift): conflict free, and because the
// swizzle depends only on the column, a lane's address is one of three per-lane bases
// (one per horizontal tap) plus a compile-time immediate (row, tile) -- no per-tap
// address registers.  Weight rows (tap, n) use the same swizzle on the row index.

// XF (2D, single source): operand transform of the src1 halo image in LDS before the
// MFMAs -- 1: conv_params.h xform 1, y = relu(xa z + xb) (the window's own rows of the
// transformed operand go to xout); 2: the conv's own norm backward on load (data gradient of a
// normalised layer: src1 = g, p.xz = z, the halo becomes dz = ca g + cb z + cc, the
// norm_bwd_apply formula and rounding); 3: head-on-load, the halo image of dY (32 channels)
// is formed from the head's per-pixel probability, target and ReLU bits (p.hg,
// head_grad.h) instead of being read from memory; 4: space-to-depth source (p.s2d: the
// DMA gathers the fine pixels of each coarse slot, structurally zero taps skipped); 5
// (2D concat): the src1 chunks are the transposed conv u = tconv2x2s2(p.ut.x) + b formed
// in LDS (conv_params.h TconvSrc), the src2 (skip) chunks are DMA'd as usual.
template <int W, int BN, int BM, bool CONCAT, int EPI, int GEO, int XF = 0>
__global__ void __launch_bounds__(NTHR) conv_win_kernel(const ConvFwdParams p) {
  static_assert(BN == 32 || BN == 64, "row-window tile is 32 or 64 output channels wide");
  static_assert(XF == 0 || ((XF == 1 || XF == 2 || XF == 3 || XF == 4) && GEO == GEO_2D && !CONCAT) ||
                    (XF == 5 && GEO == GEO_2D && CONCAT) || (XF == 3 && GEO == GEO_3D && !CONCAT),
                "operand transform: 2D single-source windows (tconv on load: 2D concat; head on load: 3D too)");
  constexpr int R = BM / W, HR = R + 2;
  // halo row pitch in 64-byte pixel slots: W + 2 columns rounded up to a multiple of 4
  // (every row starts on a 256-byte bank row); the DMA fills the image as one linear
  // run of slots, so rows need not align to the 16-slot DMA instructions
  // ALR (2D, 128-wide rows: one or two chunks per window, so the DMA address set-up is
  // not amortised): rows padded to whole 16-slot DMA pieces -- a piece then lies in one
  // halo row, its row checks and row offset are wave-uniform (scalar), and a lane's
  // column / swizzle part is the same for every piece: a few VALU per piece instead of a
  // division by the pitch and 64-bit address math (73.7 KB LDS, still two WGs per CU)
  constexpr bool ALR = GEO == GEO_2D && W == 128;
  constexpr int HWP = ALR ? (W + 2 + 15) / 16 * 16 : W + 4;
  constexpr int PPR = HWP / 16;                 // DMA pieces per halo row (ALR)
  constexpr int ROWB = HWP * 64;
  constexpr int XI = (HR * HWP + 15) / 16, WI = 9 * BN / 16;
  constexpr int XB = XI * 1024, WB = WI * 1024;
  constexpr int EPIB = (EPI == EPI_STATS || EPI == EPI_DGRAD_NORM) ? epi_lds_bytes<BM, BN>() : BM * (BN + 4) * 2;
  constexpr int LDS_BYTES = (XB + WB > EPIB) ? XB + WB : EPIB;
  constexpr int WMP = BM / 4;                   // pixels per wave
  constexpr int TM = WMP / 16, TN = BN / 16;
  constexpr int TPR = W / 16;                   // 16-pixel tiles per row
  static_assert(W >= 16 && W <= 128 && BM % W == 0 && WMP % 16 == 0, "row width");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ws = smem + XB;

  // wave index as a scalar: every per-wave quantity below (rows, DMA slots) stays in SGPRs
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Row space: rows g = (n, d, h) of Wf pixels.  Rows wider than 128 are cut into
  // nseg W-wide segments (a window = R rows x one segment; its halo columns -1 / W are
  // the neighbouring segments' pixels).  3D (KD = 3): depth tap dz reads the halo rows
  // of slice d + dz - 1, i.e. row g + (dz - 1) H, as three more 32-channel K chunks.
  constexpr int KD = GEO == GEO_3D ? 3 : 1;
  const int H = p.OH;
  const int D = GEO == GEO_3D ? p.OD : 1;
  const int Wf = GEO == GEO_SEG ? p.OW : W;
  const int nseg = GEO == GEO_SEG ? p.OW / W : 1;
  const int rows_total = p.N * D * H;
  const int M = rows_total * Wf;
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm0 = bid / tiles_n, tn = bid % tiles_n;
  const int tm = p.rev ? (int)(gridDim.x / tiles_n) - 1 - tm0 : tm0;
  const int rgi = GEO == GEO_SEG ? tm / nseg : tm;
  const int g0 = rgi * R, col0 = GEO == GEO_SEG ? (tm - rgi * nseg) * W : 0;
  const int n0 = tn * BN;
  const int dsl = GEO == GEO_3D ? (g0 / H) % D : 0;   // depth slice of the window
  const int Cin = p.C1 + p.C2;
  const int nchunks = Cin >> 5;
  constexpr int OOB = 0x7fffffff;
  // image-relative buffer bases: a window's rows (halo included) never leave its image,
  // so the 32-bit DMA offsets count from the image's first pixel and a whole tensor may
  // exceed 2 GiB (conv_fwd_prepare bounds one image)
  const int grow0 = (g0 / (D * H)) * (D * H);
  const size_t img_px = (size_t)grow0 * Wf;
  const char* s1b = (const char*)p.src1 + img_px * (XF == 4 ? 4 * p.s2d : p.C1) * 2;
  const char* s2b = p.src2 ? (const char*)p.src2 + img_px * p.C2 * 2 : s1b;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)s1b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)s2b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);

  // Wave w owns an RW-row x 16 TC-column strip of the window (StripTiles): an A
  // fragment read from halo row r at horizontal shift dw feeds the output rows r - dh
  // of all three vertical taps, so per chunk a wave reads 3 (RW + 2) TC fragments
  // instead of 9 RW TC (2-2.4x less LDS read traffic than one fragment per tap).
  constexpr int TC = W >= 128 ? 2 : 1;            // 16-pixel column tiles per strip
  constexpr int NCS = W / (16 * TC);              // column strips per window row
  constexpr int RW = R / (4 / NCS);               // rows per strip
  static_assert(NCS <= 4 && 4 % NCS == 0 && RW * TC == TM, "strip map");
  using Map = StripTiles<W, RW, TC, NCS>;
  const int r0 = (wave / NCS) * RW, c0 = (wave % NCS) * 16 * TC;
  // H % R == 0 (win_eligible): a window never spans two images, so the only rows of
  // another image are the halo rows above / below it, which the DMA fills with zeros
  // (the 'same' padding) -- the tap loop needs no image-edge branches at all, and the
  // whole chunk is one basic block the scheduler can pipeline LDS reads through.
  const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fsub = lane >> 4, fr = lane & 15;
  // per-lane fragment bases: horizontal tap dw -> column c0 + fr + dw of halo row r0
  // (c0 is a multiple of 16, so the swizzle only depends on fr + dw)
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = r0 * ROWB + c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  // one 32-channel chunk: per horizontal tap, the three vertical taps' weights are
  // held in registers and every halo-row fragment feeds up to three output rows
  // tmask: taps (bit 3 dh + dw) of this chunk that are not structurally zero (XF 4);
  // a compile-time 0x1ff everywhere else, so the tests fold away
  auto chunk_mfmas = [&](const uint32_t tmask) {
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      if (!((tmask >> dw) & 0x49u)) continue;     // no valid tap in this column
      h16x8 wf[3][TN];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[dh][j] = *(const h16x8*)(Ws + ((3 * dh + dw) * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int hr = 0; hr < RW + 2; ++hr) {
#pragma unroll
        for (int ci = 0; ci < TC; ++ci) {
          const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * ROWB + ci * 16 * 64);
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int ri = hr - dh;
            if (ri < 0 || ri >= RW) continue;
            if (!((tmask >> (3 * dh + dw)) & 1u)) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[ri * TC + ci][j] = mfma16(wf[dh][j], xf, acc[ri * TC + ci][j]);
          }
        }
      }
    }
  };
  // LDS-DMA lane roles: lane l fills physical 16-byte chunk (l & 3) of slot (l >> 2) of a
  // 16-slot run; it loads logical chunk (l & 3) ^ swizzle(slot), which depends only on l
  // because every run starts at a multiple of 16 slots.
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);

  // one 32-channel chunk of depth tap kd (input rows shifted by gsh): stage, then MFMAs
  auto run_chunk = [&](const int kc, const int kd, const int gsh) {
      const bool from1 = !CONCAT || (kc << 5) < p.C1;
      const int C = from1 ? p.C1 : p.C2;
      const int cb = from1 ? (kc << 5) : (kc << 5) - p.C1;
      if constexpr (XF == 3) {
        // head-on-load halo of depth tap kd (3D): slot (hr, hc) holds dY of pixel
        // (g0 - 1 + hr + gsh, hc - 1) formed from the head (the 2D path's formula); the
        // depth-shifted slice is inside the volume (the caller skips padding taps)
        constexpr int NSL = XI * 16, HJ = (NSL + NTHR - 1) / NTHR;
        const HeadGradCtx hctx = head_grad_ctx(p.hg);
        float hpr[HJ], htv[HJ];
        uint32_t hbits[HJ];
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
          const int sl = tid + NTHR * j;
          const int hr = sl / HWP, hc = sl - hr * HWP;
          const int gr = g0 - 1 + hr + gsh, col = hc - 1;
          const bool ok = sl < NSL && hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                          (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
          const int pix = ok ? gr * W + col : 0;
          hpr[j] = p.hg.prob[pix];
          htv[j] = bits2f(((const uint16_t*)p.hg.t)[pix]);
          hbits[j] = ok ? ((const uint32_t*)p.hg.bits)[pix] : 0u;
        }
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
          const int sl = tid + NTHR * j;
          if (sl >= NSL) continue;
          const int hc = sl % HWP;
          const float dz = head_dlogit(hpr[j], htv[j], hctx.a, hctx.bb, hctx.inv_total, hctx.bce_w, hctx.gscale);
          const int sw = (hc >> 1) & 3;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float v = dz * hctx.w[8 * k + e];
              o[e] = ((hbits[j] >> (8 * k + e)) & 1u) ? v : 0.f;
            }
            *(u32x4*)(Xs + sl * 64 + 16 * (k ^ sw)) = pack8(o);
          }
        }
      }
      {
        // halo image: row hr, slot hc holds pixel (g0 - 1 + hr + gsh, col0 + hc - 1);
        // instruction (hr, j) covers slots 16j .. 16j + 15 of row hr.  Rows outside the
        // tensor / image and columns outside [0, Wf) load zeros (out-of-range offsets).
        const __amdgpu_buffer_rsrc_t rs = from1 ? rs1 : rs2;
#pragma unroll
        for (int q = 0; q < (XI + 3) / 4; ++q) {
          const int k = wave + 4 * q;
          if (XF != 3 && k < XI) {
            const int sl = 16 * k + lslot;                  // this lane's halo slot
            const int hr = sl / HWP, hc = sl - hr * HWP;    // its row / column
            const int gr = g0 - 1 + hr + gsh;
            const int col = col0 + hc - 1;
            const bool row_in = hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in);   // same image
            // (slots past W + 1 are never read: skip them, they would be real pixels of
            // the next segment on segmented rows)
            const bool ok = row_in && (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)Wf &&
                            (GEO != GEO_SEG || hc <= W + 1);
            const int lch = (lane & 3) ^ ((hc >> 1) & 3);
            const int off = ok ? (((gr - grow0) * Wf + col) * C + cb + lch * 8) * 2 : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(Xs + k * 1024),
                                                     16, off, 0, 0, 0);
          }
        }
        // weight image: row r = tap * 32 + n (64 bytes = this chunk's 32 input channels)
        const int wl = (lslot * p.Kpad + (kc << 5) + lchunk * 8) * 2;
#pragma unroll
        for (int q = 0; q < (WI + 3) / 4; ++q) {
          const int k = wave + 4 * q;
          if (k < WI) {
            const int tap = k / (BN / 16), nb = (k % (BN / 16)) * 16;     // wave-uniform
            const int off = ((n0 + nb) * p.Kpad + (kd * 9 + tap) * Cin) * 2 + wl;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024),
                                                     16, off, 0, 0, 0);
          }
        }
      }
      __syncthreads();
      chunk_mfmas(0x1ffu);
  };
  if constexpr (GEO == GEO_3D) {
    // depth taps whose input slice is padding contribute nothing: skip them
    const int kd_lo = dsl == 0 ? 1 : 0, kd_hi = dsl == D - 1 ? 2 : 3;
    for (int kd = kd_lo; kd < kd_hi; ++kd)
      for (int kc = 0; kc < nchunks; ++kc) {
        if (kc || kd != kd_lo) __syncthreads();   // previous chunk's fragment reads are done
        run_chunk(kc, kd, (kd - 1) * H);
      }
  } else if constexpr (GEO == GEO_SEG) {
    for (int kc = 0; kc < nchunks; ++kc) {
      if (kc) __syncthreads();                    // previous chunk's fragment reads are done
      run_chunk(kc, 0, 0);
    }
  } else {
    // 2D full rows: the same staging with compile-time row pitch and no segment / depth
    // offsets, spelled out (through run_chunk the scheduler keeps ~100 more scalar
    // instructions per chunk and spills SGPRs to VGPR lanes: 2-4 % slower, A/B measured)
    // operand transform: thread t owns logical 16-byte chunk xlc = t & 3 (channels
    // cb + 8 xlc ..) of slots (t >> 2) + 64 j, so its 8 channels' coefficients are fixed
    // per chunk; the slot's physical chunk is xlc ^ swizzle(column), as the DMA wrote it
    constexpr int XNJ = (XF == 1 || XF == 2) ? (XI * 64 + NTHR - 1) / NTHR : 1;
    const int xlc = tid & 3, xs0 = tid >> 2;
    auto xslot = [&](const int j, int& hr, int& hc, int& gr, bool& ok) {
      const int sl = xs0 + (NTHR / 4) * j;
      hr = sl / HWP;
      hc = sl - hr * HWP;
      gr = g0 - 1 + hr;
      ok = hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)gr < (unsigned)rows_total &&
           (unsigned)(hc - 1) < (unsigned)W;
      return sl;
    };
    const size_t xsample = (XF == 1 || XF == 2) ? (size_t)(g0 / H) * p.xcs : 0;   // the window's sample (GroupNorm rows)
    // XF 2: z of the halo slots (the image-relative base of conv_fwd's src1 layout, C1 channels)
    const __amdgpu_buffer_rsrc_t rsz = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(XF == 2 ? (const char*)p.xz + img_px * p.C1 * 2 : s1b), (short)0, OOB, 0x00020000);
    // XF 5: u channels cb .. cb + 31 of the halo image from the coarse input.  The HR fine
    // halo rows come from NCR = R / 2 + 2 coarse rows (R even); wave w takes coarse rows
    // cq = w, w + 4, ..: it loads the row's B fragments (16 coarse pixels x 32 coarse
    // channels each, straight from global memory -- one HBM round trip per coarse row)
    // and forms the fine rows 2 cq - 1 + th inside the halo for the four phases
    // t = (th, tw) = 2 th + tw, one 16 x 16 x 32 MFMA chain per (16 coarse pixels, 16 u
    // channels) with the tap's weight rows as A (L2-resident; the next tap's are loaded
    // under the current tap's MFMAs where registers allow).  Same operands and
    // accumulation order as tconv_fwd_kernel, so u is bit-identical to the materialised
    // one.  Every slot a fragment read touches is written: rows outside the image and the
    // columns -1 / W are zeros, as the DMA's out-of-range loads would have left them.
    auto ut_chunk = [&](const int cb, auto ksc) {
      constexpr int KS = decltype(ksc)::value;    // 32-channel K steps of the coarse input
      constexpr int CW = W / 2, PB = XF == 5 ? CW / 16 : 1, NCR = R / 2 + 2;
      static_assert(XF != 5 || (R % 2 == 0 && CW % 16 == 0), "tconv on load: even window rows, coarse rows 16k wide");
      if constexpr (PB * KS <= 8) {               // (conv_fwd_prepare: (W / 32) (C / 32) <= 8)
        const int Cc = KS * 32;
        // A rows permuted so that a lane's two 16 x 16 tiles hold 8 consecutive u channels:
        // tile j row fr = channel 8 (fr >> 2) + 4 j + (fr & 3), so output rows 4 fsub + i of
        // tile j are channels 8 fsub + 4 j + i -- logical 16-byte chunk fsub of the pixel,
        // one 16-byte store.  (Each output element keeps its operands and accumulation
        // order: still bit-identical to tconv_fwd_kernel.)
        const h16* wt = (const h16*)p.ut.w + (size_t)(cb + 8 * (fr >> 2) + (fr & 3)) * p.ut.kpad + 8 * fsub;
        // the window's image in the coarse tensor (H even: fine row g -> coarse row g / 2)
        const h16* ub = (const h16*)p.ut.x + (size_t)(grow0 >> 1) * CW * Cc + (size_t)fr * Cc + 8 * fsub;
        float bs[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) bs[i] = p.ut.b[cb + 8 * fsub + i];
        h16x8 xb[PB][KS];
        h16x8 wa[2][2][KS];                       // [tw][j][ks]: both column phases of a tap row
        // store roles: in store s, lane fr writes column phase tw = s ^ ((fr >> 2) & 1).  The 8
        // lanes of a 16-byte store group (fr 0-3 / 4-7 of one fsub) then cover both 64-byte
        // halves of the 32-bank window (fine column parity) and all four swizzles
        // (column >> 1) & 3: conflict-free (tools/lds_bank_model.py check_ut_store).  With
        // one phase per store only 4 of the 8 slots are reachable (2-way); the previous
        // 8-byte per-tile stores were 4-way conflicted (35 % conflict cycles, r5 PMC).
        const int tsel = (fr >> 2) & 1;
        for (int cq = wave; cq < NCR; cq += 4) {
          // fine halo rows hr = 2 cq - 1 + th of this coarse row; in the image <=> the
          // coarse row is (window rows never leave their image, conv_fwd_prepare)
          const int crow = (g0 >> 1) - 1 + cq;                   // global coarse row
          const int gr0 = 2 * crow;
          const bool in = (2 * cq - 1 >= 1 || top_in) && (2 * cq <= R || bot_in) &&
                          (unsigned)gr0 < (unsigned)rows_total;
          if (in) {
            const h16* rp = ub + (size_t)(crow - (grow0 >> 1)) * CW * Cc;
#pragma unroll
            for (int pb = 0; pb < PB; ++pb)
#pragma unroll
              for (int ks = 0; ks < KS; ++ks) xb[pb][ks] = *(const h16x8*)(rp + (size_t)(16 * pb) * Cc + 32 * ks);
          }
          const int th_lo = cq == 0 ? 1 : 0, th_hi = cq == NCR - 1 ? 1 : 2;   // tap rows inside the halo
#pragma unroll
          for (int th = 0; th < 2; ++th) {
            if (th < th_lo || th >= th_hi) continue;
            if (in) {
#pragma unroll
              for (int tw = 0; tw < 2; ++tw)
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                  for (int ks = 0; ks < KS; ++ks)
                    wa[tw][j][ks] = *(const h16x8*)(wt + (size_t)((2 * th + tw) * p.C1 + 4 * j) * p.ut.kpad + 32 * ks);
            }
            char* xrow = Xs + (2 * cq - 1 + th) * ROWB;
#pragma unroll
            for (int pb = 0; pb < PB; ++pb) {
              u32x4 pk[2] = {(u32x4){0u, 0u, 0u, 0u}, (u32x4){0u, 0u, 0u, 0u}};
              if (in) {
#pragma unroll
                for (int tw = 0; tw < 2; ++tw)
#pragma unroll
                  for (int j = 0; j < 2; ++j) {
                    // (packed at once: one live accumulator keeps the W = 128 instance at
                    // 191 VGPRs + 64 AGPRs, two waves per SIMD; both tiles live -> 260)
                    f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
                    for (int ks = 0; ks < KS; ++ks) a = mfma16(wa[tw][j][ks], xb[pb][ks], a);
                    pk[tw][2 * j] = pack2h(a[0] + bs[4 * j], a[1] + bs[4 * j + 1]);
                    pk[tw][2 * j + 1] = pack2h(a[2] + bs[4 * j + 2], a[3] + bs[4 * j + 3]);
                  }
              }
#pragma unroll
              for (int s = 0; s < 2; ++s) {
                const int tw = s ^ tsel;
                const int hc = 2 * (16 * pb + fr) + tw + 1;
                *(u32x4*)(xrow + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3))) = tw ? pk[1] : pk[0];
              }
            }
            // halo columns 0 and W + 1 of the row (lanes 0-3 / 4-7: one 16-byte chunk each)
            if (lane < 8) *(u32x4*)(xrow + ((lane >> 2) ? W + 1 : 0) * 64 + 16 * (lane & 3)) = (u32x4){0u, 0u, 0u, 0u};
          }
        }
      }
    };
    for (int kc = 0; kc < nchunks; ++kc) {
      const bool from1 = !CONCAT || (kc << 5) < p.C1;
      // space-to-depth gathered chunk: every chunk of XF 4
      constexpr bool s2 = XF == 4;
      const int C = s2 ? p.s2d : (from1 ? p.C1 : p.C2);
      // XF 4: chunk kc = phase group (sa, sb) of the space-to-depth image, fine channels
      // cb .. cb + 31; its valid taps dh in {1 - sa, 2 - sa}, dw in {1 - sb, 2 - sb}
      const int sgrp = s2 ? kc / (p.s2d >> 5) : 0, sa = sgrp >> 1, sb = sgrp & 1;
      const int cb = s2 ? (kc << 5) - sgrp * p.s2d : (from1 ? (kc << 5) : (kc << 5) - p.C1);
      const uint32_t s2d_taps = 0x1bu << (3 * (1 - sa) + (1 - sb));   // the 2 x 2 tap block
      if (kc) __syncthreads();
      {
        const __amdgpu_buffer_rsrc_t rs = from1 ? rs1 : rs2;
#pragma unroll
        for (int q = 0; q < (XI + 3) / 4; ++q) {
          const int k = wave + 4 * q;
          if (XF != 3 && !(XF == 5 && from1) && k < XI) {
            int hr, hc;
            if constexpr (ALR) {
              hr = k / PPR;                                 // wave-uniform
              hc = 16 * (k - hr * PPR) + lslot;
            } else {
              const int sl = 16 * k + lslot;
              hr = sl / HWP;
              hc = sl - hr * HWP;
            }
            const int gr = g0 - 1 + hr;
            const int col = hc - 1;
            const bool row_in = hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in);
            const bool ok = row_in && (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
            // (ALR: pieces start on 16-slot boundaries, so the swizzle is lchunk's)
            const int lch = ALR ? lchunk : (lane & 3) ^ ((hc >> 1) & 3);
            // XF 4: the coarse slot's fine pixel (2 gr + sa, 2 col + sb) of the 2W-wide rows
            const int lr = gr - grow0;                      // image-relative row
            const int pix = s2 ? (2 * lr + sa) * (2 * W) + 2 * col + sb : lr * W + col;
            const int off = ok ? (pix * C + cb + lch * 8) * 2 : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(Xs + k * 1024),
                                                     16, off, 0, 0, 0);
          }
        }
        const int wl = (lslot * p.Kpad + (kc << 5) + lchunk * 8) * 2;
#pragma unroll
        for (int q = 0; q < (WI + 3) / 4; ++q) {
          const int k = wave + 4 * q;
          if (k < WI) {
            const int tap = k / (BN / 16), nb = (k % (BN / 16)) * 16;
            const int off = ((n0 + nb) * p.Kpad + tap * Cin) * 2 + wl;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024),
                                                     16, off, 0, 0, 0);
          }
        }
      }
      // XF 2: the thread's z granules and 8 channels' coefficients, in flight with the DMA
      u32x4 zq[XF == 2 ? XNJ : 1];
      float za[8], zb[8], zc[8];
      if constexpr (XF == 2) {
#pragma unroll
        for (int j = 0; j < XNJ; ++j) {
          int hr, hc, gr;
          bool ok;
          xslot(j, hr, hc, gr, ok);
          zq[j] = __builtin_amdgcn_raw_buffer_load_b128(
              rsz, ok ? (((gr - grow0) * W + hc - 1) * p.C1 + cb + xlc * 8) * 2 : OOB, 0, 0);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const size_t ci = xsample + cb + xlc * 8 + e;
          za[e] = p.xa[ci];
          zb[e] = p.xb[ci];
          zc[e] = p.xc[ci];
        }
      }
      if constexpr (XF == 5) {
        if (from1) {
          if (p.ut.C == 64)
            ut_chunk(cb, std::integral_constant<int, 2>{});
          else if (p.ut.C == 128)
            ut_chunk(cb, std::integral_constant<int, 4>{});
          else
            ut_chunk(cb, std::integral_constant<int, 1>{});
        }
      }
      if constexpr (XF == 3) {
        // head-on-load halo image (one 32-channel chunk): every slot of the image is
        // written (zeros outside the tensor / image, like the DMA's out-of-range loads);
        // a thread's slots' pixel data are loaded first, then formed and stored.  (One
        // slot per thread: 3 loads per slot; a chunk per thread -- conflict-free 16-byte
        // stores but 4x the loads -- measured -0.8 % on the step.)
        constexpr int NSL = XI * 16, HJ = (NSL + NTHR - 1) / NTHR;
        const HeadGradCtx hctx = head_grad_ctx(p.hg);
        float hpr[HJ], htv[HJ];
        uint32_t hbits[HJ];
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
          const int sl = tid + NTHR * j;
          const int hr = sl / HWP, hc = sl - hr * HWP;
          const int gr = g0 - 1 + hr, col = hc - 1;
          const bool ok = sl < NSL && hr < HR && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                          (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
          const int pix = ok ? gr * W + col : 0;
          hpr[j] = p.hg.prob[pix];
          htv[j] = bits2f(((const uint16_t*)p.hg.t)[pix]);
          hbits[j] = ok ? ((const uint32_t*)p.hg.bits)[pix] : 0u;
        }
#pragma unroll
        for (int j = 0; j < HJ; ++j) {
          const int sl = tid + NTHR * j;
          if (sl >= NSL) continue;
          const int hc = sl % HWP;
          const float dz = head_dlogit(hpr[j], htv[j], hctx.a, hctx.bb, hctx.inv_total, hctx.bce_w, hctx.gscale);
          const int sw = (hc >> 1) & 3;
          u32x4 ck[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            float o[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float v = dz * hctx.w[8 * k + e];
              o[e] = ((hbits[j] >> (8 * k + e)) & 1u) ? v : 0.f;
            }
            ck[k] = pack8(o);
          }
          // logical chunk k in store k: the 8 lanes of a store group hold 8 consecutive
          // slots whose swizzle sw = (column >> 1) & 3 takes each value twice (once per
          // slot parity), so the physical chunks k ^ sw land in 8 different 16-byte bank
          // groups (tools/lds_bank_model.py).  (Round 4 rotated the order by (slot >> 1) & 3
          // as the wgrad's head-on-load B does -- under THIS swizzle the rotation cancels
          // it, k + r ^ r, and every store was 4-way conflicted: 39.8 % conflict cycles.)
#pragma unroll
          for (int k = 0; k < 4; ++k) *(u32x4*)(Xs + sl * 64 + 16 * (k ^ sw)) = ck[k];
        }
      }
      __syncthreads();
      if constexpr (XF == 2) {
#pragma unroll
        for (int j = 0; j < XNJ; ++j) {
          int hr, hc, gr;
          bool ok;
          const int sl = xslot(j, hr, hc, gr, ok);
          if (!ok) continue;                              // padding stays the DMA's zeros
          char* a = Xs + sl * 64 + 16 * (xlc ^ ((hc >> 1) & 3));
          float v[8], zv[8];
          unpack8(*(const u32x4*)a, v);
          unpack8(zq[j], zv);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaf(za[e], v[e], fmaf(zb[e], zv[e], zc[e]));
          *(u32x4*)a = pack8(v);
        }
        __syncthreads();
      }
      if constexpr (XF == 1) {
        float xa[8], xb[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const size_t ci = xsample + cb + xlc * 8 + e;
          xa[e] = p.xa[ci];
          xb[e] = p.xb[ci];
        }
        // the source's dropout (xd_rate): norm.hip norm_apply's keep test and scale
        const bool xdrop = p.xd_rate > 0.f;
        const uint32_t xseed = xdrop ? (p.seed_ptr ? *p.seed_ptr : p.seed) : 0u;
        const float xinv = xdrop ? 1.f / (1.f - p.xd_rate) : 1.f;
        const uint32_t xthr = (uint32_t)(p.xd_rate * 4294967296.0);
#pragma unroll
        for (int j = 0; j < XNJ; ++j) {
          int hr, hc, gr;
          bool ok;
          const int sl = xslot(j, hr, hc, gr, ok);
          if (!ok) continue;                              // padding stays the DMA's zeros
          char* a = Xs + sl * 64 + 16 * (xlc ^ ((hc >> 1) & 3));
          float v[8];
          unpack8(*(const u32x4*)a, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(fmaf(xa[e], v[e], xb[e]), 0.f);
          if (xdrop) {
            const unsigned long long e0 = p.xd_idx0 + (unsigned long long)(gr * W + hc - 1) * C + cb + xlc * 8;
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = drop_hash(e0 + e, xseed, p.xd_salt) >= xthr ? v[e] * xinv : 0.f;
          }
          const u32x4 o = pack8(v);
          *(u32x4*)a = o;
          // the window's own rows (once: output-channel tile 0) -> xout
          if (p.xout && tn == 0 && hr >= 1 && hr <= R)
            *(u32x4*)((h16*)p.xout + (size_t)(gr * W + hc - 1) * C + cb + xlc * 8) = o;
        }
        __syncthreads();
      }
      chunk_mfmas(XF == 4 ? s2d_taps : 0x1ffu);
    }
  }
  __syncthreads();
  if constexpr (GEO == GEO_SEG)
    conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, W, W>(p, acc, smem, g0, n0, M, wave, 0, lane, tid, Wf,
                                                                 col0, tm);
  else if constexpr (GEO == GEO_2D)
    conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, 0, W>(p, acc, smem, g0 * W, n0, M, wave, 0, lane, tid, 0, 0,
                                                                  tm);
  else
    conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map>(p, acc, smem, g0 * W, n0, M, wave, 0, lane, tid, 0, 0, tm);
}

// ---------------------------------------------------------------------------------
// Persistent prefetching row window (win_pf_eligible): level 1 of the 128^2 UNet has one
// 32-channel input chunk per window, so conv_win_kernel's workgroup is a serial chain --
// DMA the 55 KB halo, wait, 144 MFMAs per wave, epilogue, exit -- and two workgroups per
// CU leave HBM idle for much of it (3.6 TB/s, 18 % MFMA busy on conv1b's forward, r5 PMC).
// Here a workgroup runs win_pf consecutive windows: the weights are staged once, and the
// next window's halo is loaded into registers (13 x 16 bytes per thread) while the
// current one's MFMAs and epilogue run, then written to LDS (XF 3, head-on-load: the
// next window's per-pixel probability, target and ReLU bits -- 12 registers -- and the
// halo is formed from them).  The epilogue's constants
// (bias, head weights) are loaded once too (EpiConst), so its only memory operations are
// stores and the prefetch is never waited on behind a load (the data-gradient epilogue's
// mask / pool-route loads still are).  Same operands, tap order and epilogue as
// conv_win_kernel<128, 32, 512, false, EPI, GEO_2D, XF>: bit-identical outputs.
constexpr int PF_HWP = 144;                   // halo row pitch in 64-byte slots (ALR's)
constexpr int PF_ROWB = PF_HWP * 64;
constexpr int PF_CPT = 6 * 128 * 4 / NTHR;    // 16-byte granules of the 6 halo rows' pixels per thread
constexpr int PF_XB = 6 * PF_ROWB, PF_WB = 9 * 32 * 64;
static_assert(512 * 36 * 2 <= PF_XB, "epilogue staging aliases the halo image");

// The workgroup's Mask weight sums (conv_params.h head_ws) -> one 100-float row: lanes l,
// l ^ 4, .. hold the same 8 channels (chunk tid & 3), folded in a fixed order, then the 4
// waves through LDS (smem: the epilogue's staging, free after a barrier)
__device__ __forceinline__ void head_ws_store(HeadWsum& hws, char* smem, const int wave, const int lane,
                                              const int tid, float* row) {
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) hws.s[k][e] += __shfl_xor(hws.s[k][e], o, 64);
  hws.u = wave_sum(hws.u);
  hws.v = wave_sum(hws.v);
  hws.w = wave_sum(hws.w);
  float* red = (float*)smem;                         // [wave][100]
  __syncthreads();                                   // the last epilogue's staging reads are done
  if (lane < 4) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wave * 100 + k * 32 + lane * 8 + e] = hws.s[k][e];
  }
  if (lane == 0) {
    red[wave * 100 + 96] = hws.u;
    red[wave * 100 + 97] = hws.v;
    red[wave * 100 + 98] = hws.w;
    red[wave * 100 + 99] = 0.f;
  }
  __syncthreads();
  if (tid < 100) row[tid] = (red[tid] + red[100 + tid]) + (red[200 + tid] + red[300 + tid]);
}

// GEO_SEG: rows of Wf = p.OW > 128 pixels as 128-wide segments (window = 4 rows x one
// segment, windows in (row group, segment) order as conv_win_kernel's); the halo columns
// -1 / 128 are the neighbouring segments' pixels (zeros only at the row ends), loaded by 48
// threads beside the affine part.
template <int EPI, int XF, int GEO = GEO_2D>
__global__ void __launch_bounds__(NTHR, 2) conv_win_pf_kernel(const ConvFwdParams p) {
  static_assert(XF == 0 || (XF == 3 && EPI == EPI_DGRAD && GEO == GEO_2D) || (XF == 1 && GEO == GEO_2D),
                "plain source, head-on-load data gradient or normalise on load");
  static_assert(GEO == GEO_2D || GEO == GEO_SEG, "2D rows");
  constexpr bool SEG = GEO == GEO_SEG;
  constexpr int W = 128, R = 4, BM = 512, BN = 32, ROWB = PF_ROWB;
  constexpr int TC = 2, NCS = 4, RW = 4, TM = RW * TC, TN = 2, WMP = BM / 4;
  using Map = StripTiles<W, RW, TC, NCS>;
  __shared__ __attribute__((aligned(1024))) char smem[PF_XB + PF_WB];
  char* Xs = smem;
  char* Ws = smem + PF_XB;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int Wf = SEG ? p.OW : W;
  const int nseg = SEG ? p.OW / W : 1;
  const int rows_total = p.N * H;
  const int M = rows_total * Wf;
  const int nwin = rows_total / R * nseg;            // H % R == 0 (win_pf_eligible)
  const int w_lo = (int)blockIdx.x * p.win_pf;
  const int w_hi = w_lo + p.win_pf < nwin ? w_lo + p.win_pf : nwin;
  if (w_lo >= w_hi) return;
  constexpr int OOB = 0x7fffffff;
  const char* src = (const char*)p.src1;

  // Halo pixels: granule c of thread t = halo row c / 2, column (t >> 2) + 64 (c & 1),
  // logical chunk t & 3 -- a 512-granule row is two 256-thread passes, so a thread's
  // global and LDS offsets are its own base plus compile-time constants and a row's
  // validity is wave-uniform.  LDS slot = column + 1, physical chunk = logical ^
  // ((slot >> 1) & 3), as conv_win_kernel's DMA leaves it; the zero columns -1 / 128
  // (slots 0 / 129) are rewritten per window (the epilogue's staging overwrites them).
  u32x4 hv[PF_CPT], ev = {0u, 0u, 0u, 0u};
  const int gl_t = tid * 16;
  const int lds_t = (1 + (tid >> 2)) * 64 + 16 * ((tid & 3) ^ (((1 + (tid >> 2)) >> 1) & 3));
  // XF 3: slot sl = tid + 256 j of the 6 x 144-slot image (conv_win_kernel's XF 3 map)
  constexpr int NSL = 6 * PF_HWP, HJ = (NSL + NTHR - 1) / NTHR;
  float hpr[HJ], htv[HJ];
  uint32_t hbits[HJ];
  HeadGradCtx hctx{};
  if constexpr (XF == 3) hctx = head_grad_ctx(p.hg);
  // XF 1 (normalise on load, conv_win_kernel's XF 1): y = relu(xa z + xb) with the thread's
  // 8 channels' coefficients of the prefetched window's sample, applied in registers before
  // the LDS store (padding rows stay zero); the window's own rows also go to xout
  float xan[8], xbn[8];
  int pf_g0 = 0;
  bool pf_top = false, pf_bot = false;
  // head_ws: the targets of the thread's 8 epilogue pixels (tid / 4 + 64 it) of the prefetched
  // window (conv_epilogue.h HeadWsum::t), loaded with its halo
  constexpr bool HWS = EPI == EPI_FWD && !SEG;
  float tnext[HWS ? 8 : 1];
  auto load_halo = [&](const int w) {
    const int tmw = p.rev ? nwin - 1 - w : w;
    const int g0 = (tmw / nseg) * R, col0 = (tmw % nseg) * W;
    if constexpr (HWS) {
      if (p.head_ws) {
#pragma unroll
        for (int it = 0; it < 8; ++it) tnext[it] = bits2f(((const uint16_t*)p.head_t)[g0 * W + (tid >> 2) + 64 * it]);
      }
    }
    if constexpr (XF == 3) {
      const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
#pragma unroll
      for (int j = 0; j < HJ; ++j) {
        const int sl = tid + NTHR * j;
        const int hr = sl / PF_HWP, hc = sl - hr * PF_HWP;
        const int gr = g0 - 1 + hr, col = hc - 1;
        const bool ok = sl < NSL && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                        (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
        const int pix = ok ? gr * W + col : 0;
        hpr[j] = p.hg.prob[pix];
        htv[j] = bits2f(((const uint16_t*)p.hg.t)[pix]);
        hbits[j] = ok ? ((const uint32_t*)p.hg.bits)[pix] : 0u;
      }
      return;
    }
    const int grow0 = (g0 / H) * H;                  // the window's image (32-bit offsets from it)
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    if constexpr (XF == 1) {
      const size_t cs = (size_t)(g0 / H) * p.xcs + (tid & 3) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xan[e] = p.xa[cs + e];
        xbn[e] = p.xb[cs + e];
      }
      pf_g0 = g0;
      pf_top = top_in;
      pf_bot = bot_in;
    }
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + (size_t)grow0 * Wf * 64), (short)0, OOB, 0x00020000);
    // byte offset of halo row 0's first pixel (negative at the image top: row 0 is then off)
    const int rowoff = ((g0 - 1 - grow0) * Wf + col0) * 64;
#pragma unroll
    for (int c = 0; c < PF_CPT; ++c) {
      const int hr = c >> 1;
      const bool ok = (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)(g0 - 1 + hr) < (unsigned)rows_total;
      hv[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? rowoff + hr * Wf * 64 + (c & 1) * 4096 + gl_t : OOB, 0, 0);
    }
    if constexpr (SEG) {
      // halo columns -1 / 128 of the segment: thread t < 48 -> row t / 8, side (t / 4) & 1, chunk t & 3
      const int hr = tid >> 3, col = ((tid >> 2) & 1) ? col0 + W : col0 - 1;
      const bool ok = tid < 48 && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                      (unsigned)(g0 - 1 + hr) < (unsigned)rows_total && (unsigned)col < (unsigned)Wf;
      ev = __builtin_amdgcn_raw_buffer_load_b128(
          rs, ok ? ((g0 - 1 + hr - grow0) * Wf + col) * 64 + (tid & 3) * 16 : OOB, 0, 0);
    }
  };
  auto store_halo = [&]() {
    if constexpr (XF == 3) {
      // dY = dlogit w (x > 0) per slot (zeros outside the image: bits 0), as conv_win_kernel
#pragma unroll
      for (int j = 0; j < HJ; ++j) {
        const int sl = tid + NTHR * j;
        if (sl >= NSL) continue;
        const int hc = sl % PF_HWP;
        const float dz = head_dlogit(hpr[j], htv[j], hctx.a, hctx.bb, hctx.inv_total, hctx.bce_w, hctx.gscale);
        const int sw = (hc >> 1) & 3;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          float o[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float v = dz * hctx.w[8 * k + e];
            o[e] = ((hbits[j] >> (8 * k + e)) & 1u) ? v : 0.f;
          }
          *(u32x4*)(Xs + sl * 64 + 16 * (k ^ sw)) = pack8(o);
        }
      }
      return;
    }
    if constexpr (XF == 1) {
#pragma unroll
      for (int c = 0; c < PF_CPT; ++c) {
        const int hr = c >> 1;
        const int gr = pf_g0 - 1 + hr;
        u32x4 v = hv[c];
        if ((hr > 0 || pf_top) && (hr < R + 1 || pf_bot) && (unsigned)gr < (unsigned)rows_total) {
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(xan[e], f[e], xbn[e]), 0.f);
          v = pack8(f);
          if (p.xout && hr >= 1 && hr <= R)
            *(u32x4*)((h16*)p.xout + ((size_t)gr * W + (tid >> 2) + 64 * (c & 1)) * 32 + (tid & 3) * 8) = v;
        }
        *(u32x4*)(Xs + lds_t + hr * ROWB + (c & 1) * 4096) = v;
      }
    } else {
#pragma unroll
      for (int c = 0; c < PF_CPT; ++c) *(u32x4*)(Xs + lds_t + (c >> 1) * ROWB + (c & 1) * 4096) = hv[c];
    }
    // (slot 0 / 129: chunk swizzle (slot >> 1) & 3 = 0 / 0)
    if (tid < 48) *(u32x4*)(Xs + (tid >> 3) * ROWB + ((tid >> 2) & 1) * 129 * 64 + 16 * (tid & 3)) = ev;
  };
  load_halo(w_lo);
  {
    // weight image (once): row tap * 32 + n, 64 bytes = the 32 input channels
    const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
    const int lslot = lane >> 2;
    const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
    const int wl = (lslot * p.Kpad + lchunk * 8) * 2;
    constexpr int WI = 9 * BN / 16;
#pragma unroll
    for (int q = 0; q < (WI + 3) / 4; ++q) {
      const int k = wave + 4 * q;
      if (k < WI) {
        const int tap = k / (BN / 16), nb = (k % (BN / 16)) * 16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024), 16,
                                                 (nb * p.Kpad + tap * 32) * 2 + wl, 0, 0, 0);
      }
    }
  }
  const int fsub = lane >> 4, fr = lane & 15;
  EpiConst<TN> ec;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      ec.bias[j][r] = (EPI != EPI_DGRAD && EPI != EPI_DGRAD_NORM && p.bias) ? p.bias[16 * j + 4 * fsub + r] : 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) ec.hw[e] = (EPI == EPI_FWD && p.head_w) ? p.head_w[(tid % 4) * 8 + e] : 0.f;
  ec.hb = (EPI == EPI_FWD && p.head_w) ? p.head_b[0] : 0.f;
  HeadWsum hws;                                      // the walk's Mask weight sums (head_ws)
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) hws.s[k][e] = 0.f;
  hws.u = hws.v = hws.w = 0.f;
  HeadT ht;                                          // the current window's targets
  ht.on = HWS && p.head_ws;
#pragma unroll
  for (int it = 0; it < 8; ++it) ht.t[it] = HWS ? tnext[it] : 0.f;
  store_halo();
  __syncthreads();

  const int r0 = (wave / NCS) * RW, c0 = (wave % NCS) * 16 * TC;
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = r0 * ROWB + c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  for (int w = w_lo; w < w_hi; ++w) {
    const int tm = p.rev ? nwin - 1 - w : w;
    const int g0 = (tm / nseg) * R, col0 = (tm % nseg) * W;
    if (w + 1 < w_hi) load_halo(w + 1);             // in flight under this window's MFMAs + epilogue
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      h16x8 wf[3][TN];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[dh][j] = *(const h16x8*)(Ws + ((3 * dh + dw) * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int hr = 0; hr < RW + 2; ++hr) {
#pragma unroll
        for (int ci = 0; ci < TC; ++ci) {
          const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * ROWB + ci * 16 * 64);
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int ri = hr - dh;
            if (ri < 0 || ri >= RW) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[ri * TC + ci][j] = mfma16(wf[dh][j], xf, acc[ri * TC + ci][j]);
          }
        }
      }
    }
    __syncthreads();                                 // fragment reads done: the epilogue stages in Xs
    if constexpr (SEG)
      conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, W, W>(p, acc, smem, g0, 0, M, wave, 0, lane, tid, Wf,
                                                                    col0, tm, &ec);
    else {
      const HeadWsum r = conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, 0, W>(
          p, acc, smem, g0 * W, 0, M, wave, 0, lane, tid, 0, 0, tm, &ec, ht);
      if constexpr (HWS) {
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int e = 0; e < 8; ++e) hws.s[k][e] += r.s[k][e];
        hws.u += r.u;
        hws.v += r.v;
        hws.w += r.w;
      }
    }
    if (w + 1 < w_hi) {
      __syncthreads();                               // staging reads done
      store_halo();
      if constexpr (HWS) {
#pragma unroll
        for (int it = 0; it < 8; ++it) ht.t[it] = tnext[it];
      }
      __syncthreads();
    }
  }
  if constexpr (EPI == EPI_FWD && !SEG) {
    if (p.head_ws) head_ws_store(hws, smem, wave, lane, tid, p.head_ws + (size_t)blockIdx.x * 100);
  }
}

// ---------------------------------------------------------------------------------
// Chunk-pipelined row window (win_cp_eligible): at levels 2-4 a window runs 2..16 input
// chunks, and conv_win_kernel's chunk step is serial -- LDS-DMA the chunk's halo image and
// 36 KB of weights, wait, MFMAs -- with two workgroups per CU to cover one's wait with the
// other's MFMAs (27-49 % MFMA busy, r5 PMC).  Here the next chunk's halo and weight images
// are loaded into registers (6-7 + 9 x 16 bytes per thread) while the current chunk's MFMAs
// run, and written to LDS after them: one barrier pair per chunk, no exposed load latency
// past the first chunk.  Same LDS images (pitch W + 4, chunk swizzle), operands, tap order
// and epilogue as conv_win_kernel<W, 64, 256, CONCAT, EPI, GEO_2D>: bit-identical outputs.
// DZ (xform 2, conv_win_kernel's XF 2): src1 = g; the z granules ride along with the g
// granules and each halo granule is stored as dz = ca g + cb z + cc, the window sample's
// coefficients of every input channel held in LDS (Ks, past the images).
template <int W, bool CONCAT, int EPI, bool DZ = false>
__global__ void __launch_bounds__(NTHR, 2) conv_win_cp_kernel(const ConvFwdParams p) {
  constexpr int BN = 64, BM = 256, R = BM / W, HR = R + 2;
  constexpr int HWP = W + 4, ROWB = HWP * 64;
  constexpr int NSLOT = HR * HWP;
  constexpr int XB = (NSLOT + 15) / 16 * 1024, WB = 9 * BN * 64;
  constexpr int XG = (NSLOT * 4 + NTHR - 1) / NTHR;     // halo granules per thread
  constexpr int WG = 9 * BN * 4 / NTHR;                 // weight granules per thread (9)
  constexpr int EPIB = (EPI == EPI_STATS || EPI == EPI_DGRAD_NORM) ? epi_lds_bytes<BM, BN>() : BM * (BN + 4) * 2;
  constexpr int KB = DZ ? 3 * CP_DZ_MAXC * 4 : 0;       // DZ coefficients (Cin <= CP_DZ_MAXC)
  constexpr int LDS_BYTES = (XB + WB + KB > EPIB) ? XB + WB + KB : EPIB;
  constexpr int WMP = BM / 4, TM = WMP / 16, TN = BN / 16;
  constexpr int TC = 1, NCS = W / 16, RW = R / (4 / NCS);
  static_assert(W >= 16 && W <= 64 && RW * TC == TM && 9 * BN * 4 % NTHR == 0, "chunk-pipelined window shape");
  using Map = StripTiles<W, RW, TC, NCS>;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  char* Xs = smem;
  char* Ws = smem + XB;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int rows_total = p.N * H;
  const int M = rows_total * W;
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm0 = bid / tiles_n, tn = bid % tiles_n;
  const int tm = p.rev ? (int)(gridDim.x / tiles_n) - 1 - tm0 : tm0;
  const int g0 = tm * R, n0 = tn * BN;
  const int Cin = p.C1 + p.C2;
  const int nchunks = Cin >> 5;
  constexpr int OOB = 0x7fffffff;
  const int grow0 = (g0 / H) * H;                       // the window's image (32-bit offsets from it)
  const size_t img_px = (size_t)grow0 * W;
  const char* s1b = (const char*)p.src1 + img_px * p.C1 * 2;
  const char* s2b = p.src2 ? (const char*)p.src2 + img_px * p.C2 * 2 : s1b;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)s1b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)s2b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
  const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
  float* Ks = (float*)(smem + XB + WB);
  const __amdgpu_buffer_rsrc_t rsz = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(DZ ? (const char*)p.xz + img_px * p.C1 * 2 : s1b), (short)0, OOB, 0x00020000);
  if constexpr (DZ) {
    // ca / cb / cc of the window's sample (GroupNorm: xcs = C1), every input channel
    const size_t xs = (size_t)(g0 / H) * p.xcs;
    for (int i = tid; i < 3 * Cin; i += NTHR) {
      const int m = i / Cin, c = i - m * Cin;
      Ks[i] = (m == 0 ? p.xa : m == 1 ? p.xb : p.xc)[xs + c];
    }
  }

  // halo granule u = tid + 256 c: slot u / 4 (row slot / HWP, column slot % HWP - 1), logical
  // chunk u % 4 at physical chunk ^ ((column slot >> 1) & 3); weight granule u: row u / 4 =
  // tap c x BN + n (n = tid / 4), logical chunk u % 4 at ^ ((row >> 1) & 3)
  u32x4 xv[XG], wv[WG];
  u32x4 zq[DZ ? XG : 1];
  uint32_t okm = 0;                                     // DZ: granules of real pixels
  auto load_chunk = [&](const int kc) {
    const bool from1 = !CONCAT || (kc << 5) < p.C1;
    const int C = from1 ? p.C1 : p.C2;
    const int cb = from1 ? (kc << 5) : (kc << 5) - p.C1;
    const __amdgpu_buffer_rsrc_t rs = from1 ? rs1 : rs2;
#pragma unroll
    for (int c = 0; c < XG; ++c) {
      const int u = tid + NTHR * c;
      const int sl = u >> 2, hr = sl / HWP, hc = sl - hr * HWP;
      const int gr = g0 - 1 + hr, col = hc - 1;
      const bool ok = sl < NSLOT && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                      (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
      xv[c] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, ok ? (((gr - grow0) * W + col) * C + cb + (u & 3) * 8) * 2 : OOB, 0, 0);
      if constexpr (DZ) {
        zq[c] = __builtin_amdgcn_raw_buffer_load_b128(
            rsz, ok ? (((gr - grow0) * W + col) * C + cb + (u & 3) * 8) * 2 : OOB, 0, 0);
        okm = c ? (okm | ((ok ? 1u : 0u) << c)) : (ok ? 1u : 0u);
      }
    }
#pragma unroll
    for (int c = 0; c < WG; ++c)
      wv[c] = __builtin_amdgcn_raw_buffer_load_b128(
          rsw, ((n0 + (tid >> 2)) * p.Kpad + c * Cin + (kc << 5) + (tid & 3) * 8) * 2, 0, 0);
  };
  auto store_chunk = [&](const int kc) {
    if constexpr (DZ) {
      // dz = ca g + (cb z + cc) of the thread's 8 channels (kc 32 + (tid & 3) 8 ..)
      const float* kb = Ks + (kc << 5) + (tid & 3) * 8;
      float ka[8], kz[8], kk[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ka[e] = kb[e];
        kz[e] = kb[Cin + e];
        kk[e] = kb[2 * Cin + e];
      }
#pragma unroll
      for (int c = 0; c < XG; ++c) {
        if (!((okm >> c) & 1u)) continue;               // padding stays zero
        float gv[8], zv[8];
        unpack8(xv[c], gv);
        unpack8(zq[c], zv);
#pragma unroll
        for (int e = 0; e < 8; ++e) gv[e] = fmaf(ka[e], gv[e], fmaf(kz[e], zv[e], kk[e]));
        xv[c] = pack8(gv);
      }
    }
#pragma unroll
    for (int c = 0; c < XG; ++c) {
      const int u = tid + NTHR * c;
      const int sl = u >> 2, hc = sl % HWP;
      if (sl < NSLOT) *(u32x4*)(Xs + sl * 64 + 16 * ((u & 3) ^ ((hc >> 1) & 3))) = xv[c];
    }
    const int wrow = tid >> 2;
#pragma unroll
    for (int c = 0; c < WG; ++c)
      *(u32x4*)(Ws + (c * BN + wrow) * 64 + 16 * ((tid & 3) ^ ((wrow >> 1) & 3))) = wv[c];
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fsub = lane >> 4, fr = lane & 15;
  const int r0 = (wave / NCS) * RW, c0 = (wave % NCS) * 16 * TC;
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = r0 * ROWB + c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  load_chunk(0);
  if constexpr (DZ) __syncthreads();                    // Ks written
  store_chunk(0);
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    if (kc + 1 < nchunks) load_chunk(kc + 1);          // in flight under this chunk's MFMAs
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
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
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[ri][j] = mfma16(wf[dh][j], xf, acc[ri][j]);
        }
      }
    }
    __syncthreads();                                    // fragment reads done
    if (kc + 1 < nchunks) {
      store_chunk(kc + 1);
      __syncthreads();
    }
  }
  conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, 0, W>(p, acc, smem, g0 * W, n0, M, wave, 0, lane, tid, 0, 0,
                                                                tm);
}

template <int W>
hipError_t launch_win_cp_w(const ConvFwdParams& p, hipStream_t s) {
  const int grid = win_grid(p);
  const bool cc = p.C2 > 0;
  if (p.xform == 2) {                                   // dz on load (win_cp_eligible: single source)
    if (cc || p.C1 > CP_DZ_MAXC) return hipErrorInvalidValue;
    if (conv_epi_mode(p) == EPI_DGRAD_NORM)
      UNET_LAUNCH((conv_win_cp_kernel<W, false, EPI_DGRAD_NORM, true>), dim3(grid), dim3(NTHR), 0, s, p);
    else if (conv_epi_mode(p) == EPI_DGRAD)
      UNET_LAUNCH((conv_win_cp_kernel<W, false, EPI_DGRAD, true>), dim3(grid), dim3(NTHR), 0, s, p);
    else
      return hipErrorInvalidValue;
    return launch_status();
  }
#define CP_EPI(CC)                                                                                           \
  switch (conv_epi_mode(p)) {                                                                                \
    case EPI_FWD: UNET_LAUNCH((conv_win_cp_kernel<W, CC, EPI_FWD>), dim3(grid), dim3(NTHR), 0, s, p); break;     \
    case EPI_DGRAD: UNET_LAUNCH((conv_win_cp_kernel<W, CC, EPI_DGRAD>), dim3(grid), dim3(NTHR), 0, s, p); break; \
    case EPI_STATS: UNET_LAUNCH((conv_win_cp_kernel<W, CC, EPI_STATS>), dim3(grid), dim3(NTHR), 0, s, p); break; \
    case EPI_DGRAD_NORM:                                                                                     \
      if (CC) return hipErrorInvalidValue;                                                                   \
      UNET_LAUNCH((conv_win_cp_kernel<W, false, EPI_DGRAD_NORM>), dim3(grid), dim3(NTHR), 0, s, p);          \
      break;                                                                                                 \
    default: UNET_LAUNCH((conv_win_cp_kernel<W, CC, EPI_GENERIC>), dim3(grid), dim3(NTHR), 0, s, p); break;     \
  }
  if (cc) {
    CP_EPI(true)
  } else {
    CP_EPI(false)
  }
#undef CP_EPI
  return launch_status();
}

hipError_t launch_win_cp(const ConvFwdParams& p, hipStream_t s) {
  return p.OW == 64 ? launch_win_cp_w<64>(p, s) : hipErrorInvalidValue;
}

// Chunk-pipelined window on 128-wide rows (win_cp128_eligible): items = (depth tap, input
// chunk) pairs; the next item's halo (12 x 16 bytes per thread, conv_win_pf_kernel's affine
// map, the depth-shifted slice in 3D) and weight rows (5 x 16 bytes) are loaded into
// registers under the current item's MFMAs.  Same images, operands, order and epilogue as
// conv_win_kernel<128, 32, 512, CONCAT, EPI, GEO>: bit-identical outputs.
template <int GEO, bool CONCAT, int EPI>
__global__ void __launch_bounds__(NTHR, 2) conv_win_cp128_kernel(const ConvFwdParams p) {
  constexpr int W = 128, R = 4, BM = 512, BN = 32, ROWB = PF_ROWB;
  constexpr int TC = 2, NCS = 4, RW = 4, TM = RW * TC, TN = 2, WMP = BM / 4;
  constexpr int NWG = 9 * BN * 4, WGR = (NWG + NTHR - 1) / NTHR;
  constexpr bool D3 = GEO == GEO_3D;
  using Map = StripTiles<W, RW, TC, NCS>;
  static_assert(epi_lds_bytes<BM, BN>() <= PF_XB, "epilogue staging aliases the halo image");
  __shared__ __attribute__((aligned(1024))) char smem[PF_XB + PF_WB];
  char* Xs = smem;
  char* Ws = smem + PF_XB;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int D = D3 ? p.OD : 1;
  const int rows_total = p.N * D * H;
  const int M = rows_total * W;
  const int tiles_n = p.Cout / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tm0 = bid / tiles_n, tn = bid % tiles_n;
  const int tm = p.rev ? (int)(gridDim.x / tiles_n) - 1 - tm0 : tm0;
  const int g0 = tm * R, n0 = tn * BN;
  const int dsl = D3 ? (g0 / H) % D : 0;
  const int Cin = p.C1 + p.C2;
  const int nchunks = Cin >> 5;
  constexpr int OOB = 0x7fffffff;
  const int grow0 = (g0 / (D * H)) * (D * H);          // the window's image / volume
  const size_t img_px = (size_t)grow0 * W;
  const char* s1b = (const char*)p.src1 + img_px * p.C1 * 2;
  const char* s2b = p.src2 ? (const char*)p.src2 + img_px * p.C2 * 2 : s1b;
  const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc((void*)s1b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs2 = __builtin_amdgcn_make_buffer_rsrc((void*)s2b, (short)0, OOB, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
  const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
  // depth taps whose input slice is padding contribute nothing: skipped
  const int kd_lo = (D3 && dsl == 0) ? 1 : 0, kd_hi = D3 ? (dsl == D - 1 ? 2 : 3) : 1;
  const int nitems = (kd_hi - kd_lo) * nchunks;

  u32x4 xv[12], wv[WGR];
  const int lds_t = (1 + (tid >> 2)) * 64 + 16 * ((tid & 3) ^ (((1 + (tid >> 2)) >> 1) & 3));
  auto load_item = [&](const int it) {
    const int kd = kd_lo + it / nchunks, kc = it - (it / nchunks) * nchunks;
    const bool from1 = !CONCAT || (kc << 5) < p.C1;
    const int C = from1 ? p.C1 : p.C2;
    const int cb = from1 ? (kc << 5) : (kc << 5) - p.C1;
    const __amdgpu_buffer_rsrc_t rs = from1 ? rs1 : rs2;
    const int shift = D3 ? (kd - 1) * H : 0;
    const int tb = ((tid >> 2) * C + cb + (tid & 3) * 8) * 2;   // the thread's column / chunk part
#pragma unroll
    for (int c = 0; c < 12; ++c) {
      const int hr = c >> 1;
      const int gr = g0 - 1 + hr;
      const bool ok = (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)gr < (unsigned)rows_total &&
                      (unsigned)(gr + shift) < (unsigned)rows_total;
      xv[c] = __builtin_amdgcn_raw_buffer_load_b128(
          rs, ok ? ((gr + shift - grow0) * W + 64 * (c & 1)) * C * 2 + tb : OOB, 0, 0);
    }
#pragma unroll
    for (int c = 0; c < WGR; ++c) {
      const int u = tid + NTHR * c;
      const int row = u >> 2, tap = row / BN, n = row - tap * BN;
      wv[c] = __builtin_amdgcn_raw_buffer_load_b128(
          rsw, u < NWG ? ((n0 + n) * p.Kpad + (kd * 9 + tap) * Cin + (kc << 5) + (tid & 3) * 8) * 2 : OOB, 0, 0);
    }
  };
  auto store_item = [&]() {
#pragma unroll
    for (int c = 0; c < 12; ++c) *(u32x4*)(Xs + lds_t + (c >> 1) * ROWB + (c & 1) * 4096) = xv[c];
    if (tid < 48) *(u32x4*)(Xs + (tid >> 3) * ROWB + ((tid >> 2) & 1) * 129 * 64 + 16 * (tid & 3)) = (u32x4){0u, 0u, 0u, 0u};
#pragma unroll
    for (int c = 0; c < WGR; ++c) {
      const int u = tid + NTHR * c;
      const int row = u >> 2;
      if (u < NWG) *(u32x4*)(Ws + row * 64 + 16 * ((tid & 3) ^ ((row >> 1) & 3))) = wv[c];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fsub = lane >> 4, fr = lane & 15;
  const int r0 = (wave / NCS) * RW, c0 = (wave % NCS) * 16 * TC;
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = r0 * ROWB + c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  load_item(0);
  // head_ws (fused head): the targets of the thread's 8 epilogue pixels (tid / 4 + 64 it),
  // loaded behind item 0's halo (whose wait they share)
  HeadT ht;
  ht.on = EPI == EPI_FWD && p.head_ws;
#pragma unroll
  for (int i = 0; i < 8; ++i) ht.t[i] = 0.f;
  if (EPI == EPI_FWD && p.head_ws) {
    // one block of 8 loads (a per-element select became 8 branches, each waiting on its load)
    const uint16_t* tp = (const uint16_t*)p.head_t + g0 * W + (tid >> 2);
    uint16_t tv[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) tv[i] = tp[64 * i];
#pragma unroll
    for (int i = 0; i < 8; ++i) ht.t[i] = bits2f(tv[i]);
  }
  store_item();
  __syncthreads();
  if constexpr (EPI == EPI_FWD) {
    // the targets are complete here (item 0's halo wait covers them): keep the loads from
    // being scheduled into the epilogue, where their round trip would be exposed
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("" : : "v"(ht.t[i]));
  }
  for (int it = 0; it < nitems; ++it) {
    if (it + 1 < nitems) load_item(it + 1);            // in flight under this item's MFMAs
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      h16x8 wf[3][TN];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[dh][j] = *(const h16x8*)(Ws + ((3 * dh + dw) * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int hr = 0; hr < RW + 2; ++hr) {
#pragma unroll
        for (int ci = 0; ci < TC; ++ci) {
          const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * ROWB + ci * 16 * 64);
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int ri = hr - dh;
            if (ri < 0 || ri >= RW) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[ri * TC + ci][j] = mfma16(wf[dh][j], xf, acc[ri * TC + ci][j]);
          }
        }
      }
    }
    __syncthreads();                                    // fragment reads done
    if (it + 1 < nitems) {
      store_item();
      __syncthreads();
    }
  }
  if constexpr (D3) {
    HeadWsum hws = conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map>(p, acc, smem, g0 * W, n0, M, wave, 0, lane,
                                                                          tid, 0, 0, tm, nullptr, ht);
    if constexpr (EPI == EPI_FWD) {
      if (p.head_ws) head_ws_store(hws, smem, wave, lane, tid, p.head_ws + (size_t)blockIdx.x * 100);
    }
  } else
    conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, 0, W>(p, acc, smem, g0 * W, n0, M, wave, 0, lane, tid, 0, 0,
                                                                  tm);
}

template <int GEO>
hipError_t launch_win_cp128_g(const ConvFwdParams& p, hipStream_t s) {
  const int grid = win_grid(p);
  const bool cc = p.C2 > 0;
#define CP1_EPI(CC)                                                                                                \
  switch (conv_epi_mode(p)) {                                                                                     \
    case EPI_FWD: UNET_LAUNCH((conv_win_cp128_kernel<GEO, CC, EPI_FWD>), dim3(grid), dim3(NTHR), 0, s, p); break;     \
    case EPI_DGRAD: UNET_LAUNCH((conv_win_cp128_kernel<GEO, CC, EPI_DGRAD>), dim3(grid), dim3(NTHR), 0, s, p); break; \
    case EPI_STATS: UNET_LAUNCH((conv_win_cp128_kernel<GEO, CC, EPI_STATS>), dim3(grid), dim3(NTHR), 0, s, p); break; \
    case EPI_DGRAD_NORM:                                                                                          \
      if (CC) return hipErrorInvalidValue;                                                                        \
      UNET_LAUNCH((conv_win_cp128_kernel<GEO, false, EPI_DGRAD_NORM>), dim3(grid), dim3(NTHR), 0, s, p);          \
      break;                                                                                                      \
    default: UNET_LAUNCH((conv_win_cp128_kernel<GEO, CC, EPI_GENERIC>), dim3(grid), dim3(NTHR), 0, s, p); break;     \
  }
  if (cc) {
    CP1_EPI(true)
  } else {
    CP1_EPI(false)
  }
#undef CP1_EPI
  return launch_status();
}

hipError_t launch_win_cp128(const ConvFwdParams& p, hipStream_t s) {
  return (p.KD == 3) ? launch_win_cp128_g<GEO_3D>(p, s) : launch_win_cp128_g<GEO_2D>(p, s);
}

// ---------------------------------------------------------------------------------
// Persistent prefetching tconv-on-load window (win_pfu_eligible; conv9a's forward).  The
// one-window XF 5 kernel is a serial chain per 512-pixel window -- coarse rows and tconv
// weights from memory, u MFMAs, LDS stores, u-chunk MFMAs, skip-chunk DMA, wait, MFMAs,
// epilogue -- at ~18 us per window for ~2.3 us of MFMA (r5 PMC: 25 % MFMA busy).  Here a
// workgroup walks win_pf consecutive 256-pixel windows (R = 2: a 4-row halo, 37 KB, beside
// both chunks' weights, 37 KB, staged once): wave w forms halo row w from coarse row
// g0 / 2 - 1 + (w + 1) / 2 with tap row (w + 1) & 1, whose tconv weight rows it holds in
// registers for the whole walk; the next window's coarse row (8 x 16 bytes per lane) is loaded
// under this window's u-chunk MFMAs, its skip halo (8 x 16 bytes per thread, the affine map
// of conv_win_pf_kernel) under the skip-chunk MFMAs and epilogue.  Same operands and
// accumulation order as conv_win_kernel's XF 5 (u bit-identical to tconv_fwd_kernel's),
// same epilogue: bit-identical outputs.
template <int KS, int EPI>
__global__ void __launch_bounds__(NTHR, 2) conv_win_pfu_kernel(const ConvFwdParams p) {
  static_assert(EPI == EPI_FWD || EPI == EPI_STATS, "persistent tconv-on-load epilogues");
  constexpr int W = 128, R = 2, HR = R + 2, BM = 256, BN = 32, ROWB = PF_ROWB;
  constexpr int TC = 2, NCS = 4, RW = 2, TM = RW * TC, TN = 2, WMP = BM / 4;
  constexpr int CW = W / 2, PB = CW / 16, Cc = KS * 32;
  constexpr int XB = HR * ROWB, WB = 9 * BN * 64;
  static_assert(BM * 64 + 4 * 2 * BN * 4 <= XB, "epilogue staging aliases the halo image");
  using Map = StripTiles<W, RW, TC, NCS>;
  __shared__ __attribute__((aligned(1024))) char smem[XB + 2 * WB];
  char* Xs = smem;
  char* Wu = smem + XB;                       // u-chunk weights
  char* Wk = smem + XB + WB;                  // skip-chunk weights
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fsub = lane >> 4, fr = lane & 15;
  const int H = p.OH;
  const int rows_total = p.N * H;
  const int M = rows_total * W;
  const int nwin = rows_total / R;
  const int w_lo = (int)blockIdx.x * p.win_pf;
  const int w_hi = w_lo + p.win_pf < nwin ? w_lo + p.win_pf : nwin;
  if (w_lo >= w_hi) return;
  constexpr int OOB = 0x7fffffff;

  // ---- once: both chunks' weight images (row tap * 32 + n: the chunk's 32 input channels)
  {
    const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
    const int lslot = lane >> 2;
    const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
    constexpr int WI = 9 * BN / 16;
#pragma unroll
    for (int q = 0; q < (2 * WI + 3) / 4; ++q) {
      const int k = wave + 4 * q;
      if (k < 2 * WI) {
        const int kc = k / WI, kk = k - kc * WI;
        const int tap = kk / (BN / 16), nb = (kk % (BN / 16)) * 16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rsw, (__attribute__((address_space(3))) void*)((kc ? Wk : Wu) + kk * 1024), 16,
            ((nb + lslot) * p.Kpad + tap * 64 + (kc << 5) + lchunk * 8) * 2, 0, 0, 0);
      }
    }
  }
  // ---- this wave's halo row: tap row th of coarse row offset cq (u = tconv weights x coarse x + b)
  const int cq = (wave + 1) >> 1, th = (wave + 1) & 1;
  h16x8 wa[2][2][KS];                          // [tw][j][ks]: both column phases of tap row th
  {
    const h16* wt = (const h16*)p.ut.w + (size_t)(8 * (fr >> 2) + (fr & 3)) * p.ut.kpad + 8 * fsub;
#pragma unroll
    for (int tw = 0; tw < 2; ++tw)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
          wa[tw][j][ks] = *(const h16x8*)(wt + (size_t)((2 * th + tw) * 32 + 4 * j) * p.ut.kpad + 32 * ks);
  }
  float bs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) bs[i] = p.ut.b[8 * fsub + i];
  EpiConst<TN> ec;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) ec.bias[j][r] = p.bias ? p.bias[16 * j + 4 * fsub + r] : 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) ec.hw[e] = 0.f;
  ec.hb = 0.f;

  h16x8 xb[PB][KS];                            // the wave's coarse row (16 px x 32 ch per fragment)
  bool xin = false;                            // (of the window the registers hold)
  auto load_coarse = [&](const int w) {
    const int g0 = (p.rev ? nwin - 1 - w : w) * R;
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const int hr = wave;                       // halo row = fine row g0 - 1 + hr
    xin = (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)(g0 - 1 + hr) < (unsigned)rows_total;
    const int crow = (g0 >> 1) - 1 + cq;       // coarse row (H even: fine row g -> g / 2)
    const h16* rp = (const h16*)p.ut.x + ((size_t)(xin ? crow : 0) * CW + fr) * Cc + 8 * fsub;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb)
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) xb[pb][ks] = *(const h16x8*)(rp + (size_t)(16 * pb) * Cc + 32 * ks);
  };
  // skip halo: granule c of thread t = halo row c / 2, column (t >> 2) + 64 (c & 1), chunk t & 3
  // (x2a: normalised on load, relu(x2a z + x2b) of the thread's 8 channels (t & 3) * 8 .. of the
  // window's sample; padding granules -- sok bit clear -- stay zero)
  u32x4 sv[8];
  uint32_t sok = 0;
  float s2a[8], s2b[8];
  const int lds_t = (1 + (tid >> 2)) * 64 + 16 * ((tid & 3) ^ (((1 + (tid >> 2)) >> 1) & 3));
  auto load_skip = [&](const int w) {
    const int g0 = (p.rev ? nwin - 1 - w : w) * R;
    const int grow0 = (g0 / H) * H;
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)((const char*)p.src2 + (size_t)grow0 * W * 64), (short)0, OOB, 0x00020000);
    const int rowoff = (g0 - 1 - grow0) * W * 64;
    sok = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const int hr = c >> 1;
      const bool ok = (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)(g0 - 1 + hr) < (unsigned)rows_total;
      sok |= (ok ? 1u : 0u) << c;
      sv[c] = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? rowoff + hr * W * 64 + (c & 1) * 4096 + tid * 16 : OOB, 0, 0);
    }
    if (p.x2a) {
      const size_t cs = (size_t)(g0 / H) * p.x2cs + (tid & 3) * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s2a[e] = p.x2a[cs + e];
        s2b[e] = p.x2b[cs + e];
      }
    }
  };
  const int tsel = (fr >> 2) & 1;
  auto form_u = [&]() {                        // halo row `wave` of u, zero columns included
    char* xrow = Xs + wave * ROWB;
#pragma unroll
    for (int pb = 0; pb < PB; ++pb) {
      u32x4 pk[2] = {(u32x4){0u, 0u, 0u, 0u}, (u32x4){0u, 0u, 0u, 0u}};
      if (xin) {
#pragma unroll
        for (int tw = 0; tw < 2; ++tw)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            f32x4 a = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) a = mfma16(wa[tw][j][ks], xb[pb][ks], a);
            pk[tw][2 * j] = pack2h(a[0] + bs[4 * j], a[1] + bs[4 * j + 1]);
            pk[tw][2 * j + 1] = pack2h(a[2] + bs[4 * j + 2], a[3] + bs[4 * j + 3]);
          }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int tw = s ^ tsel;
        const int hc = 2 * (16 * pb + fr) + tw + 1;
        *(u32x4*)(xrow + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3))) = tw ? pk[1] : pk[0];
      }
    }
    if (lane < 8) *(u32x4*)(xrow + ((lane >> 2) ? W + 1 : 0) * 64 + 16 * (lane & 3)) = (u32x4){0u, 0u, 0u, 0u};
  };
  auto store_skip = [&]() {
    if (p.x2a) {
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        if (!((sok >> c) & 1u)) continue;
        float f[8];
        unpack8(sv[c], f);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(s2a[e], f[e], s2b[e]), 0.f);
        sv[c] = pack8(f);
      }
    }
#pragma unroll
    for (int c = 0; c < 8; ++c) *(u32x4*)(Xs + lds_t + (c >> 1) * ROWB + (c & 1) * 4096) = sv[c];
    if (tid < 32) *(u32x4*)(Xs + (tid >> 3) * ROWB + ((tid >> 2) & 1) * 129 * 64 + 16 * (tid & 3)) = (u32x4){0u, 0u, 0u, 0u};
  };

  const int r0 = (wave / NCS) * RW, c0 = (wave % NCS) * 16 * TC;
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = r0 * ROWB + c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));
  f32x4 acc[TM][TN];
  auto chunk_mfmas = [&](const char* Ws) {
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
      h16x8 wf[3][TN];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int j = 0; j < TN; ++j) wf[dh][j] = *(const h16x8*)(Ws + ((3 * dh + dw) * BN + 16 * j) * 64 + wbase);
#pragma unroll
      for (int hr = 0; hr < RW + 2; ++hr) {
#pragma unroll
        for (int ci = 0; ci < TC; ++ci) {
          const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * ROWB + ci * 16 * 64);
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int ri = hr - dh;
            if (ri < 0 || ri >= RW) continue;
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[ri * TC + ci][j] = mfma16(wf[dh][j], xf, acc[ri * TC + ci][j]);
          }
        }
      }
    }
  };
  load_coarse(w_lo);
  load_skip(w_lo);
  for (int w = w_lo; w < w_hi; ++w) {
    const int tm = p.rev ? nwin - 1 - w : w;
    const int g0 = tm * R;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    form_u();
    if (w + 1 < w_hi) load_coarse(w + 1);          // under the u-chunk MFMAs and the rest
    __syncthreads();                               // u halo (and, first time, the weights) in LDS
    chunk_mfmas(Wu);
    __syncthreads();
    store_skip();
    if (w + 1 < w_hi) load_skip(w + 1);            // under the skip-chunk MFMAs and the epilogue
    __syncthreads();
    chunk_mfmas(Wk);
    __syncthreads();                               // fragment reads done: the epilogue stages in Xs
    conv_epilogue<BM, BN, WMP, BN, TM, TN, NTHR, EPI, Map, 0, W>(p, acc, smem, g0 * W, 0, M, wave, 0, lane, tid, 0, 0,
                                                                  tm, &ec);
    __syncthreads();                               // staging reads done before the next u rows
  }
}

hipError_t launch_win_pfu(const ConvFwdParams& p, hipStream_t s) {
  const int grid = win_grid(p);
  const bool st = conv_epi_mode(p) == EPI_STATS;
  if (p.ut.C == 64 && st)
    UNET_LAUNCH((conv_win_pfu_kernel<2, EPI_STATS>), dim3(grid), dim3(NTHR), 0, s, p);
  else if (p.ut.C == 64)
    UNET_LAUNCH((conv_win_pfu_kernel<2, EPI_FWD>), dim3(grid), dim3(NTHR), 0, s, p);
  else if (st)
    UNET_LAUNCH((conv_win_pfu_kernel<1, EPI_STATS>), dim3(grid), dim3(NTHR), 0, s, p);
  else
    UNET_LAUNCH((conv_win_pfu_kernel<1, EPI_FWD>), dim3(grid), dim3(NTHR), 0, s, p);
  return launch_status();
}

hipError_t launch_win_pf(const ConvFwdParams& p, hipStream_t s) {
  const int grid = win_grid(p);
  if (p.OW > 128) {
    switch (conv_epi_mode(p)) {
      case EPI_FWD: UNET_LAUNCH((conv_win_pf_kernel<EPI_FWD, 0, GEO_SEG>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case EPI_DGRAD: UNET_LAUNCH((conv_win_pf_kernel<EPI_DGRAD, 0, GEO_SEG>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case EPI_STATS: UNET_LAUNCH((conv_win_pf_kernel<EPI_STATS, 0, GEO_SEG>), dim3(grid), dim3(NTHR), 0, s, p); break;
      case EPI_DGRAD_NORM:
        UNET_LAUNCH((conv_win_pf_kernel<EPI_DGRAD_NORM, 0, GEO_SEG>), dim3(grid), dim3(NTHR), 0, s, p);
        break;
      default: UNET_LAUNCH((conv_win_pf_kernel<EPI_GENERIC, 0, GEO_SEG>), dim3(grid), dim3(NTHR), 0, s, p); break;
    }
    return launch_status();
  }
  if (p.xform) {                        // normalise on load (conv_fwd_prepare: statistics / generic epilogue)
    if (conv_epi_mode(p) == EPI_STATS)
      UNET_LAUNCH((conv_win_pf_kernel<EPI_STATS, 1>), dim3(grid), dim3(NTHR), 0, s, p);
    else if (conv_epi_mode(p) == EPI_GENERIC)
      UNET_LAUNCH((conv_win_pf_kernel<EPI_GENERIC, 1>), dim3(grid), dim3(NTHR), 0, s, p);
    else
      return hipErrorInvalidValue;
    return launch_status();
  }
  switch (conv_epi_mode(p)) {
    case EPI_FWD: UNET_LAUNCH((conv_win_pf_kernel<EPI_FWD, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case EPI_DGRAD:
      if (p.hg.prob)
        UNET_LAUNCH((conv_win_pf_kernel<EPI_DGRAD, 3>), dim3(grid), dim3(NTHR), 0, s, p);
      else
        UNET_LAUNCH((conv_win_pf_kernel<EPI_DGRAD, 0>), dim3(grid), dim3(NTHR), 0, s, p);
      break;
    case EPI_STATS: UNET_LAUNCH((conv_win_pf_kernel<EPI_STATS, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    case EPI_DGRAD_NORM: UNET_LAUNCH((conv_win_pf_kernel<EPI_DGRAD_NORM, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
    default: UNET_LAUNCH((conv_win_pf_kernel<EPI_GENERIC, 0>), dim3(grid), dim3(NTHR), 0, s, p); break;
  }
  return launch_status();
}

}  // namespace

template <int BN, int BM>
hipError_t launch_win(const ConvFwdParams& p, hipStream_t s) {
  if constexpr (BN == 32 && BM == 512) {
    if (win_pf_eligible(p)) return launch_win_pf(p, s);
    if (win_pfu_eligible(p)) return launch_win_pfu(p, s);
    if (win_cp128_eligible(p)) return launch_win_cp128(p, s);
  }
  if constexpr (BN == 64 && BM == 256) {
    if (win_cp_eligible(p)) return launch_win_cp(p, s);
  }
  const int W = p.OW > 128 ? 128 : p.OW;          // window segment width
  const int grid = win_grid(p);
  const bool cc = p.C2 > 0;
  const int epi = conv_epi_mode(p);
  const int geo = p.KD == 3 ? GEO_3D : (p.OW > W ? GEO_SEG : GEO_2D);
#define WIN_EPI(WW, CC, GG)                                                                               \
  if (epi == EPI_FWD)                                                                                     \
    UNET_LAUNCH((conv_win_kernel<WW, BN, BM, CC, EPI_FWD, GG>), dim3(grid), dim3(NTHR), 0, s, p);     \
  else if (epi == EPI_DGRAD)                                                                              \
    UNET_LAUNCH((conv_win_kernel<WW, BN, BM, CC, EPI_DGRAD, GG>), dim3(grid), dim3(NTHR), 0, s, p);   \
  else if (epi == EPI_STATS)                                                                              \
    UNET_LAUNCH((conv_win_kernel<WW, BN, BM, CC, EPI_STATS, GG>), dim3(grid), dim3(NTHR), 0, s, p);   \
  else if (epi == EPI_DGRAD_NORM && !CC)                                                                  \
    UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD_NORM, GG>), dim3(grid), dim3(NTHR), 0, s, p); \
  else if (epi == EPI_DGRAD_NORM)                                                                         \
    return hipErrorInvalidValue;                                                                          \
  else                                                                                                    \
    UNET_LAUNCH((conv_win_kernel<WW, BN, BM, CC, EPI_GENERIC, GG>), dim3(grid), dim3(NTHR), 0, s, p);
#define WIN_GEO(WW, CC)                                                                                   \
  if (geo == GEO_3D) {                                                                                    \
    WIN_EPI(WW, CC, GEO_3D)                                                                               \
  } else {                                                                                                \
    WIN_EPI(WW, CC, GEO_2D)                                                                               \
  }
#define WIN_CASE(WW)                                                                                      \
  case WW:                                                                                                \
    if constexpr (win_tile_built<BN, BM>(WW)) {                                                           \
      if (cc) {                                                                                           \
        WIN_GEO(WW, true)                                                                                 \
      } else {                                                                                            \
        WIN_GEO(WW, false)                                                                                \
      }                                                                                                   \
    } else {                                                                                              \
      return hipErrorInvalidValue;                                                                        \
    }                                                                                                     \
    break;
#define XF_CASE(WW)                                                                                           \
  case WW:                                                                                                    \
    if constexpr (win_tile_built<BN, BM>(WW)) {                                                               \
      if (p.xform == 2) {                                                                                     \
        if constexpr ((BN == 64 && BM == 256 && WW <= 64) || (BN == 32 && BM == 512 && WW == 64)) {           \
          if (epi == EPI_DGRAD_NORM)                                                                          \
            UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD_NORM, GEO_2D, 2>), dim3(grid), dim3(NTHR), 0, s, \
                        p);                                                                                   \
          else if (epi == EPI_DGRAD)                                                                          \
            UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD, GEO_2D, 2>), dim3(grid), dim3(NTHR), 0, s, p); \
          else                                                                                                \
            return hipErrorInvalidValue;                                                                      \
        } else {                                                                                              \
          return hipErrorInvalidValue;                                                                        \
        }                                                                                                     \
      } else if (epi == EPI_STATS)                                                                            \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_STATS, GEO_2D, 1>), dim3(grid), dim3(NTHR), 0, s, p); \
      else if (epi == EPI_GENERIC)                                                                            \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_GENERIC, GEO_2D, 1>), dim3(grid), dim3(NTHR), 0, s, p); \
      else                                                                                                    \
        return hipErrorInvalidValue;                                                                          \
    } else {                                                                                                  \
      return hipErrorInvalidValue;                                                                            \
    }                                                                                                         \
    break;
  if (p.hg.prob) {                      // head-on-load data gradient (conv_fwd_prepare checks the shape)
    if (epi != EPI_DGRAD || (geo != GEO_2D && geo != GEO_3D)) return hipErrorInvalidValue;
    switch (W) {
#define HG_CASE(WW)                                                                                       \
  case WW:                                                                                                \
    if constexpr (win_tile_built<BN, BM>(WW)) {                                                           \
      if (geo == GEO_3D)                                                                                  \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD, GEO_3D, 3>), dim3(grid), dim3(NTHR), 0, s, p); \
      else                                                                                                \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD, GEO_2D, 3>), dim3(grid), dim3(NTHR), 0, s, p); \
    } else {                                                                                              \
      return hipErrorInvalidValue;                                                                        \
    }                                                                                                     \
    break;
      HG_CASE(16)
      HG_CASE(32)
      HG_CASE(64)
      HG_CASE(128)
#undef HG_CASE
      default:
        return hipErrorInvalidValue;
    }
    return launch_status();
  }
  if (p.s2d) {                          // space-to-depth dgrad source (conv_fwd_prepare checks the shape)
    if ((epi != EPI_DGRAD && epi != EPI_DGRAD_NORM) || geo != GEO_2D) return hipErrorInvalidValue;
    switch (W) {
#define S2D_CASE(WW)                                                                                      \
  case WW:                                                                                                \
    if constexpr (win_tile_built<BN, BM>(WW)) {                                                           \
      if (epi == EPI_DGRAD)                                                                               \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD, GEO_2D, 4>), dim3(grid), dim3(NTHR), 0, s, p); \
      else                                                                                                \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, false, EPI_DGRAD_NORM, GEO_2D, 4>), dim3(grid), dim3(NTHR), 0, s, \
                           p);                                                                            \
    } else {                                                                                              \
      return hipErrorInvalidValue;                                                                        \
    }                                                                                                     \
    break;
      S2D_CASE(16)
      S2D_CASE(32)
      S2D_CASE(64)
      S2D_CASE(128)
#undef S2D_CASE
      default:
        return hipErrorInvalidValue;
    }
    return launch_status();
  }
  if (p.ut.x) {                         // transposed-conv source on load (conv_fwd_prepare checks the shape)
    if (!cc || geo != GEO_2D) return hipErrorInvalidValue;
    switch (W) {
#define UT_CASE(WW)                                                                                       \
  case WW:                                                                                                \
    if constexpr (WW >= 32 && win_tile_built<BN, BM>(WW) && (BM / WW) % 2 == 0) {                          \
      if (epi == EPI_FWD)                                                                                 \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, true, EPI_FWD, GEO_2D, 5>), dim3(grid), dim3(NTHR), 0, s, p); \
      else if (epi == EPI_STATS)                                                                          \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, true, EPI_STATS, GEO_2D, 5>), dim3(grid), dim3(NTHR), 0, s, p); \
      else if (epi == EPI_GENERIC)                                                                        \
        UNET_LAUNCH((conv_win_kernel<WW, BN, BM, true, EPI_GENERIC, GEO_2D, 5>), dim3(grid), dim3(NTHR), 0, s, p); \
      else                                                                                                \
        return hipErrorInvalidValue;                                                                      \
    } else {                                                                                              \
      return hipErrorInvalidValue;                                                                        \
    }                                                                                                     \
    break;
      UT_CASE(32)
      UT_CASE(64)
      UT_CASE(128)
#undef UT_CASE
      default:
        return hipErrorInvalidValue;
    }
    return launch_status();
  }
  if (p.xform) {                        // operand transform: 2D single source (conv_fwd_prepare)
    switch (W) {
      XF_CASE(16)
      XF_CASE(32)
      XF_CASE(64)
      XF_CASE(128)
      default:
        return hipErrorInvalidValue;
    }
    return launch_status();
  }
#undef XF_CASE
  if (geo == GEO_SEG) {                 // 3D volumes wider than 128 are not window-eligible
    if constexpr (!win_tile_built<BN, BM>(128)) return hipErrorInvalidValue;
    if (cc) {
      WIN_EPI(128, true, GEO_SEG)
    } else {
      WIN_EPI(128, false, GEO_SEG)
    }
    return launch_status();
  }
  switch (W) {
    WIN_CASE(16)
    WIN_CASE(32)
    WIN_CASE(64)
    WIN_CASE(128)
    default:
      return hipErrorInvalidValue;
  }
#undef WIN_CASE
#undef WIN_GEO
#undef WIN_EPI
  return launch_status();
}
#endif  // UNET_WIN_IMPL

}  // namespace unet
