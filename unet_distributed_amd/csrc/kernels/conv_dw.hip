// Fused data + weight gradient of a 3x3 conv on 128-wide rows (level 1 of the 128^2 UNet):
// one read of the output gradient dY serves both gradients (conv_params.h FusedWgrad).
//
// The split kernels each stage dY from HBM: the row-window data gradient
// (conv_win.h, EPI_DGRAD) as a halo image, the row-window weight gradient
// (conv_wgrad.hip::wgrad_win_kernel) as a window image beside a halo image of the input
// x.  Both sums can be written over the SAME dY halo:
//   dX[q][ci]        = sum_{tap, co} Wf[tap][ci][co] dY[q + tap - 1][co]       (Wf flipped)
//   dW[tap][ci][co]  = sum_q x[q][ci] dY[q - tap + 1][co]
// (q over the window's own pixels; dY outside the image is the halo's zero fill).  So a
// workgroup stages per window the (R + 2)-row dY halo image and the R-row x image
// (no halo), runs the data-gradient MFMAs (conv_win's strip map and operand reads) and
// the weight-gradient MFMAs (transposed LDS reads, k = pixels) and stores dX through the
// shared epilogue.  The dW partial stays in registers across the workgroup's contiguous
// window range and leaves as one fp32 slab row.
//
// Shape: 2D, W = 128, R = 2 rows per window (256 pixels), C1 = Cx = Cout = 32.  LDS:
// weights 18 KB (staged once per workgroup), dY halo 36 KB (4 rows x 144 slots), x 16 KB:
// 70 KB, two workgroups per CU.  Registers: a wave's 9 x 32 x 16 dW partial is 72 per
// lane, the data-gradient tile 32; the weight-gradient MFMAs run before the data-gradient
// ones so their operands are never live together.
//
// One LDS image, two read patterns: the data gradient reads 16 consecutive pixels x one
// 16-byte chunk per lane group (b128), the weight gradient 8 pixels x 4 channels per lane
// (b64 transposed).  No XOR swizzle of the chunk by column serves both when a lane group's
// transposed reads cover pixels p and p + 8 (tools/lds_bank_model.py search), but the
// k -> pixel order of an MFMA K step is free: with each half-wave reading 8 CONSECUTIVE
// pixels (k = 8 G + 4 hh + q -> pixel 16 (G >> 1) + 8 hh + 4 (G & 1) + q), conv_win's
// swizzle chunk ^ ((col >> 1) & 3) is conflict-free for both at every column shift.
//
// Normalised convs (BatchNorm / GroupNorm, round 6): the conv's pre-activation gradient is
// dz = ca g + cb z + cc per channel (norm.hip::norm_bwd_apply_kernel), g the masked
// gradient of the normalised output, z the pre-norm output.  XF 2 forms dz IN the halo
// image -- each thread loads the g and z granules of its slots into registers and writes
// fmaf(ca, g, fmaf(cb, z, cc)) rounded to 16 bits (the same values norm_bwd_apply would
// have stored), zeros outside the image -- so the dz tensor is never written or read.
// With p.hg.prob set as well (the head input conv9b), g itself is formed per pixel from
// the probability, the target and the ReLU mask [fa z + fc > 0] (head.hip
// head_norm_bwd_kernel's formula): neither g nor dz exists in memory.  The data gradient's
// destination is itself a normalised activation's gradient (EPI_DGRAD_NORM: mask from its
// pre-norm z, one {sum g, sum g z} statistics row per window).
#include "common.h"
#include "conv_params.h"
#include "conv_epilogue.h"
#include "conv_win.h"
#include "head_grad.h"

namespace unet {
namespace {

constexpr int DW_NTHR = 256;
constexpr int DW_W = 128, DW_R = 2, DW_HR = DW_R + 2, DW_BM = DW_W * DW_R, DW_BN = 32;
constexpr int DW_HWP = (DW_W + 2 + 15) / 16 * 16;     // halo row pitch in 64-byte slots (144)
constexpr int DW_PPR = DW_HWP / 16;                   // 16-slot DMA pieces per halo row
constexpr int DW_ROWB = DW_HWP * 64;
constexpr int DW_XI = DW_HR * DW_PPR;                 // dY halo pieces (1 KB each)
constexpr int DW_WI = 9 * DW_BN / 16;                 // weight pieces
constexpr int DW_AI = DW_BM / 16;                     // x image pieces
constexpr int DW_WB = DW_WI * 1024, DW_XB = DW_XI * 1024, DW_AB = DW_AI * 1024;
constexpr int DW_KB = 6 * 32 * 4;                     // XF 2 / 3 coefficients
constexpr int DW_LDS = DW_WB + DW_XB + DW_AB + DW_KB;
// the epilogue's staging tile (BN = 32: unpadded 64-byte rows + [4][2][BN] statistics
// partials, conv_epilogue.h) aliases the two physical halo rows of the window's first two
// logical rows, which the next window does not carry
static_assert(DW_BM * 64 + 4 * 2 * DW_BN * 4 <= 2 * DW_ROWB, "epilogue staging aliases two halo rows");
static_assert(4 * 64 * 16 * 4 <= DW_LDS, "slab reduction scratch");
// XF 2: granule k = tid + 256 j of the HR x 144-slot x 4-chunk halo (slots 130..143 are
// padding, stored as zeros) -> LDS byte 16 k with the chunk swizzled; a thread's chunk is
// tid & 3 for every j, so it holds one 8-channel set of coefficients
constexpr int DW_HG = DW_HR * DW_HWP * 4;
constexpr int DW_HJ = DW_HG / DW_NTHR;
static_assert(DW_HG == DW_HJ * DW_NTHR, "whole granule passes");

// per-pixel logit gradients of the halo granules (XF 4: head_grad.h, head.hip
// head_bwd_kernel's formula; XF 3: the normalised head's, head.hip hn_scalars)
template <int XF>
__device__ __forceinline__ void dw_dlogit(const ConvFwdParams& p, const float (&pr)[DW_HJ], const float (&tv)[DW_HJ],
                                          float (&dl)[DW_HJ]) {
  if constexpr (XF == 4) {
    const float I = p.hg.sums[0], St = p.hg.sums[1], Sp = p.hg.sums[2];
    const float a = -2.f / (2.f * I + 1.f), bb = 1.f / (St + Sp + 1.f);
    const float gs = p.hg.gscale ? *p.hg.gscale : 1.f;
#pragma unroll
    for (int j = 0; j < DW_HJ; ++j) dl[j] = head_dlogit(pr[j], tv[j], a, bb, p.hg.inv_total, p.hg.bce_w, gs);
  } else {
    const float gs = p.hg.gscale ? *p.hg.gscale : 1.f;
    const float al = -2.f * gs / (2.f * p.hg.sums[0] + 1.f);
    const float be = gs / (p.hg.sums[1] + p.hg.sums[2] + 1.f);
    const float ga = gs * p.hg.bce_w * p.hg.inv_total;
#pragma unroll
    for (int j = 0; j < DW_HJ; ++j) dl[j] = hn_dlogit(pr[j], tv[j], al, be, ga);
  }
}

// SEG: rows of Wf = p.OW > 128 pixels (the 512^2 model) as 128-pixel segments; windows are
// walked segment-major (segment s = window / (rows / R)), so consecutive windows of a
// workgroup are consecutive row pairs of one segment and the halo-row carry still holds;
// the halo columns -1 / 128 are the neighbouring segments' pixels (zeros at the row ends).
template <int EPI, int XF, bool SEG = false>
__global__ void __launch_bounds__(DW_NTHR, 2) conv_dw_kernel(const ConvFwdParams p) {
  static_assert(XF == 0 || XF == 2 || XF == 3 || XF == 4,
                "plain dY, norm backward on load (of the normalised head), head gradient on load");
  constexpr int W = DW_W, R = DW_R, HR = DW_HR, ROWB = DW_ROWB, BN = DW_BN;
  constexpr int TM = 4, TN = 2, TC = 2, RW = 2, NCS = 4;   // data-gradient strip: 2 rows x 32 columns per wave
  __shared__ __attribute__((aligned(1024))) char smem[DW_LDS];
  char* Ws = smem;
  char* Xs = smem + DW_WB;            // dY halo image (also the epilogue's staging tile)
  char* As = Xs + DW_XB;              // x image of the window's own rows

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int rows_total = p.N * H;
  const int Wf = SEG ? p.OW : W;                       // row width (SEG: > 128)
  const int M = rows_total * Wf;
  const int nrp = rows_total / R;                      // row pairs per segment
  const int nwin = nrp * (SEG ? Wf / W : 1);
  const int split = blockIdx.x;
  const int w_begin = (int)((long long)split * nwin / p.fw.nsplit);
  const int w_end = (int)((long long)(split + 1) * nwin / p.fw.nsplit);
  constexpr int OOB = 0x7fffffff;
  const int C = p.C1;                 // dY channels (32)
  const int Cx = p.fw.Cx;             // x channels (32)
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
  const int fsub = lane >> 4, fr = lane & 15;
  const int c0 = wave * 32;           // this wave's data-gradient column strip
  static_assert(DW_HR == 4 && DW_AI % 4 == 0, "one halo row per wave");
  // lane part of the DMA offsets: slot lslot of a 16-slot piece = column lslot - 1 of the
  // halo row (x image: column lslot), physical chunk lane & 3 = logical chunk lchunk
  const int dma_lane = ((lslot - 1) * 32 + lchunk * 8) * 2;
  const int xdma_lane = (lslot * 32 + lchunk * 8) * 2;

  // weights (flipped data-gradient copy, rows (tap, ci) of 32 co): staged once
  {
    const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.wgt, (short)0, OOB, 0x00020000);
    const int wl = (lslot * p.Kpad + lchunk * 8) * 2;
#pragma unroll
    for (int q = 0; q < (DW_WI + 3) / 4; ++q) {
      const int k = wave + 4 * q;
      if (k < DW_WI) {
        const int tap = k / (BN / 16), nb = (k % (BN / 16)) * 16;
        const int off = (nb * p.Kpad + tap * C) * 2 + wl;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsw, (__attribute__((address_space(3))) void*)(Ws + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
  }

  // data-gradient operand bases (conv_win.h chunk_mfmas): horizontal tap dw -> halo column
  // c0 + fr + dw; weight rows fr of each 16-row block
  int xbase[3];
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = fr + dw;
    xbase[dw] = c0 * 64 + hc * 64 + 16 * (fsub ^ ((hc >> 1) & 3));
  }
  const int wbase = fr * 64 + 16 * (fsub ^ ((fr >> 1) & 3));

  // weight-gradient transposed-read lane roles: lane (G, q, pp) supplies pixel
  // kp(hh) = 16 (G >> 1) + 8 hh + 4 (G & 1) + q of the 32-pixel step and channels
  // 4 pp .. 4 pp + 3 of a 16-channel block.  Wave w owns the dY channel block jw = w & 1
  // of column strips 2 (w >> 1) and 2 (w >> 1) + 1: its dW partial is 9 x 32 x 16 (72
  // registers; a whole 9 x 32 x 32 partial per wave left no room for the XF 2 halo
  // staging), at the price of reading each strip's x fragments twice (8 of 56 reads).
  const int G = lane >> 4, tq = (lane >> 2) & 3, pp = lane & 3;
  const int jw = wave & 1, sw0 = (wave >> 1) * 2;
  auto saddr = [](const int slot, const int col, const int ch) -> int {
    return slot * 64 + (((ch >> 3) ^ ((col >> 1) & 3)) << 4) + ((ch & 7) << 1);
  };
  // One base register per image and shift (strip 0; strip s is s * 2048 bytes on, the
  // same swizzle): the second read of a pair (hh = 1) is 8 pixels on, +512 bytes with the
  // same swizzle ((col + 8) >> 1 & 3 == col >> 1 & 3); the second 16-channel block flips
  // chunk bit 1, i.e. the address's bit 5 (XOR 32).
  const int kp0 = 16 * (G >> 1) + 4 * (G & 1) + tq;
  const int abase = saddr(kp0, kp0, 4 * pp);                      // x image (+ y * W * 64)
  int dbase[3];                                                    // dY halo (+ hr * ROWB)
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = kp0 + 2 - dw;                                   // dW tap (dh, dw): halo column col + 2 - dw
    dbase[dw] = saddr(hc, hc, 4 * pp) ^ (32 * jw);
  }
  auto tr8 = [&](const char* b0, const char* b1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, b0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, b1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };

  f32x4 wacc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i) wacc[t][i] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc = (f32x4){0.f, 0.f, 0.f, 0.f};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);
  // XF 2: the window sample's backward coefficients ca / cb / cc [3][32] in LDS (written
  // per window by threads 0..95, read by each thread for its 8 channels in the halo pass:
  // registers only while the halo is formed)
  float* Ks = (float*)(As + DW_AB);
  const int kch = (tid & 3) * 8;
  // Halo row carry: the next window of the same image needs halo rows g0 + 1, g0 + 2 --
  // this window's logical rows 2, 3 (already formed: XF 2 / 3 transformed).  Logical row r
  // lives in physical row r ^ 2 fl; a carried window flips fl and loads (forms) only its
  // rows 2, 3, into the physical rows the previous epilogue staged its tile in.  Halves the
  // halo's loads (and the XF 2 / 3 transform work); the MFMA address offsets become
  // hr ROWB +- 2 fl ROWB.
  int fl = 0;

  for (int win = w_begin; win < w_end; ++win) {
    const int seg = SEG ? win / nrp : 0;
    const int col0 = seg * W;                          // the window's first column
    const int g0 = (SEG ? win - seg * nrp : win) * R;
    const int grow0 = (g0 / H) * H;                    // the window's image (H % R == 0)
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const bool carry = win > w_begin && top_in;       // (wave-uniform)
    if (carry) fl ^= 1;
    const int fo = fl * 2 * ROWB;                       // physical offset of logical rows 0, 1 (rows 2, 3: -fo)
    const int k0 = carry ? 2 * DW_HWP * 4 : 0;          // first halo granule to form
    const size_t img_px = (size_t)grow0 * Wf;
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.src1 + img_px * C * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.fw.x + ((size_t)g0 * Wf + col0) * Cx * 2), (short)0, OOB, 0x00020000);
    // XF 2: the z granules of the halo (and the coefficients) are loaded into registers
    // before the barrier, so they fly while the previous window's epilogue stores drain; g
    // arrives through the dY halo DMA below and is turned into dz in place.  XF 3: the
    // DMA brings z (src1 = z), g = w dlogit [fa z + fc > 0] per pixel with dlogit from the
    // probability and target loaded here (XF 4: dY = w dlogit [y > 0] from the ReLU bits)
    u32x4 zv[XF == 2 ? DW_HJ : 1];
    // XF 3 / 4: each lane loads its granule's pixel probability / target (XF 4: the byte
    // of ReLU bits of its 8 channels); the logit gradients are formed after the DMA barrier.
    // (Measured against one load per lane + DPP quad broadcasts, and against forming the
    // logit gradients before the first barrier: per launch 0.855 vs 0.90 / 0.87 ms, XF 4.)
    float dl[XF >= 3 ? DW_HJ : 1];
    uint32_t hbits[XF == 4 ? DW_HJ : 1];
    float pr[XF >= 3 ? DW_HJ : 1], tv[XF >= 3 ? DW_HJ : 1];
    uint32_t okm = 0;
    if constexpr (XF >= 2) {
      // Ks: ca cb cc [fa fc ca*w] of the window's sample (XF 4: the head weights w)
      float kv = 0.f;
      constexpr int NK = XF == 4 ? 32 : XF == 3 ? 192 : 96;
      if (tid < NK) {
        const int m = tid >> 5, c = tid & 31;
        if constexpr (XF == 4) {
          kv = p.hg.w[c];
        } else {
          const float* src = m == 0 ? p.xa : m == 1 ? p.xb : m == 2 ? p.xc : m == 3 ? p.hg.fa : m == 4 ? p.hg.fc : p.xa;
          const size_t ci = (size_t)(g0 / H) * p.xcs + c;
          kv = src[ci];
          if (XF == 3 && m == 5) kv *= p.hg.w[c];
        }
      }
      const __amdgpu_buffer_rsrc_t rsz = __builtin_amdgcn_make_buffer_rsrc(
          (void*)((const char*)p.xz + img_px * C * 2), (short)0, OOB, 0x00020000);
#pragma unroll
      for (int j = 0; j < DW_HJ; ++j) {
        const int k = k0 + tid + DW_NTHR * j;
        const int hr = k / (DW_HWP * 4), s = (k >> 2) - hr * DW_HWP;
        const int gr = g0 - 1 + hr, col = col0 + s - 1;
        const bool ok = k < DW_HG && (hr > 0 || top_in) && (hr < R + 1 || bot_in) &&
                        (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)Wf && s <= W + 1;
        okm |= (ok ? 1u : 0u) << j;
        if constexpr (XF >= 3) {
          const int pix = ok ? gr * Wf + col : 0;
          pr[j] = p.hg.prob[pix];
          tv[j] = bits2f(((const uint16_t*)p.hg.t)[pix]);
          if constexpr (XF == 4) hbits[j] = ok ? ((const uint8_t*)p.hg.bits)[(size_t)pix * 4 + (tid & 3)] : 0u;
        }
        if constexpr (XF == 2)
          zv[j] = __builtin_amdgcn_raw_buffer_load_b128(rsz, ok ? ((gr - grow0) * Wf + col) * C * 2 + kch * 2 : OOB,
                                                        0, 0);
      }
      if (tid < NK) Ks[tid] = kv;    // (the previous window read them before its MFMAs)
    }
    __syncthreads();      // the previous window's epilogue is done with the staging tile
    // dY (XF 2: g, XF 3: z) halo image: wave w fills halo row hr = w (pixel row g0 - 1 + w)
    // -- carried: waves 2 i, 2 i + 1 the two halves of row 2 + i -- slot hc = column hc - 1,
    // as 16-slot pieces; rows of another image and columns outside [0, W) load zeros
    // (out-of-range offsets).  Per piece only an immediate changes.
    if constexpr (XF != 4) {
      const int hr = carry ? 2 + (wave >> 1) : wave;
      const int jlo = carry ? 5 * (wave & 1) : 0, jhi = carry && !(wave & 1) ? 5 : DW_PPR;
      const int gr = g0 - 1 + hr;
      const bool row_ok = (hr > 0 || top_in) && (hr < R + 1 || bot_in) && (unsigned)gr < (unsigned)rows_total;
      const int rowoff = ((gr - grow0) * Wf + col0) * C * 2;
      char* hdst = Xs + (hr ^ (2 * fl)) * ROWB;
#pragma unroll
      for (int j = 0; j < DW_PPR; ++j) {
        if (j < jlo || j >= jhi) continue;
        // (SEG: slot 16 j + lslot = column col0 + 16 j + lslot - 1, the neighbour segments'
        // pixels at slots 0 / 129; slots past 129 are never read)
        const bool ok = row_ok && (unsigned)(col0 + 16 * j + lslot - 1) < (unsigned)Wf && 16 * j + lslot <= W + 1;
        const int off = ok ? rowoff + dma_lane + j * 1024 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs1, (__attribute__((address_space(3))) void*)(hdst + j * 1024),
                                                 16, off, 0, 0, 0);
      }
    }
    // x image: slot y * W + col = pixel (g0 + y, col0 + col), the same swizzle; wave w fills
    // slots 64 w .. 64 w + 63 (row w >> 1: SEG rows are Wf apart)
#pragma unroll
    for (int i = 0; i < DW_AI / 4; ++i) {
      const int k = 4 * wave + i;
      const int xo = SEG ? ((k >> 3) * Wf + 16 * (k & 7)) * Cx * 2 : k * 1024;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (__attribute__((address_space(3))) void*)(As + k * 1024), 16,
                                               xdma_lane + xo, 0, 0, 0);
    }
    __syncthreads();
    // (the per-pixel logit gradients: formed here, after the barrier, so the probability /
    // target loads overlap the x image DMA instead of being waited on before it)
    if constexpr (XF >= 3) dw_dlogit<XF>(p, pr, tv, dl);
    if constexpr (XF == 4) {
      // dY = dlogit w (x > 0) per slot (head_grad.h head_grad_pixel), zeros outside the image
      float hw[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) hw[e] = Ks[kch + e];
#pragma unroll
      for (int j = 0; j < DW_HJ; ++j) {
        const int k = k0 + tid + DW_NTHR * j;
        if (k >= DW_HG) continue;
        const int hr = k / (DW_HWP * 4), s = (k >> 2) - hr * DW_HWP;
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = dl[j] * hw[e];
          o[e] = ((hbits[j] >> e) & 1u) ? v : 0.f;
        }
        *(u32x4*)(Xs + ((hr ^ (2 * fl)) * DW_HWP + s) * 64 + 16 * ((tid & 3) ^ ((s >> 1) & 3))) = pack8(o);
      }
      __syncthreads();
    } else if constexpr (XF >= 2) {
      // dz = fmaf(ca, g, fmaf(cb, z, cc)) in place (16-byte granule k of the halo: LDS
      // slot k >> 2, logical chunk tid & 3), zeros outside the image.  XF 3: dz =
      // (fa z + fc > 0 ? ca w dlogit : 0) + fmaf(cb, z, cc) (head.hip head_norm_bwd_kernel)
      float ka[8], kb[8], kc[8], kf[8], kg[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ka[e] = Ks[(XF == 3 ? 160 : 0) + kch + e];
        kb[e] = Ks[32 + kch + e];
        kc[e] = Ks[64 + kch + e];
        if constexpr (XF == 3) {
          kf[e] = Ks[96 + kch + e];
          kg[e] = Ks[128 + kch + e];
        }
      }
#pragma unroll
      for (int j = 0; j < DW_HJ; ++j) {
        const int k = k0 + tid + DW_NTHR * j;
        if (k >= DW_HG) continue;
        const int hr = k / (DW_HWP * 4), s = (k >> 2) - hr * DW_HWP;
        u32x4* slot = (u32x4*)(Xs + ((hr ^ (2 * fl)) * DW_HWP + s) * 64 + 16 * ((tid & 3) ^ ((s >> 1) & 3)));
        u32x4 v = {0u, 0u, 0u, 0u};
        if ((okm >> j) & 1u) {
          float gf[8], zf[8];
          if constexpr (XF == 3) {
            unpack8(*slot, zf);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float g = fmaf(kf[e], zf[e], kg[e]) > 0.f ? ka[e] * dl[j] : 0.f;
              gf[e] = g + fmaf(kb[e], zf[e], kc[e]);
            }
          } else {
            unpack8(zv[j], zf);
            unpack8(*slot, gf);
#pragma unroll
            for (int e = 0; e < 8; ++e) gf[e] = fmaf(ka[e], gf[e], fmaf(kb[e], zf[e], kc[e]));
          }
          v = pack8(gf);
        }
        *slot = v;
      }
      __syncthreads();
    }

    // ---- weight gradient: halo row hr at shift dw feeds x rows y = hr - 2 + dh
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      const int so = (sw0 + st) * 32 * 64;
      h16x8 xa[R][2];
#pragma unroll
      for (int y = 0; y < R; ++y)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int a = (abase ^ (32 * i)) + y * W * 64 + so;
          xa[y][i] = tr8(As + a, As + a + 512);
        }
#pragma unroll
      for (int hr = 0; hr < HR; ++hr) {
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const int a = dbase[dw] + hr * ROWB + so + (hr < 2 ? fo : -fo);
          const h16x8 yb = tr8(Xs + a, Xs + a + 512);
          if (dw == 1 && hr >= 1 && hr <= R) bacc = mfma16(ones, yb, bacc);   // the window's own dY: bias sums
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int y = hr - 2 + dh;
            if (y < 0 || y >= R) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i) wacc[3 * dh + dw][i] = mfma16(xa[y][i], yb, wacc[3 * dh + dw][i]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    // ---- data gradient (conv_win.h chunk_mfmas, one 32-channel chunk)
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
          const h16x8 xf = *(const h16x8*)(Xs + xbase[dw] + hr * ROWB + ci * 16 * 64 + (hr < 2 ? fo : -fo));
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
    __syncthreads();      // every wave is done reading the halo image (the staging tile aliases rows 0, 1)
    using Map = StripTiles<W, RW, TC, NCS>;
    if constexpr (SEG)
      conv_epilogue<DW_BM, BN, DW_BM / 4, BN, TM, TN, DW_NTHR, EPI, Map, W, W>(p, acc, Xs + fo, g0, 0, M, wave, 0,
                                                                              lane, tid, Wf, col0, win);
    else
      conv_epilogue<DW_BM, BN, DW_BM / 4, BN, TM, TN, DW_NTHR, EPI, Map, 0, W>(p, acc, Xs + fo, g0 * W, 0, M, wave, 0,
                                                                              lane, tid, 0, 0, win);
  }

  // ---- sum the partials of the two waves of each dY channel block (waves jw, jw + 2:
  // different column strips) and write the slab row
  float* red = (float*)smem;
  const int row = p.fw.split_lo + split;
  const int n_base = lane & 15, m_base = 4 * (lane >> 4);
  auto reduce_store = [&](const f32x4 (&v4)[2], const int t) {
    __syncthreads();
    if (wave >= 2) {    // red[fragment][wave * 64 + lane]: lanes 16 bytes apart, conflict-free
#pragma unroll
      for (int i = 0; i < 2; ++i) *(f32x4*)(red + ((i * 2 + jw) * 64 + lane) * 4) = v4[i];
    }
    __syncthreads();
    if (wave < 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const f32x4 v = v4[i] + *(const f32x4*)(red + ((i * 2 + jw) * 64 + lane) * 4);
        if (t < 9) {
          float* dst = p.fw.slab + (((size_t)row * 9 + t) * Cx + m_base + 16 * i) * C + n_base + 16 * jw;
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[(size_t)r * C] = v[r];
        } else if (i == 0 && lane < 16) {
          p.fw.bias_slab[(size_t)row * C + n_base + 16 * jw] = v[0];
        }
      }
    }
  };
#pragma unroll
  for (int t = 0; t < 9; ++t) reduce_store(wacc[t], t);
  const f32x4 bv[2] = {bacc, (f32x4){0.f, 0.f, 0.f, 0.f}};
  reduce_store(bv, 9);
}

}  // namespace

// host check of the fused data + weight gradient (nullptr: supported)
const char* conv_dw_check(const ConvFwdParams& p) {
  if (!p.fw.x) return nullptr;
  const int ep = conv_epi_mode(p);
  const bool w_ok = p.OW == DW_W || (p.OW % DW_W == 0 && p.OW <= 8192);
  if (!w_ok || p.IW != p.OW || p.OH != p.IH || p.OH % DW_R || p.KD != 1 || p.OD != 1 || p.ID != 1 ||
      p.KH != 3 || p.KW != 3 || p.stride != 1 || p.pad != 1 || p.C1 != 32 || p.C2 || p.Cout != DW_BN ||
      p.D1 != p.Cout || p.fw.Cx != 32 || (ep != EPI_DGRAD && ep != EPI_DGRAD_NORM) || p.s2d ||
      p.ut.x || p.pool_dst || p.head_w || p.rev)
    return "conv_fwd: fused weight gradient needs a 2D 32 -> 32 channel data gradient on 128-wide rows";
  if (p.xform && (p.xform != 2 || !p.xa || !p.xb || !p.xc || !p.xz || (p.xcs != 0 && p.xcs != p.C1) || p.xout))
    return "conv_fwd: fused weight gradient: norm backward on load (xform 2) needs xa / xb / xc / xz, xcs 0 or C";
  if (p.hg.prob && p.xform && (p.xform != 2 || p.hg.bits || !p.hg.fa || !p.hg.fc || !p.hg.t || !p.hg.sums ||
                                !p.hg.w || p.route_gy))
    return "conv_fwd: fused weight gradient: the normalised head's gradient on load needs xform 2, "
           "fa / fc (no bits), t, sums, w";
  if (p.hg.prob && !p.xform && (!p.hg.bits || !p.hg.t || !p.hg.sums || !p.hg.w || p.route_gy || ep != EPI_DGRAD))
    return "conv_fwd: fused weight gradient: the head gradient on load needs bits, t, sums, w";
  if (!p.fw.slab || !p.fw.bias_slab || p.fw.nsplit < 1 || p.fw.split_lo < 0)
    return "conv_fwd: fused weight gradient needs slab / bias_slab and nsplit >= 1";
  if ((long long)p.OH * p.OW * 32 * 2 >= (1LL << 31) - 64) return "conv_fwd: one image exceeds 2 GiB";
  if (p.OW > DW_W && (p.xform || p.hg.prob || p.nz))
    return "conv_fwd: fused weight gradient on segmented rows: plain dY source, EPI_DGRAD only";
  return nullptr;
}

int conv_dw_grid(const ConvFwdParams& p) { return p.fw.nsplit; }

// statistics rows of the EPI_DGRAD_NORM epilogue: one per 2-row window (256 pixels)
int conv_dw_stat_rows(const ConvFwdParams& p) { return p.N * p.OH / DW_R; }

hipError_t launch_conv_dw(const ConvFwdParams& p, hipStream_t s) {
  const int ep = conv_epi_mode(p);
  const dim3 grid(p.fw.nsplit), blk(DW_NTHR);
  if (p.OW > DW_W) {
    if (ep != EPI_DGRAD || p.xform || p.hg.prob) return hipErrorInvalidValue;
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD, 0, true>), grid, blk, 0, s, p);
  } else if (ep == EPI_DGRAD && !p.xform && !p.hg.prob)
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD, 0>), grid, blk, 0, s, p);
  else if (ep == EPI_DGRAD && !p.xform)
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD, 4>), grid, blk, 0, s, p);
  else if (ep == EPI_DGRAD && p.xform == 2 && !p.hg.prob)
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD, 2>), grid, blk, 0, s, p);
  else if (ep == EPI_DGRAD_NORM && !p.xform && !p.hg.prob)
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD_NORM, 0>), grid, blk, 0, s, p);
  else if (ep == EPI_DGRAD_NORM && p.xform == 2 && !p.hg.prob)
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD_NORM, 2>), grid, blk, 0, s, p);
  else if (ep == EPI_DGRAD_NORM && p.xform == 2)
    UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD_NORM, 3>), grid, blk, 0, s, p);
  else
    return hipErrorInvalidValue;
  return launch_status();
}

}  // namespace unet
