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
// 70 KB, two workgroups per CU.  Registers: the 9 x 32 x 32 dW partial is 144 per lane,
// the data-gradient tile 32; the weight-gradient MFMAs run before the data-gradient ones
// so their operands are never live together.
//
// One LDS image, two read patterns: the data gradient reads 16 consecutive pixels x one
// 16-byte chunk per lane group (b128), the weight gradient 8 pixels x 4 channels per lane
// (b64 transposed).  No XOR swizzle of the chunk by column serves both when a lane group's
// transposed reads cover pixels p and p + 8 (tools/lds_bank_model.py search), but the
// k -> pixel order of an MFMA K step is free: with each half-wave reading 8 CONSECUTIVE
// pixels (k = 8 G + 4 hh + q -> pixel 16 (G >> 1) + 8 hh + 4 (G & 1) + q), conv_win's
// swizzle chunk ^ ((col >> 1) & 3) is conflict-free for both at every column shift.
#include "common.h"
#include "conv_params.h"
#include "conv_epilogue.h"
#include "conv_win.h"

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
constexpr int DW_LDS = DW_WB + DW_XB + DW_AB;
static_assert(epi_lds_bytes<DW_BM, DW_BN>() <= DW_XB, "epilogue staging aliases the dY halo image");
static_assert(4 * 64 * 16 * 4 <= DW_LDS, "slab reduction scratch");

template <int EPI>
__global__ void __launch_bounds__(DW_NTHR, 2) conv_dw_kernel(const ConvFwdParams p) {
  constexpr int W = DW_W, R = DW_R, HR = DW_HR, ROWB = DW_ROWB, BN = DW_BN;
  constexpr int TM = 4, TN = 2, TC = 2, RW = 2, NCS = 4;   // data-gradient strip: 2 rows x 32 columns per wave
  __shared__ __attribute__((aligned(1024))) char smem[DW_LDS];
  char* Ws = smem;
  char* Xs = smem + DW_WB;            // dY halo image (also the epilogue's staging tile)
  char* As = Xs + DW_XB;              // x image of the window's own rows

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = p.OH;
  const int rows_total = p.N * H;
  const int M = rows_total * W;
  const int nwin = rows_total / R;
  const int split = blockIdx.x;
  const int w_begin = (int)((long long)split * nwin / p.fw.nsplit);
  const int w_end = (int)((long long)(split + 1) * nwin / p.fw.nsplit);
  constexpr int OOB = 0x7fffffff;
  const int C = p.C1;                 // dY channels (32)
  const int Cx = p.fw.Cx;             // x channels (32)
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ ((lslot >> 1) & 3);
  const int fsub = lane >> 4, fr = lane & 15;
  const int c0 = wave * 32;           // this wave's column strip (both gradients)
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
  // 4 pp .. 4 pp + 3 of a 16-channel block
  const int G = lane >> 4, tq = (lane >> 2) & 3, pp = lane & 3;
  auto saddr = [](const int slot, const int col, const int ch) -> int {
    return slot * 64 + (((ch >> 3) ^ ((col >> 1) & 3)) << 4) + ((ch & 7) << 1);
  };
  // One base register per image and shift: the second read of a pair (hh = 1) is 8
  // pixels on, +512 bytes with the same swizzle ((col + 8) >> 1 & 3 == col >> 1 & 3); the
  // second 16-channel block flips chunk bit 1, i.e. the address's bit 5 (XOR 32).
  const int kp0 = 16 * (G >> 1) + 4 * (G & 1) + tq;
  const int abase = saddr(c0 + kp0, c0 + kp0, 4 * pp);            // x image (+ y * W * 64)
  int dbase[3];                                                    // dY halo (+ hr * ROWB)
#pragma unroll
  for (int dw = 0; dw < 3; ++dw) {
    const int hc = c0 + kp0 + 2 - dw;                              // dW tap (dh, dw): halo column col + 2 - dw
    dbase[dw] = saddr(hc, hc, 4 * pp);
  }
  auto tr8 = [&](const char* b0, const char* b1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, b0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, b1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };

  f32x4 wacc[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) wacc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);

  for (int win = w_begin; win < w_end; ++win) {
    const int g0 = win * R;
    const int grow0 = (g0 / H) * H;                    // the window's image (H % R == 0)
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const size_t img_px = (size_t)grow0 * W;
    const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.src1 + img_px * C * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)p.fw.x + (size_t)g0 * W * Cx * 2), (short)0, OOB, 0x00020000);
    __syncthreads();      // the previous window's epilogue is done with the staging tile
    // dY halo image: wave w fills halo row hr = w (pixel row g0 - 1 + w), slot hc =
    // column hc - 1, as 9 pieces of 16 slots; rows of another image and columns outside
    // [0, W) load zeros (out-of-range offsets).  Per piece only an immediate changes.
    {
      const int gr = g0 - 1 + wave;
      const bool row_ok = (wave > 0 || top_in) && (wave < R + 1 || bot_in) && (unsigned)gr < (unsigned)rows_total;
      const int rowoff = (gr - grow0) * W * C * 2;
#pragma unroll
      for (int j = 0; j < DW_PPR; ++j) {
        const bool ok = row_ok && (j > 0 || lslot > 0) && (16 * j + lslot - 1 < W);
        const int off = ok ? rowoff + dma_lane + j * 1024 : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs1, (__attribute__((address_space(3))) void*)(Xs + wave * ROWB + j * 1024),
                                                 16, off, 0, 0, 0);
      }
    }
    // x image: slot y * W + col = pixel (g0 + y, col), the same swizzle; wave w fills slots
    // 64 w .. 64 w + 63
#pragma unroll
    for (int i = 0; i < DW_AI / 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsx, (__attribute__((address_space(3))) void*)(As + (4 * wave + i) * 1024),
                                               16, xdma_lane + (4 * wave + i) * 1024, 0, 0, 0);
    __syncthreads();

    // ---- weight gradient: halo row hr at shift dw feeds x rows y = hr - 2 + dh
    {
      h16x8 xa[R][2];
#pragma unroll
      for (int y = 0; y < R; ++y)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int a = (abase ^ (32 * i)) + y * W * 64;
          xa[y][i] = tr8(As + a, As + a + 512);
        }
#pragma unroll
      for (int hr = 0; hr < HR; ++hr) {
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          h16x8 yb[2];
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int a = (dbase[dw] ^ (32 * j)) + hr * ROWB;
            yb[j] = tr8(Xs + a, Xs + a + 512);
          }
          if (dw == 1 && hr >= 1 && hr <= R) {        // the window's own dY pixels: bias sums
#pragma unroll
            for (int j = 0; j < 2; ++j) bacc[j] = mfma16(ones, yb[j], bacc[j]);
          }
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int y = hr - 2 + dh;
            if (y < 0 || y >= R) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int j = 0; j < 2; ++j) wacc[3 * dh + dw][i][j] = mfma16(xa[y][i], yb[j], wacc[3 * dh + dw][i][j]);
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
    __syncthreads();      // every wave is done reading the halo image (the staging tile aliases it)
    using Map = StripTiles<W, RW, TC, NCS>;
    conv_epilogue<DW_BM, BN, DW_BM / 4, BN, TM, TN, DW_NTHR, EPI, Map, 0, W>(p, acc, Xs, g0 * W, 0, M, wave, 0, lane,
                                                                            tid, 0, 0, win);
  }

  // ---- sum the four waves' partials (different column strips) and write the slab row
  float* red = (float*)smem;
  const int row = p.fw.split_lo + split;
  const int n_base = lane & 15, m_base = 4 * (lane >> 4);
  auto reduce_store = [&](const f32x4 (&v4)[2][2], const int t) {
    __syncthreads();
    if (wave > 0) {     // red[fragment][wave * 64 + lane]: lanes 16 bytes apart, conflict-free
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) *(f32x4*)(red + ((i * 2 + j) * 256 + wave * 64 + lane) * 4) = v4[i][j];
    }
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 v = v4[i][j];
#pragma unroll
          for (int o = 1; o < 4; ++o) v += *(const f32x4*)(red + ((i * 2 + j) * 256 + o * 64 + lane) * 4);
          if (t < 9) {
            float* dst = p.fw.slab + (((size_t)row * 9 + t) * Cx + m_base + 16 * i) * C + n_base + 16 * j;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)r * C] = v[r];
          } else if (i == 0 && lane < 16) {
            p.fw.bias_slab[(size_t)row * C + n_base + 16 * j] = v[0];
          }
        }
    }
  };
#pragma unroll
  for (int t = 0; t < 9; ++t) reduce_store(wacc[t], t);
  const f32x4 z = (f32x4){0.f, 0.f, 0.f, 0.f};
  const f32x4 bv[2][2] = {{bacc[0], bacc[1]}, {z, z}};
  reduce_store(bv, 9);
}

}  // namespace

// host check of the fused data + weight gradient (nullptr: supported)
const char* conv_dw_check(const ConvFwdParams& p) {
  if (!p.fw.x) return nullptr;
  const int ep = conv_epi_mode(p);
  if (p.OW != DW_W || p.IW != DW_W || p.OH != p.IH || p.OH % DW_R || p.KD != 1 || p.OD != 1 || p.ID != 1 ||
      p.KH != 3 || p.KW != 3 || p.stride != 1 || p.pad != 1 || p.C1 != 32 || p.C2 || p.Cout != DW_BN ||
      p.D1 != p.Cout || p.fw.Cx != 32 || ep != EPI_DGRAD || p.xform || p.hg.prob || p.s2d || p.ut.x ||
      p.pool_dst || p.head_w || p.rev)
    return "conv_fwd: fused weight gradient needs a 2D 32 -> 32 channel data gradient on 128-wide rows";
  if (!p.fw.slab || !p.fw.bias_slab || p.fw.nsplit < 1 || p.fw.split_lo < 0)
    return "conv_fwd: fused weight gradient needs slab / bias_slab and nsplit >= 1";
  if ((long long)p.OH * p.OW * 32 * 2 >= (1LL << 31) - 64) return "conv_fwd: one image exceeds 2 GiB";
  return nullptr;
}

int conv_dw_grid(const ConvFwdParams& p) { return p.fw.nsplit; }

hipError_t launch_conv_dw(const ConvFwdParams& p, hipStream_t s) {
  if (conv_epi_mode(p) != EPI_DGRAD) return hipErrorInvalidValue;
  UNET_LAUNCH((conv_dw_kernel<EPI_DGRAD>), dim3(p.fw.nsplit), dim3(DW_NTHR), 0, s, p);
  return launch_status();
}

}  // namespace unet
