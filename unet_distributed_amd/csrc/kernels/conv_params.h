// Host/device parameter blocks of the conv kernels (POD, passed by value).
#pragma once
#include <stdint.h>

// Shared by the bf16 (`unet`) and fp16 (`unet_f16`) builds of the kernels (see
// common.h): the parameter blocks live outside the element-type namespaces so both
// builds' launchers take the same host types.
namespace unet_types {

// Dry dispatch (host): while set, the kernel launchers resolve their dispatch -- template
// instantiation, tile, epilogue -- and return the status they would return, without
// launching (UNET_LAUNCH / launch_status in common.h).  The executor's plan validation
// uses it on a CPU host to prove every planned launch has a built kernel
// (runtime/plan_check.py).  Defined in runtime/bindings.cpp.
bool dry_dispatch();

// Gradient of the segmentation head's input formed on load (head-on-load): the consumer
// kernel builds dY[p][c] = dlogit(p) * w[c] * (x[p][c] > 0) itself from the per-pixel
// probability / target, the loss sums and the head input's ReLU bits, so the head
// backward never writes the full-resolution dY (head.hip::head_dlogit is the formula).
// prob == nullptr: off.
struct HeadGrad {
  const float* prob;          // [P] sigmoid outputs
  const void* t;              // [P] 16-bit targets
  const float* sums;          // {I, St, Sp, BCE} of the forward
  const float* w;             // [C] fp32 head weights
  const uint8_t* bits;        // [P][C / 8] ReLU bits of the head input
  const float* gscale;        // device loss scale (nullptr: 1)
  float inv_total, bce_w;     // 1 / (pixels of the batch), BCE weight (0: Dice only)
  // normalised head input (conv_dw.hip, xform 2 + prob, bits == nullptr): the ReLU mask is
  // [fa z + fc > 0] of the pre-norm z (p.xz) instead of bits; [C] or [N][C] (p.xcs)
  const float* fa;
  const float* fc;
};

// Transposed-conv source on load (2D row-window forward of a decoder conv whose first
// source u = tconv2x2s2(x) + b is read by nothing else -- the composite backward never
// re-reads it): each 32-channel chunk of u is formed in LDS from the coarse input
// (conv_win.h XF 5), so u is never written to or read from memory and the transposed
// conv's own forward launch disappears.  x == nullptr: off.
struct TconvSrc {
  const void* x;              // [N][OH/2][OW/2][C] 16-bit coarse input
  const void* w;              // 16-bit [4][C1][kpad]: tap (th, tw) = 2 th + tw, u channel, coarse channel
  const float* b;             // [C1] fp32 bias
  int C, kpad;                // coarse channels (32, 64 or 128), weight row pitch
};

// Weight gradient fused into a row-window data gradient (conv_dw.hip): the data
// gradient dX = conv(dY, W_flipped) of a 3x3 conv stages the dY halo image of each window
// in LDS; the same image gives the conv's weight-gradient partials
//   dW[tap][ci][co] += sum_{q in window} x[q][ci] dY[q - tap + 1][co]
// against the window's own pixels of the conv's forward input x -- dY is read once for
// both.  Each workgroup walks a contiguous window range, keeps its dW partial in
// registers and writes one fp32 slab row (the wgrad_win slab layout, reduced in fixed
// order by multi_reduce).  x == nullptr: off.
struct FusedWgrad {
  const void* x;              // [N][H][W][Cx] 16-bit forward input of the conv
  float* slab;                // [split_lo + nsplit rows at least][9][Cx][C1] fp32
  float* bias_slab;           // [.. rows][C1] fp32 column sums of dY (the bias gradient)
  int Cx, nsplit, split_lo;   // x channels, workgroups (slab rows) of this launch, first row
};

// Implicit-GEMM "NT" convolution: out[q][n] = epilogue(sum_{tap,c} X[q*s + tap - pad][c] * W[n][tap][c])
// GEMM M = output pixels q over [N][OD][OH][OW], GEMM N = Cout, K = taps * Cin.
// One kernel serves: conv forward, conv dgrad (flipped/transposed weights),
// transposed-conv forward (1x1 GEMM + pixel-shuffle store) and transposed-conv
// dgrad (2x2 stride-2 conv).
struct ConvFwdParams {
  int N, OD, OH, OW;          // output grid (GEMM rows)
  int ID, IH, IW;             // input grid, full-resolution coordinates
  int KD, KH, KW, stride, pad;
  int C1, C2;                 // input channels read from src1 / src2 (concat-free skip)
  int up1;                    // src1 is stored at 1/up1 resolution (nearest upsample fold)
  const void* src1;
  const void* src2;
  const void* wgt;            // bf16 [Cout][Kpad], row = (tap, channel), zero padded to a multiple of 64
  const float* bias;          // [Cout] or nullptr
  int Cout;
  int relu;
  float out_scale;
  float drop_rate;            // >0: inverted dropout on the output
  uint32_t seed, salt;
  // element-index offset of the dropout hash: a launch over images [c nb, ..) of a batch
  // draws the keep-mask of those elements of the whole-batch launch (two-stream forward)
  unsigned long long drop_idx0;
  const uint32_t* seed_ptr;   // non-null: the per-step seed is read from device memory
                              // (HIP-graph replay, where kernel arguments are frozen)
  void* dst1;                 // channels [0, D1)
  void* dst2;                 // channels [D1, Cout)
  int D1;
  const void* mask1;          // nullptr or tensor shaped like dst1: out *= (mask1 > 0)
  const void* mask2;
  float mask_scale1, mask_scale2;
  int shuffle;                // 0, or number of upsampled dims (2/3): tconv pixel shuffle
  // Fused normalisation statistics (deterministic: per-tile partial sums, no atomics).
  // stats: nullptr or [rows][2][Cout] -- one row per M tile of the launch
  // (conv_stat_tiles).  Forward (EPI_STATS): row = {sum z, sum z^2} of the tile's
  // bf16-rounded outputs.  Data gradient (EPI_DGRAD_NORM): {sum g, sum g * nz}.
  float* stats;
  // EPI_DGRAD_NORM: the destination is the gradient of a normalised activation
  // y = dropout(relu(u)), u = na * nz + nc; the gradient is masked by u > 0 and the
  // forward's dropout keep (recomputed from nd_rate / seed / nd_salt, scaled by
  // 1 / (1 - nd_rate)).  na / nc: [Cout] (BatchNorm, ncs = 0) or [N][Cout]
  // (GroupNorm, ncs = Cout; pixel q's sample is q / npix).
  const void* nz;
  const float* na;
  const float* nc;
  int ncs, npix;
  float nd_rate;
  uint32_t nd_salt;
  // Fused 2x2 max-pool (row-window forward of a convNb, EPI_FWD): the epilogue also
  // writes the pooled tensor [N][H/2][W/2][Cout] and the first-argmax codes of
  // elementwise.hip::maxpool2_fwd (one uint32 per pooled pixel x 8 channels), so the
  // separate pool launch and its full re-read of the conv output disappear.
  void* pool_dst;
  uint32_t* pool_code;
  // ReLU bit masks, 1 bit per element: [pixels][C / 8] bytes, bit e of byte b set when
  // channel 8b + e of the stored 16-bit activation is > 0.  relu_bits: written by a ReLU
  // forward (generic / EPI_FWD epilogue).  mask_bits bit 0 / 1: mask1 / mask2 point to
  // such bit tensors instead of activations -- the data gradient's ReLU mask then costs
  // 1/16 of the bytes of re-reading the activation.
  uint8_t* relu_bits;
  int mask_bits;
  // Fused 2x2 max-pool backward in a data gradient (2D row-window EPI_DGRAD, the skip
  // half of a decoder conv's dgrad, deferred until the pool's output gradient exists):
  // the epilogue adds route_gy[pooled pixel][c] where this pixel is the first argmax of
  // its window and the maximum is positive (pool_code, maxpool2_fwd layout) -- the
  // gradient of the convNb output in one pass, no separate skip-gradient tensor.
  const void* route_gy;
  // Operand transform on load (2D row-window conv, src1 only): the halo image is
  // rewritten in LDS before the MFMAs, so a normalisation pass never runs on its own --
  //   xform 1: src1 = pre-norm z, operand y = relu(xa z + xb)   (forward of a normalised
  //            activation's consumer; eval / train alike)
  // coefficients [C] (xcs = 0, BatchNorm) or [N][C] (xcs = C, GroupNorm; a window lies
  // in one sample); xc / xz are unused by the conv.  xout (optional): the transformed operand's own-window rows are also
  // stored there (the weight gradient reads them), by output-channel tile 0.
  int xform, xcs;
  const float* xa;
  const float* xb;
  const float* xc;
  const void* xz;
  void* xout;
  // xform 1 with the source layer's inverted dropout (its keep mask from drop_hash of the
  // element index xd_idx0 + pixel * C1 + channel, seed / seed_ptr, salt xd_salt): the
  // operand is dropout(relu(xa z + xb)), what norm_apply would have stored
  float xd_rate;
  uint32_t xd_salt;
  unsigned long long xd_idx0;
  // skip source (src2) normalised on load, y2 = relu(x2a z2 + x2b) ([C2] or [N][C2], x2cs):
  // the persistent tconv-on-load window only (conv_win_pfu_kernel; conv9a of the normalised
  // configs, whose skip activation is then never stored)
  const float* x2a;
  const float* x2b;
  int x2cs;
  int tile;                  // 0 = auto, else forced tile config id (tuning / A-B tests)
  // Fused segmentation head (row-window forward, Cout == 32, EPI_FWD only): per pixel
  // z = sum_c out[c] head_w[c] + head_b -> head_logit (fp32) for head_finish
  const float* head_w;
  const float* head_b;
  float* head_logit;
  // Mask weight-gradient sums in the forward (conv_win_pf_kernel with the fused head): per
  // pixel u = t p (1 - p), v = p (1 - p), w = p - t (p = sigmoid(logit), t = head_t) and
  // one row per workgroup of head_ws: {sum u y_c, sum v y_c, sum w y_c} (3 x 32 channel-major
  // blocks), sum u, sum v, sum w, pad -- head.hip head_wsum_grad turns them into the Mask
  // gradients once the loss sums are known.  head_nostore: the activation itself is not
  // stored (its ReLU bits are): nothing else reads it.
  const void* head_t;
  float* head_ws;
  int head_nostore;
  int rev;                    // row-window kernels: windows in reverse order (the consumer starts
                              // where its producer ended, on the tail still in the Infinity Cache)
  int win_pf;                 // > 0: 2D 128-wide 32 -> 32 channel row windows run persistently,
                              // win_pf consecutive windows per workgroup (conv_win_pf_kernel)
  int win_cp;                 // >= 1: 64-channel row windows of 64-wide rows with two or more input
                              // chunks load the next chunk under the current one's MFMAs
                              // (conv_win_cp_kernel); >= 2: also 128-wide rows, 3D or two or more
                              // chunks (conv_win_cp128_kernel)
  HeadGrad hg;                // 2D row-window data gradient of the head input: src1 (dY) formed
                              // on load (one 32-channel chunk), see HeadGrad
  // Space-to-depth source (2D row-window, composite transposed-conv data gradient):
  // s2d = C > 0 -> src1 is a FINE [N][2H][2W][C] tensor read as the coarse H x W image
  // with 4C channels (a, b, c) = src1[2h + a][2w + b][c]; C1 = 4C.  Each 32-channel chunk
  // lies in one phase group (a, b) whose 3x3 taps are structurally zero outside the 2x2
  // support dh in {1 - a, 2 - a}, dw in {1 - b, 2 - b}: those MFMAs are skipped.
  int s2d;
  TconvSrc ut;                // src1 = transposed conv of ut.x formed on load (see TconvSrc)
  FusedWgrad fw;              // weight-gradient partials from the same dY halo (see FusedWgrad)
  // filled by conv_fwd_prepare (host): K padded to 64, per-tap pixel deltas / offsets
  int Kpad;
  int tap_delta[27];
  signed char tap_d[27], tap_h[27], tap_w[27];
};

// "TN" weight-gradient GEMM with split-K over pixels:
//   slab[split][tap][m][n] = sum_{q in split} A[q*s + tap - pad][m] * B[q][n]
// conv 3x3:  A = layer input X (m = Cin), B = dY_pre (n = Cout)  -> HWIO
// tconv 2x2: A = dOut (m = Cout),         B = layer input (n = Cin) -> (kh,kw,Cout,Cin)
struct WgradParams {
  int N, QD, QH, QW;          // pixel grid of B (the K dimension)
  int AD, AH, AW;             // spatial grid of A
  int KD, KH, KW, stride, pad;
  int M1, M2;                 // A channels from a1 / a2 (concat input of decoder convs)
  int upA;                    // a1 stored at 1/upA resolution
  const void* a1;
  const void* a2;
  const void* b;              // [Q][Nc]
  int Nc;
  int splits;                 // K splits (grid dim)
  int split_lo, split_n;      // this launch runs splits [split_lo, split_lo + split_n) (split_n 0 = to the
                              // end): a weight gradient issued in parts as its dY is produced
  int tap_groups;             // taps handled per WG = (KD*KH*KW)/tap_groups
  int xcd;                    // set by wgrad_launch: bit 0 = window kernels, bit 1 = tiled kernel map
                              // logical workgroups to XCDs in contiguous runs (common.h xcd_remap)
  float* slab;                // [splits][taps][M][Nc] fp32
  // fused bias gradient: 0 = off, 1 = column sums of B (conv: dY -> n),
  // 2 = column sums of A over the WG's taps (tconv: dOut -> m)
  int bias_mode;
  float* bias_slab;           // [splits][tap_groups][M or Nc] fp32
  int win;                    // 0 = row-window kernel when eligible, -1 = never (A/B tests)
  // xform 2 (first-layer window wgrad): b = g (gradient of the normalised output) and the
  // B operand dz = xa g + xb z + xc (z = xz, the pre-norm output) is formed in LDS -- the
  // norm backward's dz of the first layer, read by nothing else, is never materialised
  // (coefficients [Nc] or [N][Nc], xcs = Nc).
  int xform, xcs;
  const float* xa;
  const float* xb;
  const float* xc;
  const void* xz;
  HeadGrad hg;                // window wgrad of the head input conv: the B operand (dY, 32 channels)
                              // formed on load, see HeadGrad
  int pair;
  // 128-wide row-window weight gradient with register prefetch of the next window
  // (conv_wgrad.hip wgrad_pf128_kernel; option wg_pf)
  int pf;                   // window wgrad, 32-channel output blocks on column-unit rows: wave-pair
                              // partials (conv_wgrad.hip wgrad_win_kernel PAIR, three workgroups per CU)
  // filled by the launcher
  int lqw, lqh, lqd;          // log2 of the pixel grid (power-of-two fast path)
  signed char tap_d[27], tap_h[27], tap_w[27];
};

// fp32 path (f32.hip): implicit-GEMM convolution out[q][n] = epi(sum_k A[q][k] W[k][n]),
// A = im2col of src1 | src2 (k = tap * (C1 + C2) + c, forward-conv tap semantics:
// input = output * stride + tap - pad), W = [K][Cout] row-major (the TF HWIO kernel
// flattened, or a transposed / flipped copy for data gradients and transposed convs).
struct F32Conv {
  int N, OD, OH, OW, ID, IH, IW, KD, KH, KW, stride, pad;
  int C1, C2, Cout;
  const float* src1;
  const float* src2;
  const float* wgt;
  const float* bias;           // [Cout] (shuffle: [Cout >> shuffle]) or nullptr
  float* dst;
  int relu;
  float drop_rate;             // inverted dropout (drop_hash of the bf16 path)
  uint32_t seed, salt;
  unsigned long long drop_idx0;
  const uint32_t* seed_ptr;
  const float* mask;           // consumer ReLU mask: out = mask > 0 ? out * mask_scale : 0
  float mask_scale;
  int shuffle;                 // 2 / 3: transposed-conv pixel-shuffle store, Cout = taps * channels
  int ldw;                     // weight row stride (>= Cout: a column range of a wider kernel)
};

// fp32 weight gradient: slab[split][tap][m][n] = sum_{q in split} A[q * stride + tap - pad][m] B[q][n]
struct F32Wgrad {
  int N, QD, QH, QW, AD, AH, AW, KD, KH, KW, stride, pad;
  int M1, M2, Nc;
  const float* a1;
  const float* a2;
  const float* b;
  float* slab;                 // [splits][taps][M1 + M2][Nc]
  int splits;
};

// Tile configuration chosen for a wgrad problem (shared with the host planner).
struct WgradCfg {
  int BM, BN, NTAP, smallc;
};

// One gradient of a batched slab reduction (conv_wgrad.hip::multi_reduce*).  Built on
// the host (runtime/native_engine.py mirrors this layout, 96 bytes).
struct ReduceJob {
  const float* slab;     // [splits][n4 * 4]
  float* out;            // [n4o * 4]
  float* stage;          // [groups][n4 * 4] (unused when direct)
  long long n4, n4o;     // float4 elements per split / of the output
  long long p1_begin;    // first global thread index of phase 1 (groups * n4 threads)
  long long p2_begin;    // first global thread index of phase 2 (n4o threads)
  int splits, groups;
  int taps, Mtot, Mout, Nc;
  int rg, rkeep;
  int direct, pad_;
};

// Segment descriptor of the fused Adam + bf16 repack kernel (adam.hip).
struct PackSeg {
  int off, n;          // element range in the flat master buffer
  int kind;            // 0 = none (bias / fp32-only), 1 = conv, 2 = tconv
  int T, Ci, Co;       // taps, input/output channels (TF kernel semantics)
  int Ci_pad, rowstride;  // fwd copy: row length (K padded to 64)
  int dg_rowstride, pad_;  // dgrad copy: row length
  long long fwd_off;   // element offset into the bf16 weight arena, -1 = none
  long long dg_off;    // dgrad copy, -1 = none
};

}  // namespace unet_types

namespace unet {
using namespace unet_types;
}  // namespace unet
