// Head-on-load: the gradient of the segmentation head's input, formed where it is
// consumed (conv_params.h HeadGrad).  The formula is the one of head.hip's backward
// (`model.py:13-21` -log Dice, optional BCE):
//   dL/dp      = -2 t / (2I + 1) + 1 / (St + Sp + 1)
//   dlogit     = g (dL/dp p (1 - p) + bce_w (p - t) / P_total)         (g: loss scale)
//   dY[p][c]   = dlogit(p) w[c] (x[p][c] > 0)                          (ReLU of the head input)
// dY is rank-1 per pixel, so a consumer reads 10 bytes per pixel (probability, target,
// 32 ReLU bits) instead of the 64-byte materialised gradient.
#pragma once
#include "common.h"
#include "conv_params.h"

namespace unet {

__device__ __forceinline__ float head_dlogit(float pr, float tv, float a, float bb, float inv_total, float bce_w,
                                             float gscale) {
  // explicit fused multiply-adds: every kernel that inlines this rounds identically
  // (a contraction left to the compiler may differ between call sites)
  const float dice = __builtin_fmaf(a, tv, bb) * pr * (1.f - pr);
  return __builtin_fmaf(bce_w * (pr - tv), inv_total, dice) * gscale;
}

// Normalised head input (head.hip norm_head_loss / head_norm_bwd): the logit gradient as
// al u + be v + ga w with u = t p (1 - p), v = p (1 - p), w = p - t and the batch scalars of
// hn_scalars -- explicit fused multiply-adds, so every kernel inlining it rounds alike
__device__ __forceinline__ float hn_dlogit(float pr, float tv, float al, float be, float ga) {
  const float vv = pr * (1.f - pr);
  return __builtin_fmaf(al * tv, vv, __builtin_fmaf(be, vv, ga * (pr - tv)));
}

// Per-launch constants (wave-uniform: scalar registers).  The head weights are loaded
// here, unconditionally: a load under the per-element ReLU-bit select compiles to a
// branch + scalar load + wait per element (a 128-deep serialised chain per window).
struct HeadGradCtx {
  float a, bb, inv_total, bce_w, gscale;
  float w[32];
};

__device__ __forceinline__ HeadGradCtx head_grad_ctx(const HeadGrad& hg) {
  HeadGradCtx c;
  const float I = hg.sums[0], St = hg.sums[1], Sp = hg.sums[2];
  c.a = -2.f / (2.f * I + 1.f);
  c.bb = 1.f / (St + Sp + 1.f);
  c.inv_total = hg.inv_total;
  c.bce_w = hg.bce_w;
  c.gscale = hg.gscale ? *hg.gscale : 1.f;
#pragma unroll
  for (int k = 0; k < 32; ++k) c.w[k] = hg.w[k];
  return c;
}

// dY of pixel `pix` of a 32-channel head input as four 16-byte chunks (chunk k = channels
// 8k .. 8k + 7), rounded exactly like head.hip::head_bwd_kernel's stored gradient
__device__ __forceinline__ void head_grad_pixel(const HeadGrad& hg, const HeadGradCtx& c, int pix, u32x4 (&out)[4]) {
  const float pr = hg.prob[pix];
  const float tv = bits2f(((const uint16_t*)hg.t)[pix]);
  const float dz = head_dlogit(pr, tv, c.a, c.bb, c.inv_total, c.bce_w, c.gscale);
  const uint32_t m = ((const uint32_t*)hg.bits)[pix];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float v = dz * c.w[8 * k + e];
      o[e] = ((m >> (8 * k + e)) & 1u) ? v : 0.f;
    }
    out[k] = pack8(o);
  }
}

}  // namespace unet
