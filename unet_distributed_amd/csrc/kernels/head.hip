// Fused segmentation head + loss on gfx950 (16-byte lanes: C/8 lanes per pixel).
//
// Forward (`model.py:119-120` Mask 1x1 conv + sigmoid, `model.py:4-21` Dice):
//   z_p = sum_c x[p][c] w[c] + b;   prob_p = sigmoid(z_p)
//   per-block partials of {I = sum t*p, St = sum t, Sp = sum p, BCE = sum bce(z, t)}
//   then ONE deterministic block reduces the partials -> sums[4] on device
//   (no host sync; metrics are read lazily by the logger).
// Backward:
//   dL/dp = -2 t / (2I + 1) + 1 / (St + Sp + 1)              (-log Dice)
//   dz    = g * (dL/dp * p (1 - p) + bce_w * (p - t) / P_total)
//   dx[p][c] = dz w[c] * (x[p][c] > 0)   (ReLU of conv9b folded in)
//   dW[c] = sum dz x[p][c], db = sum dz   -> per-block partials, reduced deterministically.
#include "common.h"
#include "head_grad.h"

namespace unet {

namespace {

constexpr int HT = 256;

// Forward: one thread per pixel (the sigmoid / BCE transcendentals then run once per
// pixel on full waves; a lane-per-chunk mapping measured 2x slower here).
template <int C>
__global__ void __launch_bounds__(HT) head_fwd_kernel(const h16* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ b, const h16* __restrict__ t,
                                                      int P, float* __restrict__ prob, float* __restrict__ partial) {
  __shared__ float red[4][HT / 64];
  float wr[C];
#pragma unroll
  for (int c = 0; c < C; ++c) wr[c] = w[c];
  const float bias = b[0];
  float sI = 0.f, sT = 0.f, sP = 0.f, sB = 0.f;
  for (int p = blockIdx.x * HT + threadIdx.x; p < P; p += gridDim.x * HT) {
    float z = bias;
#pragma unroll
    for (int c8 = 0; c8 < C / 8; ++c8) {
      float f[8];
      unpack8(*(const u32x4*)(x + (size_t)p * C + c8 * 8), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) z += f[e] * wr[c8 * 8 + e];
    }
    const float pr = 1.f / (1.f + __expf(-z));
    prob[p] = pr;
    if (t) {
      const float tv = (float)t[p];
      sI += tv * pr;
      sT += tv;
      sP += pr;
      sB += fmaxf(z, 0.f) - z * tv + log1pf(__expf(-fabsf(z)));
    } else {
      sP += pr;
    }
  }
  sI = wave_sum(sI);
  sT = wave_sum(sT);
  sP = wave_sum(sP);
  sB = wave_sum(sB);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = sI;
    red[1][wv] = sT;
    red[2][wv] = sP;
    red[3][wv] = sB;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int k = 0; k < HT / 64; ++k) s += red[threadIdx.x][k];
    partial[blockIdx.x * 4 + threadIdx.x] = s;
  }
}

// Finish of the fused head: prob holds the fp32 logits written by the head-input
// conv's epilogue (conv_epilogue.h); sigmoid in place and the same per-block
// {I, St, Sp, BCE} partials as head_fwd_kernel.
__global__ void __launch_bounds__(HT) head_finish_kernel(float* __restrict__ prob, const h16* __restrict__ t, int P,
                                                         float* __restrict__ partial) {
  __shared__ float red[4][HT / 64];
  float sI = 0.f, sT = 0.f, sP = 0.f, sB = 0.f;
  auto one = [&](float z, float tv, bool has_t) -> float {
    const float pr = 1.f / (1.f + __expf(-z));
    if (has_t) {
      sI += tv * pr;
      sT += tv;
      sP += pr;
      sB += fmaxf(z, 0.f) - z * tv + log1pf(__expf(-fabsf(z)));
    } else {
      sP += pr;
    }
    return pr;
  };
  // 4 pixels per thread (16-byte logit / 8-byte target accesses), scalar tail
  const int P4 = P >> 2;
  for (int i = blockIdx.x * HT + threadIdx.x; i < P4; i += gridDim.x * HT) {
    f32x4 z = ((const f32x4*)prob)[i];
    float tv[4] = {0.f, 0.f, 0.f, 0.f};
    if (t) {
      const u32x2 tw = ((const u32x2*)t)[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) tv[e] = bits2f((uint16_t)(tw[e >> 1] >> (16 * (e & 1))));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) z[e] = one(z[e], tv[e], t != nullptr);
    ((f32x4*)prob)[i] = z;
  }
  for (int p = 4 * P4 + blockIdx.x * HT + threadIdx.x; p < P; p += gridDim.x * HT)
    prob[p] = one(prob[p], t ? (float)t[p] : 0.f, t != nullptr);
  sI = wave_sum(sI);
  sT = wave_sum(sT);
  sP = wave_sum(sP);
  sB = wave_sum(sB);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = sI;
    red[1][wv] = sT;
    red[2][wv] = sP;
    red[3][wv] = sB;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
    for (int k = 0; k < HT / 64; ++k) s += red[threadIdx.x][k];
    partial[blockIdx.x * 4 + threadIdx.x] = s;
  }
}

// out[j] = sum_b partial[b][j]: one block per column j (row stride `width`), fixed order
__global__ void __launch_bounds__(256) partial_reduce_kernel(const float* __restrict__ partial, int nb, int width,
                                                             float* __restrict__ out) {
  __shared__ float red[256];
  const int j = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nb; k += 256) s += partial[(size_t)k * width + j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = red[0];
}

template <int C>
__global__ void __launch_bounds__(HT) head_bwd_kernel(const h16* __restrict__ x, const float* __restrict__ w,
                                                      const float* __restrict__ prob, const h16* __restrict__ t,
                                                      const float* __restrict__ sums, int P, float inv_total,
                                                      float bce_w, float gscale, const float* __restrict__ gscale_ptr,
                                                      h16* __restrict__ dx, float* __restrict__ partial) {
  constexpr int CP = C / 8;
  if (gscale_ptr) gscale = *gscale_ptr;      // loss scale kept on the device (fp16 dynamic scaling)
  __shared__ float red[HT / 64][C + 1];
  const int cc = threadIdx.x % CP;
  float wr[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) wr[e] = w[cc * 8 + e];
  const float I = sums[0], St = sums[1], Sp = sums[2];
  const float a = -2.f / (2.f * I + 1.f);
  const float bb = 1.f / (St + Sp + 1.f);
  float gw[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float gb = 0.f;
  const long long total = (long long)P * CP;
  for (long long i = blockIdx.x * (long long)HT + threadIdx.x; i < total; i += (long long)gridDim.x * HT) {
    const int p = (int)(i / CP);
    const float pr = prob[p];
    const float tv = (float)t[p];
    const float dz = head_dlogit(pr, tv, a, bb, inv_total, bce_w, gscale);
    if (cc == 0) gb += dz;
    float f[8], o[8];
    unpack8(*(const u32x4*)(x + i * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      gw[e] += dz * f[e];
      o[e] = f[e] > 0.f ? dz * wr[e] : 0.f;      // ReLU of the head's input folded in
    }
    // dx == nullptr (head-on-load): the consumers form dx themselves (head_grad.h); only
    // the head's weight / bias gradients are reduced here
    if (dx) *(u32x4*)(dx + i * 8) = pack8(o);
  }
  // lanes l, l + CP, l + 2CP, ... hold the same channels: fold them, then across waves
#pragma unroll
  for (int e = 0; e < 8; ++e)
#pragma unroll
    for (int o = CP; o < 64; o <<= 1) gw[e] += __shfl_xor(gw[e], o, 64);
  gb = wave_sum(gb);
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (ln < CP) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[wv][ln * 8 + e] = gw[e];
  }
  if (ln == 0) red[wv][C] = gb;
  __syncthreads();
  for (int j = threadIdx.x; j <= C; j += HT) {
    float s = 0.f;
    for (int k = 0; k < HT / 64; ++k) s += red[k][j];
    partial[(size_t)blockIdx.x * (C + 1) + j] = s;
  }
}

// dY of the head input from its ReLU bits (head_wsum without head-on-load: the fused-head
// forward stores neither the head input nor needs it here -- the Mask gradients come from its
// sums): dx[p][c] = dlogit(p) w[c] where bit c of pixel p is set, head_bwd_kernel's values.
// bits: C / 8 bytes per pixel (byte = channel chunk, bit e = channel 8 chunk + e).
template <int C>
__global__ void __launch_bounds__(HT) head_dy_kernel(const uint8_t* __restrict__ bits, const float* __restrict__ w,
                                                     const float* __restrict__ prob, const h16* __restrict__ t,
                                                     const float* __restrict__ sums, int P, float inv_total,
                                                     float bce_w, float gscale, const float* __restrict__ gscale_ptr,
                                                     h16* __restrict__ dx) {
  constexpr int CP = C / 8;
  if (gscale_ptr) gscale = *gscale_ptr;
  const int cc = threadIdx.x % CP;
  float wr[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) wr[e] = w[cc * 8 + e];
  const float I = sums[0], St = sums[1], Sp = sums[2];
  const float a = -2.f / (2.f * I + 1.f);
  const float bb = 1.f / (St + Sp + 1.f);
  const int total = P * CP;                            // < 2^31 (head_check / planner)
  for (int i = blockIdx.x * HT + threadIdx.x; i < total; i += gridDim.x * HT) {
    const int p = i / CP;
    const float dz = head_dlogit(prob[p], (float)t[p], a, bb, inv_total, bce_w, gscale);
    const uint32_t m = bits[i];
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = ((m >> e) & 1u) ? dz * wr[e] : 0.f;
    *(u32x4*)(dx + (size_t)i * 8) = pack8(o);
  }
}

// Mask gradients from the forward's sums (conv_params.h head_ws; conv_win_pf_kernel with the
// fused head): head_grad.h's dlogit = A u + B v + G w per pixel with the batch scalars
// A = a gs, B = bb gs, G = bce_w inv_total gs, so
//   grad_w[c] = A sum u y_c + B sum v y_c + G sum w y_c,   grad_b = A sum u + B sum v + G sum w
// -- the head input need not be re-read (nor stored).  Block j < 32: channel j, block 32:
// the bias; fixed-order column sums over the rows.
__global__ void __launch_bounds__(256) head_wsum_grad_kernel(const float* __restrict__ rows, int nr,
                                                             const float* __restrict__ sums, float inv_total,
                                                             float bce_w, float gscale,
                                                             const float* __restrict__ gscale_ptr,
                                                             float* __restrict__ gw, float* __restrict__ gb) {
  __shared__ float red[3][256];
  if (gscale_ptr) gscale = *gscale_ptr;
  const int j = blockIdx.x;
  float s[3] = {0.f, 0.f, 0.f};
  for (int k = threadIdx.x; k < nr; k += 256) {
#pragma unroll
    for (int m = 0; m < 3; ++m) s[m] += rows[(size_t)k * 100 + (j < 32 ? 32 * m + j : 96 + m)];
  }
#pragma unroll
  for (int m = 0; m < 3; ++m) red[m][threadIdx.x] = s[m];
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
#pragma unroll
      for (int m = 0; m < 3; ++m) red[m][threadIdx.x] += red[m][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float I = sums[0], St = sums[1], Sp = sums[2];
    const float a = -2.f / (2.f * I + 1.f);
    const float bb = 1.f / (St + Sp + 1.f);
    const float g = (a * gscale) * red[0][0] + (bb * gscale) * red[1][0] + (bce_w * inv_total * gscale) * red[2][0];
    if (j < 32)
      gw[j] = g;
    else
      gb[0] = g;
  }
}

// grad_w[c] = sum_b partial[b][c], grad_b = sum_b partial[b][C]: one block per column
__global__ void __launch_bounds__(256) head_grad_reduce_kernel(const float* __restrict__ partial, int nb, int C,
                                                               float* __restrict__ gw, float* __restrict__ gb) {
  __shared__ float red[256];
  const int j = blockIdx.x;
  float s = 0.f;
  for (int k = threadIdx.x; k < nb; k += 256) s += partial[(size_t)k * (C + 1) + j];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    if (j < C)
      gw[j] = red[0];
    else
      gb[0] = red[0];
  }
}

}  // namespace

int head_blocks(int P) {
  int nb = (P + HT - 1) / HT;
  if (nb > 1024) nb = 1024;
  if (nb < 1) nb = 1;
  return nb;
}

const char* head_check(int C) {
  if (C != 32 && C != 64 && C != 16) return "head: feature channels must be 16, 32 or 64";
  return nullptr;
}

hipError_t head_fwd_launch(const void* x, const float* w, const float* b, const void* t, int P, int C, float* prob,
                           float* partial, float* sums, hipStream_t s) {
  const int nb = head_blocks(P);
  switch (C) {
    case 16:
      UNET_LAUNCH(head_fwd_kernel<16>, dim3(nb), dim3(HT), 0, s, (const h16*)x, w, b, (const h16*)t, P,
                         prob, partial);
      break;
    case 32:
      UNET_LAUNCH(head_fwd_kernel<32>, dim3(nb), dim3(HT), 0, s, (const h16*)x, w, b, (const h16*)t, P,
                         prob, partial);
      break;
    default:
      UNET_LAUNCH(head_fwd_kernel<64>, dim3(nb), dim3(HT), 0, s, (const h16*)x, w, b, (const h16*)t, P,
                         prob, partial);
  }
  UNET_LAUNCH(partial_reduce_kernel, dim3(4), dim3(256), 0, s, partial, nb, 4, sums);
  return launch_status();
}

hipError_t head_bwd_launch(const void* x, const float* w, const float* prob, const void* t, const float* sums, int P,
                           int C, float inv_total, float bce_w, float gscale, const float* gscale_ptr, void* dx,
                           float* partial, float* gw, float* gb, hipStream_t s) {
  const int nb = head_blocks(P);
  switch (C) {
    case 16:
      UNET_LAUNCH(head_bwd_kernel<16>, dim3(nb), dim3(HT), 0, s, (const h16*)x, w, prob, (const h16*)t,
                         sums, P, inv_total, bce_w, gscale, gscale_ptr, (h16*)dx, partial);
      break;
    case 32:
      UNET_LAUNCH(head_bwd_kernel<32>, dim3(nb), dim3(HT), 0, s, (const h16*)x, w, prob, (const h16*)t,
                         sums, P, inv_total, bce_w, gscale, gscale_ptr, (h16*)dx, partial);
      break;
    default:
      UNET_LAUNCH(head_bwd_kernel<64>, dim3(nb), dim3(HT), 0, s, (const h16*)x, w, prob, (const h16*)t,
                         sums, P, inv_total, bce_w, gscale, gscale_ptr, (h16*)dx, partial);
  }
  UNET_LAUNCH(head_grad_reduce_kernel, dim3(C + 1), dim3(256), 0, s, partial, nb, C, gw, gb);
  return launch_status();
}

hipError_t head_dy_launch(const void* bits, const float* w, const float* prob, const void* t, const float* sums, int P,
                          int C, float inv_total, float bce_w, float gscale, const float* gscale_ptr, void* dx,
                          hipStream_t s) {
  if ((long long)P * (C / 8) >= (1LL << 31)) return hipErrorInvalidValue;
  const int nb = head_blocks(P);
  switch (C) {
    case 16:
      UNET_LAUNCH(head_dy_kernel<16>, dim3(nb), dim3(HT), 0, s, (const uint8_t*)bits, w, prob, (const h16*)t, sums,
                  P, inv_total, bce_w, gscale, gscale_ptr, (h16*)dx);
      break;
    case 32:
      UNET_LAUNCH(head_dy_kernel<32>, dim3(nb), dim3(HT), 0, s, (const uint8_t*)bits, w, prob, (const h16*)t, sums,
                  P, inv_total, bce_w, gscale, gscale_ptr, (h16*)dx);
      break;
    default:
      UNET_LAUNCH(head_dy_kernel<64>, dim3(nb), dim3(HT), 0, s, (const uint8_t*)bits, w, prob, (const h16*)t, sums,
                  P, inv_total, bce_w, gscale, gscale_ptr, (h16*)dx);
  }
  return launch_status();
}

hipError_t head_wsum_grad_launch(const float* rows, int nrows, const float* sums, float inv_total, float bce_w,
                                 float gscale, const float* gscale_ptr, float* gw, float* gb, hipStream_t s) {
  UNET_LAUNCH(head_wsum_grad_kernel, dim3(33), dim3(256), 0, s, rows, nrows, sums, inv_total, bce_w, gscale,
              gscale_ptr, gw, gb);
  return launch_status();
}

hipError_t partial_reduce_launch(const float* partial, int nb, int width, float* out, hipStream_t s) {
  UNET_LAUNCH(partial_reduce_kernel, dim3(width), dim3(256), 0, s, partial, nb, width, out);
  return launch_status();
}

// Normalised head input in one pass (norm mode): y = relu(fa z + fc) of the head's
// input conv is stored (the head backward reads it) and the 1x1 head's logit
// sum_c y[c] w[c] + b is written to `logit` (head_finish turns it into probabilities
// and loss partials) -- head_fwd's full re-read of y disappears.  The CP = C / 8 lanes
// of a pixel are adjacent; their partial dots are combined by xor shuffles.
template <int C>
__global__ void __launch_bounds__(HT) norm_head_kernel(const h16* __restrict__ z, const float* __restrict__ fa,
                                                       const float* __restrict__ fc, int cstride, int npix,
                                                       const float* __restrict__ w, const float* __restrict__ b,
                                                       int P, h16* __restrict__ y, float* __restrict__ logit) {
  constexpr int CP = C / 8;
  const int cc = threadIdx.x % CP;
  float wr[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) wr[e] = w[cc * 8 + e];
  const float bias = b[0];
  const long long total = (long long)P * CP;
  for (long long i = blockIdx.x * (long long)HT + threadIdx.x; i < total; i += (long long)gridDim.x * HT) {
    const int p = (int)(i / CP);
    const size_t cb = (size_t)(p / npix) * cstride + cc * 8;
    float f[8];
    unpack8(*(const u32x4*)(z + i * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(fa[cb + e], f[e], fc[cb + e]), 0.f);
    const u32x4 v = pack8(f);
    *(u32x4*)(y + i * 8) = v;
    unpack8(v, f);
    float d = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) d += f[e] * wr[e];
#pragma unroll
    for (int o = 1; o < CP; o <<= 1) d += __shfl_xor(d, o, 64);
    if (cc == 0) logit[p] = d + bias;
  }
}

hipError_t norm_head_launch(const void* z, const float* fa, const float* fc, int cstride, int npix, const float* w,
                            const float* b, int P, int C, void* y, float* logit, hipStream_t s) {
  const int nb = head_blocks(P * (C / 8) / 4 + 1);
  switch (C) {
    case 16:
      UNET_LAUNCH(norm_head_kernel<16>, dim3(nb), dim3(HT), 0, s, (const h16*)z, fa, fc, cstride, npix, w, b,
                         P, (h16*)y, logit);
      break;
    case 32:
      UNET_LAUNCH(norm_head_kernel<32>, dim3(nb), dim3(HT), 0, s, (const h16*)z, fa, fc, cstride, npix, w, b,
                         P, (h16*)y, logit);
      break;
    default:
      UNET_LAUNCH(norm_head_kernel<64>, dim3(nb), dim3(HT), 0, s, (const h16*)z, fa, fc, cstride, npix, w, b,
                         P, (h16*)y, logit);
  }
  return launch_status();
}

// ---------------------------------------------------------------------------------
// Norm-mode training head: the loss and every pixel sum the head's backward needs are
// formed in the forward pass, so the backward reads the head input's z once.
//
// The logit gradient is linear in three per-pixel terms with batch-scalar weights,
//   dlogit_p = al u_p + be v_p + ga w_p,   u = t p (1 - p), v = p (1 - p), w = p - t,
//   al = -2 gs / (2 I + 1), be = gs / (St + Sp + 1), ga = gs bce_w / P_total
// (gs: loss scale), and the scalars are only known once the loss sums are.  So the
// sums the backward needs over pixels -- the 1x1 head's weight gradient sum_p dlogit y_c
// and the head input's norm-backward statistics {sum_p g_c, sum_p g_c z_c} of
// g_c = dlogit w_c m_c (m_c = [fa z + fc > 0], as the dgrad-norm epilogue recomputes it)
// -- are al/be/ga combinations of six per-channel sums {u, v, w} x {m, m z} that the
// forward accumulates beside the logits (y = m (fa z + fc), so sum dlogit y_c =
// fa_c sum dlogit m z + fc_c sum dlogit m: the weight gradient of the unrounded y).
// The backward is then
//   head_norm_coef:  rows [R][2][C] + head weight/bias gradient from the block partials
//   bn/gn_stats:     dz coefficients a, b, c (unchanged)
//   head_norm_bwd:   dz = a w dlogit m + b z + c  (dlogit from prob and t per pixel)
// replacing head_bwd (y read, dx written), the moments pass over (dx, z) and
// norm_bwd_apply (dx, z read).  The activation y itself need not be stored.
//
// Block partial row (hn_width(C) floats): [k][C] for k = 0..5 = U_m V_m W_m U_mz V_mz
// W_mz, then Su Sv Sw I St Sp BCE and one pad float.
// Grid (blocks per sample, N): the rows of sample n are consecutive (GroupNorm).
__host__ __device__ constexpr int hn_width(int C) { return 6 * C + 8; }

namespace {

__device__ __forceinline__ void hn_scalars(const float* __restrict__ sums, float inv_total, float bce_w, float gs,
                                           float& al, float& be, float& ga) {
  al = -2.f * gs / (2.f * sums[0] + 1.f);
  be = gs / (sums[1] + sums[2] + 1.f);
  ga = gs * bce_w * inv_total;
}

template <int C>
__global__ void __launch_bounds__(HT) __attribute__((amdgpu_waves_per_eu(2))) norm_head_loss_kernel(const h16* __restrict__ z, const float* __restrict__ fa,
                                                            const float* __restrict__ fc, int cstride, int npix,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            const h16* __restrict__ t, h16* __restrict__ y,
                                                            float* __restrict__ prob, float* __restrict__ partial) {
  constexpr int CP = C / 8, PPB = HT / CP, WD = hn_width(C);
  __shared__ float red[HT / 64][WD];
  const int n = blockIdx.y, nbp = gridDim.x, blk = blockIdx.x;
  const int cc = threadIdx.x % CP, pr0 = threadIdx.x / CP, c0 = cc * 8;
  float wr[8], A[8], B[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    wr[e] = w[c0 + e];
    A[e] = fa[(size_t)n * cstride + c0 + e];
    B[e] = fc[(size_t)n * cstride + c0 + e];
  }
  const float bias = b[0];
  float acc[6][8];
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[k][e] = 0.f;
  float su = 0.f, sv = 0.f, sw = 0.f, sI = 0.f, sT = 0.f, sP = 0.f, sB = 0.f;
  const int p0 = (int)((long long)blk * npix / nbp), p1 = (int)((long long)(blk + 1) * npix / nbp);
  const size_t sb = (size_t)n * npix;
  // per-pixel scalar terms (probability store, loss sums, BCE): one lane's share
  auto scalars = [&](const float zl, const float pr, const float tv, const size_t q) {
    const float vv = pr * (1.f - pr), uu = tv * vv, ww = pr - tv;
    prob[q] = pr;
    su += uu;
    sv += vv;
    sw += ww;
    sI += tv * pr;
    sT += tv;
    sP += pr;
    sB += fmaxf(zl, 0.f) - zl * tv + log1pf(__expf(-fabsf(zl)));
  };
  // channel sums of one pixel (every lane of the pixel holds its logit zl / probability pr)
  auto pixel = [&](const u32x4 raw, const float tv, const size_t q, float& zl_out, float& pr_out) {
    float zf[8], v[8], yv[8];
    unpack8(raw, zf);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = fmaf(A[e], zf[e], B[e]);
      yv[e] = fmaxf(v[e], 0.f);
    }
    const u32x4 yp = pack8(yv);
    if (y) *(u32x4*)(y + q * C + c0) = yp;
    unpack8(yp, yv);                                 // the logit of the stored 16-bit y
    float d = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) d += yv[e] * wr[e];
#pragma unroll
    for (int o = 1; o < CP; o <<= 1) d += __shfl_xor(d, o, 64);
    const float zl = d + bias;
    const float pr = 1.f / (1.f + __expf(-zl));
    const float vv = pr * (1.f - pr), uu = tv * vv, ww = pr - tv;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float m = v[e] > 0.f ? 1.f : 0.f;
      const float mz = m * zf[e];
      acc[0][e] = fmaf(m, uu, acc[0][e]);
      acc[1][e] = fmaf(m, vv, acc[1][e]);
      acc[2][e] = fmaf(m, ww, acc[2][e]);
      acc[3][e] = fmaf(mz, uu, acc[3][e]);
      acc[4][e] = fmaf(mz, vv, acc[4][e]);
      acc[5][e] = fmaf(mz, ww, acc[5][e]);
    }
    zl_out = zl;
    pr_out = pr;
  };
  // the CP lanes of one pixel are adjacent and always take the same path.  KU = CP pixel
  // steps per iteration, their loads issued before any is used (memory-level parallelism:
  // the per-pixel chain load -> dot -> shuffles -> sigmoid is long); the scalar terms of
  // step u are formed by lane cc = u of each pixel group, so the transcendental tail runs
  // once per pixel across the group instead of on one lane while the other CP - 1 idle
  // (it was most of the kernel's VALU time)
  // (KH groups of KU steps per iteration: 2 KU loads of 16 bytes in flight per lane -- with
  // one group the pass ran at 2.8 TB/s, latency-bound at two waves per SIMD)
  constexpr int KU = CP, KH = 2;
  int p = p0 + pr0;
  for (; p + (KH * KU - 1) * PPB < p1; p += KH * KU * PPB) {
    u32x4 raw[KH][KU];
    float tv[KH][KU];
#pragma unroll
    for (int h = 0; h < KH; ++h)
#pragma unroll
      for (int u = 0; u < KU; ++u) {
        const size_t q = sb + p + (h * KU + u) * PPB;
        raw[h][u] = *(const u32x4*)(z + q * C + c0);
        tv[h][u] = (float)t[q];
      }
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      float zl[KU], pr[KU];
#pragma unroll
      for (int u = 0; u < KU; ++u) pixel(raw[h][u], tv[h][u], sb + p + (h * KU + u) * PPB, zl[u], pr[u]);
      float zs = zl[0], ps = pr[0], ts = tv[h][0];
#pragma unroll
      for (int u = 1; u < KU; ++u) {
        zs = cc == u ? zl[u] : zs;
        ps = cc == u ? pr[u] : ps;
        ts = cc == u ? tv[h][u] : ts;
      }
      scalars(zs, ps, ts, sb + p + (h * KU + cc) * PPB);
    }
  }
  for (; p < p1; p += PPB) {
    const size_t q = sb + p;
    const float tq = (float)t[q];
    float zl, pr;
    pixel(*(const u32x4*)(z + q * C + c0), tq, q, zl, pr);
    if (cc == 0) scalars(zl, pr, tq, q);
  }
  // lanes l, l + CP, l + 2 CP, ... of a wave hold the same channels
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = CP; o < 64; o <<= 1) acc[k][e] += __shfl_xor(acc[k][e], o, 64);
  su = wave_sum(su);
  sv = wave_sum(sv);
  sw = wave_sum(sw);
  sI = wave_sum(sI);
  sT = wave_sum(sT);
  sP = wave_sum(sP);
  sB = wave_sum(sB);
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (ln < CP) {
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[wv][k * C + ln * 8 + e] = acc[k][e];
  }
  if (ln == 0) {
    float* r = &red[wv][6 * C];
    r[0] = su;
    r[1] = sv;
    r[2] = sw;
    r[3] = sI;
    r[4] = sT;
    r[5] = sP;
    r[6] = sB;
    r[7] = 0.f;
  }
  __syncthreads();
  float* out = partial + ((size_t)n * nbp + blk) * WD;
  for (int j = threadIdx.x; j < WD; j += HT) {
    float s = red[0][j];
#pragma unroll
    for (int k = 1; k < HT / 64; ++k) s += red[k][j];
    out[j] = s;
  }
}

// Blocks 0 .. C: head weight (j < C) / bias (j == C) gradient, column sums over the nb
// partial rows in a fixed order (row r belongs to sample r / nbp: fa / fc [C] or [N][C]).
// Blocks past C: norm-backward rows
//   rows[r][0][c] = w_c (al U_m + be V_m + ga W_m)[r][c],  rows[r][1][c] = w_c (... m z ...)
__global__ void __launch_bounds__(256) head_norm_coef_kernel(const float* __restrict__ partial, int nb, int nbp,
                                                             int C, const float* __restrict__ sums,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ fa,
                                                             const float* __restrict__ fc, int cstride,
                                                             float inv_total, float bce_w, float gscale,
                                                             const float* __restrict__ gscale_ptr,
                                                             float* __restrict__ rows, float* __restrict__ gw,
                                                             float* __restrict__ gb) {
  __shared__ float red[256];
  const float gs = gscale_ptr ? *gscale_ptr : gscale;
  float al, be, ga;
  hn_scalars(sums, inv_total, bce_w, gs, al, be, ga);
  const int WD = hn_width(C);
  if ((int)blockIdx.x <= C) {
    const int j = blockIdx.x;
    float s = 0.f;
    for (int k = threadIdx.x; k < nb; k += 256) {
      const float* r = partial + (size_t)k * WD;
      if (j < C) {
        const size_t ci = (size_t)(k / nbp) * cstride + j;
        s += fa[ci] * (al * r[3 * C + j] + be * r[4 * C + j] + ga * r[5 * C + j]) +
             fc[ci] * (al * r[j] + be * r[C + j] + ga * r[2 * C + j]);
      } else {
        s += al * r[6 * C] + be * r[6 * C + 1] + ga * r[6 * C + 2];
      }
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int h = 128; h > 0; h >>= 1) {
      if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (j < C)
        gw[j] = red[0];
      else
        gb[0] = red[0];
    }
    return;
  }
  const long long total = (long long)nb * C;
  for (long long i = (long long)(blockIdx.x - C - 1) * 256 + threadIdx.x; i < total;
       i += (long long)(gridDim.x - C - 1) * 256) {
    const int r = (int)(i / C), c = (int)(i - (long long)r * C);
    const float* pr = partial + (size_t)r * WD + c;
    rows[((size_t)r * 2 + 0) * C + c] = w[c] * (al * pr[0] + be * pr[C] + ga * pr[2 * C]);
    rows[((size_t)r * 2 + 1) * C + c] = w[c] * (al * pr[3 * C] + be * pr[4 * C] + ga * pr[5 * C]);
  }
}

// dz = a (w dlogit m) + b z + c for the head input (coefficients [C] or [N][C]); grid
// (blocks per sample, N), one 8-channel column per thread as norm_bwd_apply
__global__ void __launch_bounds__(256) head_norm_bwd_kernel(
    const h16* __restrict__ z, const float* __restrict__ prob, const h16* __restrict__ t,
    const float* __restrict__ sums, const float* __restrict__ w, const float* __restrict__ fa,
    const float* __restrict__ fc, const float* __restrict__ ca, const float* __restrict__ cb,
    const float* __restrict__ ccf, int cstride, int P, int C, float inv_total, float bce_w, float gscale,
    const float* __restrict__ gscale_ptr, h16* __restrict__ dz) {
  const int n = blockIdx.y, nbp = gridDim.x, blk = blockIdx.x;
  const int cpr = C / 8, rstep = 256 / cpr;
  const int cc = threadIdx.x % cpr, rs = threadIdx.x / cpr;
  if (rs >= rstep) return;
  const float gs = gscale_ptr ? *gscale_ptr : gscale;
  float al, be, ga;
  hn_scalars(sums, inv_total, bce_w, gs, al, be, ga);
  const int c0 = cc * 8;
  float aw[8], bz[8], c1[8], A[8], B[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const size_t k = (size_t)n * cstride + c0 + e;
    aw[e] = ca[k] * w[c0 + e];
    bz[e] = cb[k];
    c1[e] = ccf[k];
    A[e] = fa[k];
    B[e] = fc[k];
  }
  const int p0 = (int)((long long)blk * P / nbp), p1 = (int)((long long)(blk + 1) * P / nbp);
  const size_t sb = (size_t)n * P;
#pragma unroll 4
  for (int p = p0 + rs; p < p1; p += rstep) {
    const size_t q = sb + p;
    float zf[8];
    unpack8(*(const u32x4*)(z + q * C + c0), zf);
    const float dl = hn_dlogit(prob[q], (float)t[q], al, be, ga);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = fmaf(A[e], zf[e], B[e]) > 0.f ? aw[e] * dl : 0.f;
      zf[e] = g + fmaf(bz[e], zf[e], c1[e]);
    }
    *(u32x4*)(dz + q * C + c0) = pack8(zf);
  }
}

}  // namespace

int hn_blocks_per_sample(int N, int P) {
  int nbp = (4096 + N - 1) / N;
  const int maxb = (P + 255) / 256;
  if (nbp > maxb) nbp = maxb;
  return nbp < 1 ? 1 : nbp;
}

int hn_partial_floats(int N, int P, int C) { return N * hn_blocks_per_sample(N, P) * hn_width(C); }

hipError_t norm_head_loss_launch(const void* z, const float* fa, const float* fc, int cstride, int N, int npix,
                                 const float* w, const float* b, const void* t, void* y, int C, float* prob,
                                 float* partial, float* sums, hipStream_t s) {
  const int nbp = hn_blocks_per_sample(N, npix);
  const dim3 grid(nbp, N);
  switch (C) {
    case 16:
      UNET_LAUNCH(norm_head_loss_kernel<16>, grid, dim3(HT), 0, s, (const h16*)z, fa, fc, cstride, npix, w, b,
                         (const h16*)t, (h16*)y, prob, partial);
      break;
    case 32:
      UNET_LAUNCH(norm_head_loss_kernel<32>, grid, dim3(HT), 0, s, (const h16*)z, fa, fc, cstride, npix, w, b,
                         (const h16*)t, (h16*)y, prob, partial);
      break;
    default:
      UNET_LAUNCH(norm_head_loss_kernel<64>, grid, dim3(HT), 0, s, (const h16*)z, fa, fc, cstride, npix, w, b,
                         (const h16*)t, (h16*)y, prob, partial);
  }
  // loss sums {I, St, Sp, BCE}: columns 6C + 3 .. 6C + 6 of the block rows
  UNET_LAUNCH(partial_reduce_kernel, dim3(4), dim3(256), 0, s, partial + 6 * C + 3, N * nbp, hn_width(C),
                     sums);
  return launch_status();
}

hipError_t head_norm_coef_launch(const float* partial, int N, int npix, int C, const float* sums, const float* w,
                                 const float* fa, const float* fc, int cstride, float inv_total, float bce_w,
                                 float gscale, const float* gscale_ptr, float* rows, float* gw, float* gb,
                                 hipStream_t s) {
  const int nbp = hn_blocks_per_sample(N, npix), nb = N * nbp;
  long long eb = ((long long)nb * C + 255) / 256;
  if (eb > 2048) eb = 2048;
  UNET_LAUNCH(head_norm_coef_kernel, dim3(C + 1 + (int)eb), dim3(256), 0, s, partial, nb, nbp, C, sums, w, fa,
                     fc, cstride, inv_total, bce_w, gscale, gscale_ptr, rows, gw, gb);
  return launch_status();
}

hipError_t head_norm_bwd_launch(const void* z, const float* prob, const void* t, const float* sums, const float* w,
                                const float* fa, const float* fc, const float* ca, const float* cb, const float* cc,
                                int cstride, int N, int P, int C, float inv_total, float bce_w, float gscale,
                                const float* gscale_ptr, void* dz, hipStream_t s) {
  int nbp = (1024 + N - 1) / N;
  const int maxb = (P + 255) / 256;
  nbp = nbp > maxb ? maxb : (nbp < 1 ? 1 : nbp);
  UNET_LAUNCH(head_norm_bwd_kernel, dim3(nbp, N), dim3(256), 0, s, (const h16*)z, prob, (const h16*)t, sums, w,
                     fa, fc, ca, cb, cc, cstride, P, C, inv_total, bce_w, gscale, gscale_ptr, (h16*)dz);
  return launch_status();
}

hipError_t head_finish_launch(float* prob, const void* t, int P, float* partial, float* sums, hipStream_t s) {
  // one float4 of logits per thread (latency-bound otherwise); 4 nb floats of
  // partials must fit the head's workspace of head_blocks(P) x (C + 5) >= 21
  // head_blocks(P) floats (C >= 16, head_check)
  int nb = (P / 4 + HT - 1) / HT;
  nb = nb > 4096 ? 4096 : (nb < 1 ? 1 : nb);
  if (nb > 5 * head_blocks(P)) nb = 5 * head_blocks(P);
  UNET_LAUNCH(head_finish_kernel, dim3(nb), dim3(HT), 0, s, prob, (const h16*)t, P, partial);
  UNET_LAUNCH(partial_reduce_kernel, dim3(4), dim3(256), 0, s, partial, nb, 4, sums);
  return launch_status();
}

}  // namespace unet
