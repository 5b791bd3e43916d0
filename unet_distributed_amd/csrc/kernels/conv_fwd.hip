// Implicit-GEMM convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16), NHWC/NDHWC bf16.
//
// out[q][n] = epilogue( sum_{tap, c} X[q*stride + tap - pad][c] * W[n][tap][c] )
//
// * GEMM M = output pixels (B*D*H*W), N = Cout, K = taps x Cin; K-step = one tap x 32 channels.
// * A (pixels) and B (weights) tiles are staged global->VGPR->LDS with one
//   register prefetch stage in flight while the MFMAs consume the other LDS
//   buffer (cdna_hip_programming.md §5.5 T14); 64-byte LDS rows with a
//   per-row-quad XOR swizzle of the 16-byte chunks so both the ds_write_b128
//   staging and the ds_read_b128 fragment reads are bank-conflict free
//   (checked by tools/lds_bank_model.py).
// * The MFMA is issued as W x X^T so an accumulator register row runs along
//   Cout: each lane then owns 4 consecutive channels of one pixel, which packs
//   to 8 bytes for the LDS-staged, fully coalesced 16 B/lane epilogue store.
// * Fused epilogue: scale, bias, ReLU, inverted dropout (counter hash),
//   per-channel BN statistics, ReLU-mask of the consumer-side backward
//   (out *= mask > 0), channel split into two destination tensors (dgrad of a
//   concat input), transposed-conv pixel shuffle.
// * src1/src2 concat and nearest-upsample are folded into the A-tile address
//   generation: the skip concat is never materialised.
//
// Reference semantics: Conv2D 3x3 'same' + ReLU (`model.py:47-117`),
// Conv2DTranspose 2x2/2 (`model.py:79-113`), concatenate (`model.py:76-113`),
// Dropout(0.2) (`model.py:60,66`).
#include "common.h"
#include "conv_params.h"

namespace unet {

namespace {

constexpr int NTHR = 256;

__device__ __forceinline__ int swz4(int row) {  // chunk XOR for 64-byte rows
  return (0x78 >> (2 * ((row >> 2) & 3))) & 3;
}

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

// SMALLC: first-layer mode for Cin in {4, 8}: the K index runs over (tap, ci)
// jointly (K = taps*Cin padded to a multiple of 32) so a 16-byte A chunk holds
// 8/Cin taps; the weights are stored [Cout][Kpad] with zero padding.
template <int BM, int BN, int WAVES_M, int WAVES_N, bool SMALLC>
__global__ void __launch_bounds__(NTHR) conv_fwd_kernel(const ConvFwdParams p) {
  constexpr int WM = BM / WAVES_M, WN = BN / WAVES_N;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_PER_T = (BM * 4 + NTHR - 1) / NTHR;
  constexpr int B_PER_T = (BN * 4 + NTHR - 1) / NTHR;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int EPI_STRIDE = (BN + 4) * 2;  // bytes; 8B-aligned, conflict-free b64 writes
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
  const int cblocks = SMALLC ? 1 : (Cin >> 5);
  const int Kpad = ((KT * Cin + 31) >> 5) << 5;
  const int nk = SMALLC ? (Kpad >> 5) : KT * cblocks;
  const size_t Ktot = SMALLC ? (size_t)Kpad : (size_t)KT * Cin;
  const int ccol = tid & 3;
  const int upd = p.ID > 1 ? p.up1 : 1;  // 2D: depth is never upsampled
  const int ID1 = p.ID / upd, IH1 = p.IH / p.up1, IW1 = p.IW / p.up1;

  // ---- per-thread A rows (fixed for the whole K loop)
  int a_n[A_PER_T], a_d[A_PER_T], a_h[A_PER_T], a_w[A_PER_T];
  bool a_ok[A_PER_T];
#pragma unroll
  for (int i = 0; i < A_PER_T; ++i) {
    const int r = (tid >> 2) + 64 * i;
    const int q = m0 + r;
    a_ok[i] = (r < BM) && (q < M);
    PixCoord c = decompose(a_ok[i] ? q : 0, p.OD, p.OH, p.OW);
    a_n[i] = c.n;
    a_d[i] = c.d * p.stride - (p.KD > 1 ? p.pad : 0);   // 2D: depth is not padded
    a_h[i] = c.h * p.stride - p.pad;
    a_w[i] = c.w * p.stride - p.pad;
  }
  const bf16* wbase = (const bf16*)p.wgt;

  u32x4 ra[A_PER_T], rb[B_PER_T];

  auto load_stage_small = [&](int ks) {
    // chunk = 8 consecutive k = (8 / Cin) taps x Cin channels
    const int k0 = ks * 32 + ccol * 8;
    const int tpc = 8 / Cin;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      u32x4 v = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        if (e >= tpc) break;
        const int tap = k0 / Cin + e;
        if (tap >= KT || !a_ok[i]) continue;
        const int kw = tap % p.KW, kh = (tap / p.KW) % p.KH, kd = tap / (p.KW * p.KH);
        const int id = a_d[i] + kd, ih = a_h[i] + kh, iw = a_w[i] + kw;
        if ((unsigned)id >= (unsigned)p.ID || (unsigned)ih >= (unsigned)p.IH || (unsigned)iw >= (unsigned)p.IW)
          continue;
        const size_t pix = (((size_t)a_n[i] * p.ID + id) * p.IH + ih) * p.IW + iw;
        const bf16* src = (const bf16*)p.src1 + pix * Cin;
        if (Cin == 8) {
          v = *(const u32x4*)src;
        } else {
          const u32x2 h = *(const u32x2*)src;
          v[2 * e] = h[0];
          v[2 * e + 1] = h[1];
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int r = (tid >> 2) + 64 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (r < BN) v = *(const u32x4*)(wbase + (size_t)(n0 + r) * Ktot + k0);
      rb[i] = v;
    }
  };
  auto load_stage = [&](int ks) {
    if constexpr (SMALLC) {
      load_stage_small(ks);
      return;
    }
    const int tap = ks / cblocks;
    const int c0 = (ks - tap * cblocks) << 5;
    const int kw = tap % p.KW;
    const int kh = (tap / p.KW) % p.KH;
    const int kd = tap / (p.KW * p.KH);
    const bool from1 = c0 < p.C1;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int id = a_d[i] + kd, ih = a_h[i] + kh, iw = a_w[i] + kw;
      const bool ok = a_ok[i] && (unsigned)id < (unsigned)p.ID && (unsigned)ih < (unsigned)p.IH &&
                      (unsigned)iw < (unsigned)p.IW;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (ok) {
        const bf16* src;
        if (from1) {
          const size_t pix = (((size_t)a_n[i] * ID1 + id / upd) * IH1 + ih / p.up1) * IW1 + iw / p.up1;
          src = (const bf16*)p.src1 + pix * p.C1 + c0 + ccol * 8;
        } else {
          const size_t pix = (((size_t)a_n[i] * p.ID + id) * p.IH + ih) * p.IW + iw;
          src = (const bf16*)p.src2 + pix * p.C2 + (c0 - p.C1) + ccol * 8;
        }
        v = *(const u32x4*)src;
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int r = (tid >> 2) + 64 * i;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (r < BN) v = *(const u32x4*)(wbase + (size_t)(n0 + r) * Ktot + (size_t)tap * Cin + c0 + ccol * 8);
      rb[i] = v;
    }
  };
  auto store_stage = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_PER_T; ++i) {
      const int r = (tid >> 2) + 64 * i;
      if (r < BM) *(u32x4*)(As + r * 64 + 16 * (ccol ^ swz4(r))) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER_T; ++i) {
      const int r = (tid >> 2) + 64 * i;
      if (r < BN) *(u32x4*)(Bs + r * 64 + 16 * (ccol ^ swz4(r))) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // per-lane fragment offset inside a 16-row slab (swizzle depends on lane only)
  const int frag_off = (lane & 15) * 64 + 16 * ((lane >> 4) ^ swz4(lane & 15));

  load_stage(0);
  store_stage(0);
  __syncthreads();
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load_stage(ks + 1);
    const char* As = smem + buf * STAGE;
    const char* Bs = As + A_BYTES;
    bf16x8 xf[TM], wf[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
      xf[i] = *(const bf16x8*)(As + (wm * WM + i * 16) * 64 + frag_off);
#pragma unroll
    for (int j = 0; j < TN; ++j)
      wf[j] = *(const bf16x8*)(Bs + (wn * WN + j * 16) * 64 + frag_off);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(wf[j], xf[i], acc[i][j]);
    if (ks + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  // register phase: acc[i][j][r] = out[pixel = m0 + wm*WM + i*16 + (lane&15)]
  //                                   [chan  = n0 + wn*WN + j*16 + (lane>>4)*4 + r]
  char* E = smem;
  const float inv_keep = p.drop_rate > 0.f ? 1.f / (1.f - p.drop_rate) : 1.f;
  const uint32_t drop_thr = (uint32_t)(p.drop_rate * 4294967296.0);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WN + j * 16 + (lane >> 4) * 4;
    const int n = n0 + nl;
    float bsv[4], msc[4];
    const int Dtb = p.shuffle ? (p.Cout >> p.shuffle) : p.Cout;
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
      // reduce over the 16 pixel-lanes sharing (lane>>4), then one atomic per channel
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
  const int Dt = p.shuffle ? (p.Cout >> p.shuffle) : 0;  // tconv output channels
#pragma unroll 2
  for (int c = tid; c < NCHUNK; c += NTHR) {
    const int ml = c / CPR, cb = c % CPR;
    const int q = m0 + ml;
    if (q >= M) continue;
    const int n = n0 + cb * 8;
    u32x2 lo = *(const u32x2*)(E + ml * EPI_STRIDE + cb * 16);
    u32x2 hi = *(const u32x2*)(E + ml * EPI_STRIDE + cb * 16 + 8);
    u32x4 v = {lo[0], lo[1], hi[0], hi[1]};
    size_t off;
    bf16* dst;
    const void* mk;
    if (p.shuffle) {
      const int tap = n / Dt, co = n - tap * Dt;
      PixCoord pc = decompose(q, p.OD, p.OH, p.OW);
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
        // bf16 > 0  <=>  sign bit clear and not +0 (relu outputs are never -0 ... treat -0 as 0)
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

template <int BM, int BN, int WAVES_M, int WAVES_N, bool SMALLC = false>
hipError_t launch_cfg(const ConvFwdParams& p, hipStream_t s) {
  const int M = p.N * p.OD * p.OH * p.OW;
  const int grid = ((M + BM - 1) / BM) * (p.Cout / BN);
  hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, WAVES_M, WAVES_N, SMALLC>), dim3(grid), dim3(NTHR), 0, s, p);
  return hipGetLastError();
}

}  // namespace

// Returns nullptr on success, or a message describing why the shape is unsupported.
const char* conv_fwd_check(const ConvFwdParams& p) {
  const bool smallc = (p.C1 == 4 || p.C1 == 8) && p.C2 == 0;
  if (smallc) {
    if (p.up1 != 1 || p.shuffle) return "conv_fwd: small-Cin mode supports plain convs only";
  } else if (p.C1 <= 0 || (p.C1 % 32) || (p.C2 % 32)) {
    return "conv_fwd: input channels must be multiples of 32 (or 4/8 for the first layer)";
  }
  if (p.Cout % 32) return "conv_fwd: Cout must be a multiple of 32";
  if (p.D1 <= 0 || p.D1 > p.Cout || (p.D1 % 8)) return "conv_fwd: bad channel split D1";
  if (p.D1 < p.Cout && !p.dst2) return "conv_fwd: dst2 missing for channel split";
  if (p.up1 != 1 && p.up1 != 2) return "conv_fwd: up1 must be 1 or 2";
  if (p.up1 == 2 && ((p.ID % 2 && p.ID != 1) || p.IH % 2 || p.IW % 2)) return "conv_fwd: upsample needs even dims";
  if (p.C2 > 0 && !p.src2) return "conv_fwd: src2 missing";
  if (p.shuffle && (p.Cout % (1 << p.shuffle))) return "conv_fwd: shuffle needs Cout % taps == 0";
  if (p.shuffle && ((p.Cout >> p.shuffle) % 8)) return "conv_fwd: shuffle channels must be multiples of 8";
  if (p.shuffle && p.D1 != p.Cout) return "conv_fwd: shuffle with channel split unsupported";
  if (p.stats && p.shuffle) return "conv_fwd: stats with shuffle unsupported";
  if ((long long)p.N * p.OD * p.OH * p.OW >= (1LL << 31)) return "conv_fwd: too many pixels";
  return nullptr;
}

hipError_t conv_fwd_launch(const ConvFwdParams& p, hipStream_t s) {
  const int M = p.N * p.OD * p.OH * p.OW;
  if ((p.C1 == 4 || p.C1 == 8) && p.C2 == 0) {
    if (p.Cout % 64 == 0) return launch_cfg<128, 64, 2, 2, true>(p, s);
    return launch_cfg<256, 32, 4, 1, true>(p, s);
  }
  if (p.Cout % 128 == 0 && M >= 8192) return launch_cfg<128, 128, 2, 2>(p, s);
  if (p.Cout % 64 == 0) return launch_cfg<128, 64, 2, 2>(p, s);
  return launch_cfg<256, 32, 4, 1>(p, s);
}

}  // namespace unet
