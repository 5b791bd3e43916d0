// Shared epilogue of the implicit-GEMM conv kernels (conv_fwd.hip, conv_win.hip).
//
// Input: the MFMA accumulators of a BM x BN output tile issued as W x X^T, i.e.
//   acc[i][j][r] = out[pixel = m0 + wm*WM + i*16 + (lane&15)]
//                     [chan  = n0 + wn*WN + j*16 + (lane>>4)*4 + r].
// Register phase: scale, bias, ReLU, inverted dropout (counter hash), BN statistics,
// channel-split mask scale; packed to bf16 into an LDS staging tile.  Coalesced
// phase: 16-byte chunks per thread to one of two destinations (concat dgrad),
// optional consumer-side ReLU mask (out *= mask > 0) and transposed-conv pixel shuffle.
#pragma once
#include "common.h"
#include "conv_params.h"

namespace unet {

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

// EPI selects a specialised epilogue (launch-time choice, conv_epi_mode below):
//   0 generic (every feature read from p at run time), 1 forward (bias + ReLU only),
//   2 data gradient (mask scales, consumer ReLU masks, optional channel split),
//   3 pre-normalisation forward (bias, no activation) + per-tile {sum z, sum z^2},
//   4 data gradient of a normalised activation: ReLU / dropout mask recomputed from the
//     pre-norm tensor and the norm coefficients + per-tile {sum g, sum g z}.
// Modes 3 / 4 are the fused Conv+BatchNorm/GroupNorm blocks: the statistics leave the
// kernel as fixed-order per-tile partials (no atomics, bit-reproducible).
enum { EPI_GENERIC = 0, EPI_FWD = 1, EPI_DGRAD = 2, EPI_STATS = 3, EPI_DGRAD_NORM = 4 };

// LDS of the epilogue: the BM x BN staging tile plus [waves][2][BN] fp32 of
// statistics partials (modes 3 / 4)
template <int BM, int BN, int NTHR = 256>
constexpr int epi_lds_bytes() {
  return BM * (BN + 4) * 2 + (NTHR / 64) * 2 * BN * 4;
}

// Fused max-pool backward (route_gy): pooled pixel of output pixel q, and in rk the
// window corner q is, in elementwise.hip::maxpool2_fwd_kernel's order -- 2D k =
// 2 (h & 1) + (w & 1), 3D k = 4 (d & 1) + 2 (h & 1) + (w & 1) (q = ((n D + d) H + h) W + w)
__device__ __forceinline__ size_t route_pix(const ConvFwdParams& p, int q, uint32_t& rk) {
  const int g = q / p.OW, w = q - g * p.OW;
  if (p.OD > 1) {
    const int s = g / p.OH, h = g - s * p.OH;
    rk = ((uint32_t)(s & 1) << 2) | ((uint32_t)(h & 1) << 1) | (uint32_t)(w & 1);
    return ((size_t)(s >> 1) * (p.OH >> 1) + (h >> 1)) * (p.OW >> 1) + (w >> 1);
  }
  rk = ((uint32_t)(g & 1) << 1) | (uint32_t)(w & 1);
  return (size_t)(g >> 1) * (p.OW >> 1) + (w >> 1);
}
// channel e of a pool code word routes to corner rk (its first maximum, and positive)
__device__ __forceinline__ bool route_hit(uint32_t cw, int e, uint32_t rk, bool d3) {
  const uint32_t k = d3 ? (cw >> (3 * e)) & 7u : (cw >> (2 * e)) & 3u;
  return k == rk && ((cw >> (24 + e)) & 1u);
}

// nullptr when the normalisation fields of p form a supported epilogue
__host__ __device__ inline const char* conv_norm_epi_check(const ConvFwdParams& p) {
  if (!p.stats && !p.nz) return nullptr;
  if (!p.stats) return "conv_fwd: nz (dgrad-norm epilogue) needs a stats buffer";
  if (p.relu || p.shuffle || p.drop_rate > 0.f || p.out_scale != 1.f || p.D1 != p.Cout || p.mask1 || p.mask2 ||
      p.head_w || p.relu_bits || p.mask_bits || (p.route_gy && !p.nz))
    return "conv_fwd: statistics epilogue takes no ReLU / dropout / shuffle / scale / split / mask / head";
  if (p.nz && (p.bias || !p.na || !p.nc || p.npix <= 0 || p.mask_scale1 != 1.f || (p.ncs != 0 && p.ncs != p.Cout)))
    return "conv_fwd: dgrad-norm epilogue needs na / nc / npix, no bias";
  return nullptr;
}

__host__ __device__ inline int conv_epi_mode(const ConvFwdParams& p) {
  if (p.nz) return EPI_DGRAD_NORM;
  if (p.stats) return EPI_STATS;
  if (p.shuffle || p.drop_rate > 0.f || p.out_scale != 1.f) return EPI_GENERIC;
  if (p.relu && p.D1 == p.Cout && !p.mask1 && !p.mask2 && p.mask_scale1 == 1.f) return EPI_FWD;
  if (!p.relu && !p.bias) return EPI_DGRAD;
  return EPI_GENERIC;
}

// Pixel-tile maps: window-relative first pixel of accumulator tile i of wave wm.
// LinearTiles: a wave owns WM consecutive pixels.  StripTiles: a wave owns an RW-row x
// (16 TC)-column strip of a row window of width W (column strips cs = wave % NCS, row
// groups wave / NCS), tile i = (row i / TC, column tile i % TC).
template <int WM>
struct LinearTiles {
  __device__ static int base(int wm, int i) { return wm * WM + i * 16; }
};
template <int W, int RW, int TC, int NCS>
struct StripTiles {
  __device__ static int base(int wave, int i) {
    return ((wave / NCS) * RW + i / TC) * W + (wave % NCS) * 16 * TC + (i % TC) * 16;
  }
};

// Epilogue constants a persistent caller loads once (conv_win.h conv_win_pf_kernel): the
// lane's bias values bias[j][r] (channel n0 + 16 j + 4 (lane >> 4) + r) and the fused head's
// weights.  With them the EPI_FWD epilogue issues no global loads, so the caller's
// prefetch of the next window -- issued before it -- is never waited on behind them.
template <int TN>
struct EpiConst {
  float bias[TN][4];
  float hw[8];
  float hb;
};

// Mask weight-gradient sums of one tile (conv_params.h head_ws), returned by the fused-head
// epilogue when HeadT::on: the thread's 8 channels' {sum u y, sum v y, sum w y} and, on the
// pixel's chunk-0 lane, {sum u, sum v, sum w}.  HeadT::t: the targets of the thread's pixels
// of the tile (chunk iteration it: pixel tid / 4 + 64 it), prefetched by the persistent caller
// with the window's halo (a global load in the epilogue would wait on that prefetch).  Both
// travel by value: a pointer to the caller's accumulators kept them in scratch.
struct HeadWsum {
  float s[3][8];
  float u, v, w;
};
struct HeadT {
  float t[8];
  bool on;
};

// SEGW > 0: the tile is a row window of SEGW-wide row segments (window kernels on rows
// wider than one window, or any row-window kernel): tile pixel ml is at row
// m0 + ml / SEGW (m0 = first row), column col0 + ml % SEGW of rows `pitch` pixels wide.
// SEGW == 0: tile pixel ml is output pixel m0 + ml.
// stat_row: this tile's row of p.stats (modes 3 / 4).  TROW > 0: the tile is BM / TROW
// whole rows of TROW pixels (row-window kernels; enables the fused max-pool).
template <int BM, int BN, int WM, int WN, int TM, int TN, int NTHR, int EPI = EPI_GENERIC,
          class MapM = LinearTiles<WM>, int SEGW = 0, int TROW = 0>
__device__ __forceinline__ HeadWsum conv_epilogue(const ConvFwdParams p, f32x4 (&acc)[TM][TN], char* smem,
                                                  const int m0, const int n0, const int M, const int wm,
                                                  const int wn, const int lane, const int tid,
                                                  const int pitch = 0, const int col0 = 0, const int stat_row = 0,
                                                  const EpiConst<TN>* ec = nullptr, const HeadT ht = HeadT{}) {
  HeadWsum hws;
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) hws.s[k][e] = 0.f;
  hws.u = hws.v = hws.w = 0.f;
  auto qof = [&](int ml) -> int {
    if constexpr (SEGW > 0) return (m0 + ml / SEGW) * pitch + col0 + (ml % SEGW);
    else return m0 + ml;
  };
  // Staging tile rows (pixels).  BN = 32: unpadded 64-byte rows, 16-byte chunk c of pixel ml
  // at c ^ ((ml >> 2) & 3), its two 8-byte halves swapped when (ml >> 1) & 1.  The register
  // phase's 8-byte writes go 16 lanes at a time over 32 banks (16 consecutive pixels, one
  // half of one chunk): pixel parity picks the 64-byte half of the bank window, (ml >> 2) & 3
  // the chunk, (ml >> 1) & 1 the half -- 16 distinct slots, conflict-free.  Without the half
  // swap only 8 slots are reachable (2-way: 17-18 % conflict cycles on the level-1 windows,
  // r5 PMC pass; tools/lds_bank_model.py check_epi).  The coalesced phase's 16-byte chunk
  // reads (4 lanes per pixel) are unaffected and swap the halves back in registers.
  // Wider tiles: rows padded by 8 bytes.
  constexpr bool ESWZ = BN == 32;
  constexpr int EPI_STRIDE = ESWZ ? 64 : (BN + 4) * 2;
  auto eoff = [](const int ml, const int chunk) -> int {
    return ESWZ ? ml * 64 + 16 * (chunk ^ ((ml >> 2) & 3)) : ml * EPI_STRIDE + 16 * chunk;
  };
  // byte offset of the 8-byte half of channels nl .. nl + 3 (nl % 4 == 0) of pixel ml
  auto ehalf = [](const int ml, const int nl) -> int {
    return ESWZ ? ml * 64 + 16 * ((nl >> 3) ^ ((ml >> 2) & 3)) + ((2 * (nl & 7)) ^ (8 * ((ml >> 1) & 1)))
                : ml * EPI_STRIDE + 2 * nl;
  };
  auto eread = [&](const int ml, const int chunk) -> u32x4 {
    if constexpr (ESWZ) {
      const u32x4 v = *(const u32x4*)(smem + eoff(ml, chunk));
      return ((ml >> 1) & 1) ? (u32x4){v[2], v[3], v[0], v[1]} : v;
    } else {
      const u32x2 lo = *(const u32x2*)(smem + eoff(ml, chunk));
      const u32x2 hi = *(const u32x2*)(smem + eoff(ml, chunk) + 8);
      return (u32x4){lo[0], lo[1], hi[0], hi[1]};
    }
  };
  // register phase: acc[i][j][r] = out[pixel = m0 + wm*WM + i*16 + (lane&15)]
  //                                   [chan  = n0 + wn*WN + j*16 + (lane>>4)*4 + r]
  char* E = smem;
  float* SP = (float*)(smem + BM * EPI_STRIDE);       // [4][2][BN] statistics partials
  constexpr bool G = EPI == EPI_GENERIC;
  constexpr bool kNormG = EPI == EPI_DGRAD_NORM;
  const bool kRelu = G ? (p.relu != 0) : (EPI == EPI_FWD);
  const bool kBias = EPI != EPI_DGRAD && !kNormG && p.bias;
  const bool kDrop = G && p.drop_rate > 0.f;
  constexpr bool kStats = EPI == EPI_STATS;
  const bool kShuffle = G && p.shuffle;
  constexpr bool kMaskScale = EPI == EPI_GENERIC || EPI == EPI_DGRAD;
  const float inv_keep = p.drop_rate > 0.f ? 1.f / (1.f - p.drop_rate) : 1.f;
  const uint32_t drop_thr = (uint32_t)(p.drop_rate * 4294967296.0);
  const uint32_t seed = (kDrop && p.seed_ptr) ? *p.seed_ptr : p.seed;
  const int Dtb = kShuffle ? (p.Cout >> p.shuffle) : p.Cout;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * WN + j * 16 + (lane >> 4) * 4;
    const int n = n0 + nl;
    float bsv[4], msc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      bsv[r] = ec ? ec->bias[j][r] : (kBias ? p.bias[kShuffle ? (n + r) % Dtb : n + r] : 0.f);
      msc[r] = kMaskScale ? ((n + r < p.D1) ? p.mask_scale1 : p.mask_scale2) : 1.f;
    }
    if constexpr (EPI == EPI_FWD) {
      // bias + ReLU: packed fp32 adds, the ReLU on the packed 16-bit pair (relu2h; the
      // same bits as clamping before the rounding)
      const f32x2 b01 = {bsv[0], bsv[1]}, b23 = {bsv[2], bsv[3]};
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int ml = MapM::base(wm, i) + (lane & 15);
        f32x2 a01 = (f32x2){acc[i][j][0], acc[i][j][1]} + b01;
        f32x2 a23 = (f32x2){acc[i][j][2], acc[i][j][3]} + b23;
        u32x2 pk;
        pk[0] = relu2h(pack2h(a01[0], a01[1]));
        pk[1] = relu2h(pack2h(a23[0], a23[1]));
        *(u32x2*)(E + ehalf(ml, nl)) = pk;
      }
      continue;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = MapM::base(wm, i) + (lane & 15);
      const int q = qof(ml);
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = G ? acc[i][j][r] * p.out_scale + bsv[r] : acc[i][j][r] + bsv[r];
        if (kRelu) x = fmaxf(x, 0.f);
        if (kDrop) {
          const uint32_t h = drop_hash((uint64_t)q * p.Cout + n + r + p.drop_idx0, seed, p.salt);
          x = (h >= drop_thr) ? x * inv_keep : 0.f;
        }
        if (kMaskScale) x *= msc[r];
        v[r] = x;
      }
      u32x2 pk;
      pk[0] = pack2h(v[0], v[1]);
      pk[1] = pack2h(v[2], v[3]);
      *(u32x2*)(E + ehalf(ml, nl)) = pk;
    }
  }
  __syncthreads();

  // coalesced phase: 16-byte chunks, consecutive threads -> consecutive channels
  constexpr int CPR = BN / 8;
  constexpr int NCHUNK = BM * CPR;
  // statistics rows (modes 3 / 4): thread (chunk column cb) holds s1[8], s2[8] of its
  // rows; lanes congruent mod CPR are summed by xor shuffles, then the NTHR / 64 waves
  // in fixed order through LDS -> p.stats[stat_row][mom][n0 + c]
  auto stats_out = [&](float (&s1)[8], float (&s2)[8], int cb) {
#pragma unroll
    for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    const int wv = tid >> 6;
    if ((tid & 63) < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        SP[(wv * 2 + 0) * BN + cb * 8 + e] = s1[e];
        SP[(wv * 2 + 1) * BN + cb * 8 + e] = s2[e];
      }
    }
    __syncthreads();
    for (int t = tid; t < 2 * BN; t += NTHR) {
      const int mom = t / BN, c = t - mom * BN;
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < NTHR / 64; ++w) a += SP[(w * 2 + mom) * BN + c];
      p.stats[((size_t)stat_row * 2 + mom) * p.Cout + n0 + c] = a;
    }
  };
  if constexpr (kStats) {
    // pre-normalisation output z: store, and accumulate {sum z, sum z^2} of the stored
    // (bf16-rounded) values the consumers will read
    static_assert(NCHUNK % NTHR == 0 && NTHR % CPR == 0 && CPR <= 64, "statistics tiling");
    constexpr int NIT = NCHUNK / NTHR, RPI = NTHR / CPR;
    const int cb = tid % CPR, ml0 = tid / CPR;
    const int n = n0 + cb * 8;
    h16* dst = (h16*)p.dst1;
    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int ml = ml0 + it * RPI;
      const int q = qof(ml);
      if (q >= M) continue;
      const u32x4 v = eread(ml, cb);
      *(u32x4*)(dst + (size_t)q * p.Cout + n) = v;
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += f[e];
        s2[e] = fmaf(f[e], f[e], s2[e]);
      }
    }
    stats_out(s1, s2, cb);
    return hws;
  }
  if constexpr (kNormG) {
    // gradient of y = dropout(relu(na z + nc)): mask recomputed from the pre-norm z the
    // forward stored (the normalised y is never needed), plus the tile's {sum g, sum g z}
    static_assert(NCHUNK % NTHR == 0 && NTHR % CPR == 0 && CPR <= 64, "dgrad-norm tiling");
    constexpr int NIT = NCHUNK / NTHR, RPI = NTHR / CPR;
    const int cb = tid % CPR, ml0 = tid / CPR;
    const int n = n0 + cb * 8;
    h16* dst = (h16*)p.dst1;
    const h16* zt = (const h16*)p.nz;
    // a tile never spans two samples when the coefficients are per sample (host check)
    const size_t crow = p.ncs ? (size_t)(qof(0) / p.npix) * p.ncs : 0;
    float ca[8], cc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ca[e] = p.na[crow + n + e];
      cc[e] = p.nc[crow + n + e];
    }
    u32x4 zv[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int q = qof(ml0 + it * RPI);
      if (q < M) zv[it] = *(const u32x4*)(zt + (size_t)q * p.Cout + n);
    }
    // fused max-pool backward (route_gy; the skip half of a decoder data gradient): the
    // pooled gradient is added at each window's recorded argmax before the mask
    const bool route = p.route_gy != nullptr, d3 = p.OD > 1;
    u32x4 rg[NIT];
    uint32_t rc[NIT], rk[NIT];
    if (route) {
      const int cpp = p.Cout >> 3;
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = qof(ml0 + it * RPI);
        if (q < M) {
          const size_t pq = route_pix(p, q, rk[it]);
          rc[it] = p.pool_code[pq * cpp + (n >> 3)];
          rg[it] = *(const u32x4*)((const h16*)p.route_gy + pq * p.Cout + n);
        }
      }
    }
    const bool drop = p.nd_rate > 0.f;
    const float dscale = drop ? 1.f / (1.f - p.nd_rate) : 1.f;
    const uint32_t dthr = (uint32_t)(p.nd_rate * 4294967296.0);
    const uint32_t dseed = p.seed_ptr ? *p.seed_ptr : p.seed;
    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int ml = ml0 + it * RPI;
      const int q = qof(ml);
      if (q >= M) continue;
      float g[8], z[8];
      unpack8(eread(ml, cb), g);
      unpack8(zv[it], z);
      if (route) {
        float gg[8];
        unpack8(rg[it], gg);
        const uint32_t cw = rc[it];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (route_hit(cw, e, rk[it], d3)) g[e] += gg[e];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bool keep = fmaf(ca[e], z[e], cc[e]) > 0.f;
        if (drop) keep = keep && drop_hash((uint64_t)q * p.Cout + n + e, dseed, p.nd_salt) >= dthr;
        g[e] = keep ? g[e] * dscale : 0.f;
      }
      const u32x4 gv = pack8(g);
      *(u32x4*)(dst + (size_t)q * p.Cout + n) = gv;
      unpack8(gv, g);                                   // the stored (rounded) gradient
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s1[e] += g[e];
        s2[e] = fmaf(g[e], z[e], s2[e]);
      }
    }
    stats_out(s1, s2, cb);
    return hws;
  }
  if constexpr (EPI == EPI_DGRAD && NCHUNK % NTHR == 0 && NTHR % CPR == 0) {
    // a thread's channel chunk (hence destination tensor, row stride and mask) is the
    // same for all its rows: issue every ReLU-mask load first, then mask and store
    constexpr int NIT = NCHUNK / NTHR, RPI = NTHR / CPR;
    const int cb = tid % CPR, ml0 = tid / CPR;
    const int n = n0 + cb * 8;
    const bool side1 = n < p.D1;
    const int rs = side1 ? p.D1 : p.Cout - p.D1;
    const int co = side1 ? n : n - p.D1;
    h16* dst = (h16*)(side1 ? p.dst1 : p.dst2);
    const h16* mk = (const h16*)(side1 ? p.mask1 : p.mask2);
    const bool mbit = (p.mask_bits >> (side1 ? 0 : 1)) & 1;
    u32x4 mv[NIT];
    uint32_t mb[NIT];
    if (mk) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = qof(ml0 + it * RPI);
        if (q < M) {
          if (mbit)
            mb[it] = ((const uint8_t*)mk)[((size_t)q * rs + co) >> 3];
          else
            mv[it] = *(const u32x4*)(mk + (size_t)q * rs + co);
        }
      }
    }
    // fused pool backward (route_gy, one destination; route_pix / route_hit)
    const bool route = p.route_gy != nullptr, d3 = p.OD > 1;
    u32x4 rg[NIT];
    uint32_t rc[NIT], rk[NIT];
    if (route) {
      const int cpp = p.Cout >> 3;
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int q = qof(ml0 + it * RPI);
        if (q < M) {
          const size_t pq = route_pix(p, q, rk[it]);
          rc[it] = p.pool_code[pq * cpp + (n >> 3)];
          rg[it] = *(const u32x4*)((const h16*)p.route_gy + pq * p.Cout + n);
        }
      }
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int ml = ml0 + it * RPI;
      const int q = qof(ml);
      if (q >= M) continue;
      u32x4 v = eread(ml, cb);
      if (mk) v = mbit ? keep_bits(v, mb[it]) : keep_pos(v, mv[it]);
      if (route) {
        // the (masked, 16-bit rounded) skip gradient plus the routed pool gradient,
        // in the order and precision of elementwise.hip::maxpool2_bwd_code_kernel
        float o[8], gg[8];
        unpack8(v, o);
        unpack8(rg[it], gg);
        const uint32_t cw = rc[it];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (route_hit(cw, e, rk[it], d3)) o[e] += gg[e];
        v = pack8(o);
      }
      *(u32x4*)(dst + (size_t)q * rs + co) = v;
    }
    return hws;
  }
  const int Dt = kShuffle ? (p.Cout >> p.shuffle) : 0;
  // Fused segmentation head (forward of conv9b, BN == Cout == 32): the CPR = 4
  // consecutive threads holding one pixel's four 8-channel chunks dot them with the
  // 1x1 head weights (the same bf16-rounded activations head.hip::head_fwd_kernel
  // reads) and combine by two lane swaps; the fp32 logit is stored per pixel -- the
  // 268 MB re-read of a separate head launch becomes a 17 MB one.
  constexpr bool kHeadable = EPI == EPI_FWD && BN == 32 && NTHR % CPR == 0;
  const bool kHead = kHeadable && p.head_w != nullptr;
  float hw[8], hb = 0.f;
  constexpr int HIT = kHeadable ? NCHUNK / NTHR : 1;     // chunk iterations per thread
  static_assert(!kHeadable || (NCHUNK % NTHR == 0 && HIT % CPR == 0 && HIT <= 8), "fused head tiling");
  float hz[HIT];
  int hq[HIT];
#pragma unroll
  for (int k = 0; k < HIT; ++k) {
    hz[k] = 0.f;
    hq[k] = M;                                          // skipped (q >= M) unless set below
  }
  if (kHeadable && kHead) {
#pragma unroll
    for (int e = 0; e < 8; ++e) hw[e] = ec ? ec->hw[e] : p.head_w[(tid % CPR) * 8 + e];
    hb = ec ? ec->hb : p.head_b[0];
  }
  // (fully unrolled with the fused head, whose per-iteration logits live in registers)
  constexpr int NITER = (NCHUNK + NTHR - 1) / NTHR;
  constexpr int UNR = kHeadable ? NITER : 2;
#pragma unroll UNR
  for (int it = 0; it < NITER; ++it) {
    const int c = tid + it * NTHR;
    if (NCHUNK % NTHR && c >= NCHUNK) break;
    const int ml = c / CPR, cb = c % CPR;
    const int q = qof(ml);
    if (q >= M) continue;
    const int n = n0 + cb * 8;
    u32x4 v = eread(ml, cb);
    size_t off;
    h16* dst;
    const void* mk;
    bool mbit = false;
    if (EPI == EPI_FWD || EPI == EPI_STATS) {
      off = (size_t)q * p.Cout + n;
      dst = (h16*)p.dst1;
      mk = nullptr;
    } else if (kShuffle) {
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
      dst = (h16*)p.dst1;
      mk = p.mask1;
      mbit = p.mask_bits & 1;
    } else if (n < p.D1) {
      off = (size_t)q * p.D1 + n;
      dst = (h16*)p.dst1;
      mk = p.mask1;
      mbit = p.mask_bits & 1;
    } else {
      off = (size_t)q * (p.Cout - p.D1) + (n - p.D1);
      dst = (h16*)p.dst2;
      mk = p.mask2;
      mbit = (p.mask_bits >> 1) & 1;
    }
    if (EPI != EPI_FWD && EPI != EPI_STATS && mk) {
      // (off is a multiple of 8: the bit tensor's byte of these 8 channels is off / 8)
      v = mbit ? keep_bits(v, ((const uint8_t*)mk)[off >> 3]) : keep_pos(v, *(const u32x4*)((const h16*)mk + off));
    }
    if (!(kHeadable && kHead && p.head_nostore)) *(u32x4*)(dst + off) = v;
    // (EPI_FWD: ReLU outputs from relu2h, never -0 -- the cheap form)
    if (EPI == EPI_FWD && p.relu_bits) p.relu_bits[off >> 3] = (uint8_t)pos_bits_relu(v);
    if (G && p.relu_bits) p.relu_bits[off >> 3] = (uint8_t)pos_bits(v);
    if constexpr (kHeadable) {
      if (kHead) {
        float f[8];
        unpack8(v, f);
        float z = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) z += f[e] * hw[e];
        z += __shfl_xor(z, 1, 64);     // the pixel's 4 chunk lanes (all active or all not)
        z += __shfl_xor(z, 2, 64);
        hz[it] = z + hb;
        hq[it] = q;
        if (ht.on) {
          // the probability head_finish forms from this logit, the target: the Mask weight
          // gradient's per-pixel factors (head_grad.h head_dlogit = A u + B v + G w)
          const float zl = z + hb;
          // (hardware reciprocal: the IEEE division made the forward +12 %; the sums feed only
          // the Mask gradient, within fp32 rounding of head_finish's probability)
          const float pr = __builtin_amdgcn_rcpf(1.f + __expf(-zl));
          const float tv = ht.t[it];
          const float vv = pr * (1.f - pr), uu = tv * vv, ww = pr - tv;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            hws.s[0][e] = fmaf(uu, f[e], hws.s[0][e]);
            hws.s[1][e] = fmaf(vv, f[e], hws.s[1][e]);
            hws.s[2][e] = fmaf(ww, f[e], hws.s[2][e]);
          }
          if (cb == 0) {
            hws.u += uu;
            hws.v += vv;
            hws.w += ww;
          }
        }
      }
    }
  }
  if constexpr (kHeadable) {
    if (kHead) {
      // the 4 lanes of a pixel group hold the same HIT logits: lane cb stores
      // iterations cb, cb + 4, ...; head.hip::head_finish turns them into
      // probabilities and loss partials
      const int cb = tid % CPR;
#pragma unroll
      for (int k = 0; k < HIT / CPR; ++k) {
        float z = hz[CPR * k];
        int q = hq[CPR * k];
#pragma unroll
        for (int r = 1; r < CPR; ++r) {
          z = cb == r ? hz[CPR * k + r] : z;
          q = cb == r ? hq[CPR * k + r] : q;
        }
        if (q < M) p.head_logit[q] = z;
      }
    }
  }
  if constexpr (EPI == EPI_FWD && TROW > 0 && (BM / TROW) % 2 == 0 && TROW % 2 == 0) {
    if (p.pool_dst) {
      // 2x2 max-pool of the tile's complete row pairs (a window starts on an even row
      // and holds an even number of rows): max + first-argmax code per channel, the
      // "max > 0" flag in bit 24 + e (elementwise.hip::maxpool2_fwd_kernel layout)
      constexpr int PC = TROW / 2, NP = (BM / TROW / 2) * PC * CPR;
      const int Wp = p.OW >> 1, cpp = p.Cout >> 3;
      h16* pdst = (h16*)p.pool_dst;
      for (int k = tid; k < NP; k += NTHR) {
        const int cb = k % CPR, pp = k / CPR;
        const int pr = pp / PC, pc = pp - pr * PC;
        const int ml00 = 2 * pr * TROW + 2 * pc;
        const int q00 = qof(ml00);
        if (q00 >= M) continue;
        // the staged values are ReLU outputs (>= 0, never -0): their 16-bit patterns
        // order like the values, so key = bits << 16 | (3 - kk) as int32 gives max and
        // first argmax (ties: larger 3 - kk wins) in one integer max per element
        int32_t key[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) key[e] = INT32_MIN;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const int ml = ml00 + (kk >> 1) * TROW + (kk & 1);
          const u32x4 v = eread(ml, cb);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            key[2 * e] = max(key[2 * e], (int32_t)((v[e] << 16) | (3u - kk)));
            key[2 * e + 1] = max(key[2 * e + 1], (int32_t)((v[e] & 0xffff0000u) | (3u - kk)));
          }
        }
        uint32_t w = 0;
        u32x4 mv;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          w |= ((3u - ((uint32_t)key[e] & 3u)) << (2 * e)) | ((key[e] > 3 ? 1u : 0u) << (24 + e));
#pragma unroll
        for (int e = 0; e < 4; ++e)
          mv[e] = ((uint32_t)key[2 * e] >> 16) | ((uint32_t)key[2 * e + 1] & 0xffff0000u);
        const int grow = q00 / p.OW, gcol = q00 - grow * p.OW;
        const size_t pq = (size_t)(grow >> 1) * Wp + (gcol >> 1);
        *(u32x4*)(pdst + pq * p.Cout + n0 + cb * 8) = mv;
        p.pool_code[pq * cpp + (n0 >> 3) + cb] = w;
      }
    }
  }
  return hws;
}

}  // namespace unet
