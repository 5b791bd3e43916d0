// Pipelined row-window weight gradient for the mid UNet levels (2D 3x3 'same' convs on
// full rows 16..64 wide): the window loop of conv_wgrad.hip::wgrad_win_kernel with its
// per-window stage double-buffered in LDS, so window w+1's input halo and dY image stream
// in by LDS-DMA while window w's MFMAs run.
//
// Why (profiles/r3_stall_breakdown.md): the 4-wave window wgrad stages one window, drains
// it (vmcnt(0) + barrier) and only then computes; its two workgroups per CU spend 43-45 %
// of wave-cycles parked on that wait at 45-49 % MFMA busy on 16..64-wide rows.  Here ONE
// 8-wave workgroup per CU (still 2 waves per SIMD) holds two window stages (2 x 62-68 KB);
// the 8 waves split each window's pixels twice as finely as the 4 waves did (4 or 8
// pixel-split waves per output-channel block), and reduce their partials through LDS at
// the end as before.  Per (tap, ci, co) the sum over a window's pixels is split across
// the waves differently from the 4-wave kernel, so the slabs agree to fp32 rounding, not
// bit for bit; the split-K reduction after them is unchanged (deterministic).
#include "common.h"
#include "conv_params.h"

namespace unet {

hipError_t launch_wgrad_pipe(const WgradParams& p, hipStream_t s);

namespace {

constexpr int WP_NTHR = 512;

template <int W, int QO, bool CONCAT>
__global__ void __launch_bounds__(WP_NTHR) wgrad_pipe_kernel(const WgradParams p) {
  constexpr int BMW = 256, R = BMW / W, HR = R + 2;
  constexpr int HWP = ((W + 2 + 15) / 16) * 16, IPR = HWP / 16, ROWB = HWP * 64;
  constexpr int XI = HR * IPR, YI = QO * BMW / 16;
  constexpr int XB = XI * 1024, YB = YI * 1024, STAGE = XB + YB;
  constexpr int NW = WP_NTHR / 64;
  constexpr int PS = NW / QO;                           // pixel-split waves per co block
  static_assert(W == 16 || W == 32 || W == 64, "pipelined window wgrad: 16..64-wide rows");
  static_assert(NW * 64 * 16 * 4 <= STAGE, "partial reduction fits one stage");
  static_assert(2 * STAGE <= 160 * 1024, "two stages fit the 160 KB LDS");
  // two stages as two LDS objects (distinct alias scopes: the fragment reads of one stage
  // never wait for the DMA in flight into the other)
  __shared__ __attribute__((aligned(1024))) char lds0[STAGE];
  __shared__ __attribute__((aligned(1024))) char lds1[STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qo = wave % QO, ps = wave / QO;
  const int H = p.QH;
  const int rows_total = p.N * H;
  const int Mq = rows_total * W;
  const int nwin = (rows_total + R - 1) / R;
  const int Mtot = p.M1 + p.M2;
  const int cob = p.Nc / (32 * QO);
  const int ntile = (Mtot / 32) * cob;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);     // one split's tiles on one XCD
  const int lsplit = bid / ntile;
  const int split = p.split_lo + lsplit;
  const int tile = bid - lsplit * ntile;
  const int ci_blk = tile / cob, co_blk = tile - ci_blk * cob;
  const int ci0 = ci_blk * 32, co0 = co_blk * 32 * QO;
  const bool from1 = !CONCAT || ci0 < p.M1;
  const int CA = from1 ? p.M1 : p.M2, ca0 = from1 ? ci0 : ci0 - p.M1;
  constexpr int OOB = 0x7fffffff;
  const char* abase = (const char*)(from1 ? p.a1 : p.a2);
  const char* bbase = (const char*)p.b;
  const int w_begin = (int)((long long)split * nwin / p.splits);
  const int w_end = (int)((long long)(split + 1) * nwin / p.splits);
  const bool do_bias = p.bias_mode == 1 && ci_blk == 0;

  f32x4 acc[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  f32x4 bacc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
  const u32x4 ones_u = {kOnes2, kOnes2, kOnes2, kOnes2};
  const h16x8 ones = __builtin_bit_cast(h16x8, ones_u);

  // LDS-DMA lane roles (slot 16k + lslot, physical chunk lane & 3), as wgrad_win_kernel
  const int lslot = lane >> 2;
  const int lchunk = (lane & 3) ^ (((lslot >> 3) & 1) << 1);
  const int xl = ((lslot - 1) * CA + ca0 + lchunk * 8) * 2;
  const int yl = (lslot * p.Nc + co0 + lchunk * 8) * 2;
  const int G = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;

  auto tr_addr = [&](int slot, int col, int ch) -> int {   // ch: channel within the 32-ch slot
    const int swz = ((col >> 3) & 1) << 1;
    return slot * 64 + (((ch >> 3) ^ swz) << 4) + ((ch & 7) << 1);
  };
  auto tr8 = [&](const char* base0, const char* base1) -> h16x8 {
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(short4v, base1));
    const u32x2 l2 = __builtin_bit_cast(u32x2, lo), h2 = __builtin_bit_cast(u32x2, hi);
    const u32x4 v = {l2[0], l2[1], h2[0], h2[1]};
    return __builtin_bit_cast(h16x8, v);
  };

  // stage window `win`: the (R + 2)-row input halo (zero rows outside its image: H % R
  // == 0, a window never spans two images) and the window's dY pixels
  auto stage = [&](const int win, char* st) {
    const int g0 = win * R;
    const bool top_in = (g0 % H) != 0, bot_in = ((g0 + R) % H) != 0;
    const int rb = max(g0 - 1, 0);
    const __amdgpu_buffer_rsrc_t rsa =
        __builtin_amdgcn_make_buffer_rsrc((void*)(abase + (size_t)rb * W * CA * 2), (short)0, OOB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb =
        __builtin_amdgcn_make_buffer_rsrc((void*)(bbase + (size_t)g0 * W * p.Nc * 2), (short)0, OOB, 0x00020000);
#pragma unroll
    for (int qq = 0; qq < (XI + NW - 1) / NW; ++qq) {
      const int k = wave + NW * qq;
      if (k < XI) {
        const int hr = k / IPR, j = k - hr * IPR;
        const int gr = g0 - 1 + hr;
        const int col = 16 * j + lslot - 1;
        const bool row_in = (hr > 0 || top_in) && (hr < R + 1 || bot_in);
        const bool ok = row_in && (unsigned)gr < (unsigned)rows_total && (unsigned)col < (unsigned)W;
        const int off = ok ? ((gr - rb) * W + 16 * j) * CA * 2 + xl : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsa, (__attribute__((address_space(3))) void*)(st + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
    char* Ys = st + XB;
#pragma unroll
    for (int qq = 0; qq < (YI + NW - 1) / NW; ++qq) {
      const int k = wave + NW * qq;
      if (k < YI) {
        const int o = k / (BMW / 16), sb = (k - o * (BMW / 16)) * 16;
        const int pix = g0 * W + sb;
        const int off = (pix + lslot < Mq) ? (sb * p.Nc + 32 * o) * 2 + yl : OOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsb, (__attribute__((address_space(3))) void*)(Ys + k * 1024), 16,
                                                 off, 0, 0, 0);
      }
    }
  };

  // one window's MFMAs from stage `st` (the column-unit / row-pair paths of wgrad_win_kernel)
  auto compute = [&](const char* st) {
    const char* Xs = st;
    const char* Yq = st + XB + qo * (BMW * 64);
    if constexpr (W >= 32) {
      // column units 32 pixels wide x RWG rows, one per wave
      constexpr int NCOL = W / 32;
      constexpr int RG = PS > NCOL ? PS / NCOL : 1;
      constexpr int RWG = R / RG;
      static_assert(R % RG == 0 && RWG >= 1 && NCOL * RG == PS, "wgrad column units: one per wave");
      const int lp = 8 * G + q;
      const int u = ps;
      const int cu = u % NCOL, rr0 = (u / NCOL) * RWG;
      const int c0 = cu * 32;
      int ab[3][2][2], yb[2][2];
#pragma unroll
      for (int dw = 0; dw < 3; ++dw)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int col = c0 + dw + lp + 4 * hh;
            ab[dw][i][hh] = tr_addr(rr0 * HWP + col, col, 16 * i + 4 * pp);
          }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int sl = rr0 * W + c0 + lp + 4 * hh;
          yb[j][hh] = tr_addr(sl, sl, 16 * j + 4 * pp);
        }
      h16x8 bf[RWG][2];
#pragma unroll
      for (int hr = 0; hr < RWG + 2; ++hr) {
        if (hr < RWG) {
#pragma unroll
          for (int j = 0; j < 2; ++j) bf[hr][j] = tr8(Yq + yb[j][0] + hr * W * 64, Yq + yb[j][1] + hr * W * 64);
          if (do_bias) {
#pragma unroll
            for (int j = 0; j < 2; ++j) bacc[j] = mfma16(ones, bf[hr][j], bacc[j]);
          }
        }
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          h16x8 af[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) af[i] = tr8(Xs + ab[dw][i][0] + hr * ROWB, Xs + ab[dw][i][1] + hr * ROWB);
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int y = hr - dh;
            if (y < 0 || y >= RWG) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int j = 0; j < 2; ++j) acc[3 * dh + dw][i][j] = mfma16(af[i], bf[y][j], acc[3 * dh + dw][i][j]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      // 16-wide rows: a 32-pixel K step is a pair of rows; each wave owns NP pairs
      constexpr int NP = R / 2 / PS;
      static_assert(NP >= 1 && NP * 2 * PS == R, "wgrad row pairs");
      const int y0 = ps * 2 * NP;
      const int lp = 8 * G + q;
      const int lr = lp >> 4, lc = lp & 15;
      int ab[3][2][2];
#pragma unroll
      for (int dw = 0; dw < 3; ++dw)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int col = lc + dw + 4 * hh;
            ab[dw][i][hh] = tr_addr((y0 + lr) * HWP + col, col, 16 * i + 4 * pp);
          }
      h16x8 bf[NP][2];
#pragma unroll
      for (int hr = 0; hr <= 2 * NP; ++hr) {
        if (!(hr & 1) && hr < 2 * NP) {
          const int s0 = (y0 + hr) * W + lp, s1 = s0 + 4;
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bf[hr >> 1][j] = tr8(Yq + tr_addr(s0, s0, 16 * j + 4 * pp), Yq + tr_addr(s1, s1, 16 * j + 4 * pp));
          if (do_bias) {
#pragma unroll
            for (int j = 0; j < 2; ++j) bacc[j] = mfma16(ones, bf[hr >> 1][j], bacc[j]);
          }
        }
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          h16x8 af[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) af[i] = tr8(Xs + ab[dw][i][0] + hr * ROWB, Xs + ab[dw][i][1] + hr * ROWB);
#pragma unroll
          for (int dh = 0; dh < 3; ++dh) {
            const int y = hr - dh;
            if (y < 0 || y >= 2 * NP || (y & 1)) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int j = 0; j < 2; ++j)
                acc[3 * dh + dw][i][j] = mfma16(af[i], bf[y >> 1][j], acc[3 * dh + dw][i][j]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  if (w_begin < w_end) stage(w_begin, lds0);
  for (int win = w_begin; win < w_end; win += 2) {
    __syncthreads();                 // window win landed (vmcnt(0) + barrier); stage 1 free
    if (win + 1 < w_end) stage(win + 1, lds1);
    compute(lds0);
    if (win + 1 < w_end) {
      __syncthreads();               // window win + 1 landed; stage 0 free
      if (win + 2 < w_end) stage(win + 2, lds0);
      compute(lds1);
    }
  }

  // ---- reduce the pixel-split partials (waves with the same qo) and write the slab
  // acc[t][i][j][r] = dW[t][ci0 + 16i + 4(lane>>4) + r][co0 + 32qo + 16j + (lane&15)]
  float* red = (float*)lds0;
  const int n_base = co0 + 32 * qo + (lane & 15);
  const int m_base = ci0 + 4 * (lane >> 4);
  auto reduce_store = [&](const f32x4 (&v4)[2][2], const int t) {
    __syncthreads();
    if (ps > 0) {
      float* dst = red + (wave * 64 + lane) * 16;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) *(f32x4*)(dst + (i * 2 + j) * 4) = v4[i][j];
    }
    __syncthreads();
    if (ps == 0) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          f32x4 v = v4[i][j];
#pragma unroll
          for (int o = 1; o < PS; ++o) v += *(const f32x4*)(red + ((qo + QO * o) * 64 + lane) * 16 + (i * 2 + j) * 4);
          if (t < 9) {
            float* dst = p.slab + (((size_t)split * 9 + t) * Mtot + m_base + 16 * i) * p.Nc + n_base + 16 * j;
#pragma unroll
            for (int r = 0; r < 4; ++r) dst[(size_t)r * p.Nc] = v[r];
          } else if (i == 0 && lane < 16) {
            p.bias_slab[(size_t)split * p.Nc + n_base + 16 * j] = v[0];
          }
        }
    }
  };
#pragma unroll
  for (int t = 0; t < 9; ++t) reduce_store(acc[t], t);
  if (do_bias) {
    const f32x4 z = (f32x4){0.f, 0.f, 0.f, 0.f};
    const f32x4 bv[2][2] = {{bacc[0], bacc[1]}, {z, z}};
    reduce_store(bv, 9);
  }
}

template <int W, int QO>
hipError_t launch_w(const WgradParams& p, hipStream_t s) {
  const int splits = p.split_n > 0 ? p.split_n : p.splits - p.split_lo;
  const int grid = ((p.M1 + p.M2) / 32) * (p.Nc / (32 * QO)) * splits;
  if (p.M2 > 0)
    hipLaunchKernelGGL((wgrad_pipe_kernel<W, QO, true>), dim3(grid), dim3(WP_NTHR), 0, s, p);
  else
    hipLaunchKernelGGL((wgrad_pipe_kernel<W, QO, false>), dim3(grid), dim3(WP_NTHR), 0, s, p);
  return hipGetLastError();
}

}  // namespace

// (conv_wgrad.hip checks eligibility: 2D full rows 16..64 wide, H % (256 / W) == 0,
// plain / concat A, no head-on-load / operand transform)
hipError_t launch_wgrad_pipe(const WgradParams& p, hipStream_t s) {
  const bool q2 = p.Nc % 64 == 0;
  switch (p.QW) {
    case 16: return q2 ? launch_w<16, 2>(p, s) : launch_w<16, 1>(p, s);
    case 32: return q2 ? launch_w<32, 2>(p, s) : launch_w<32, 1>(p, s);
    case 64: return q2 ? launch_w<64, 2>(p, s) : launch_w<64, 1>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace unet
