// Python bindings and the native launch-plan executor.
//
// The Python layer never touches the HIP runtime for hot-path work: it passes
// raw device pointers (tensor.data_ptr()) and the current HIP stream handle,
// so this module has no dependency on the PyTorch C++ ABI.
//
// Two ways to launch:
//  * immediate functions (conv_fwd, wgrad, ...) used by the kernel tests
//    (tests/test_gpu_kernels.py) and the tuning scripts;
//  * `Plan`: the UNet executor records every launch of a training step ONCE
//    (all shapes, pointers and epilogue flags resolved at plan time) and then
//    replays ranges of it from C++ with no per-kernel Python overhead.  Ranges
//    are the segments between gradient-bucket boundaries, so the Python side
//    can issue the RCCL allreduce of a finished bucket on the comm stream
//    while the next backward segment runs.
//
// This replaces the reference's TF graph runtime (`test_dist.py:183-298`
// builds the graph, `test_dist.py:396-398` runs one step per sess.run).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <functional>
#include <stdexcept>
#include <string>
#include <tuple>
#include <vector>

#include "launch_api.h"

namespace py = pybind11;
using namespace unet;

namespace {

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void check_msg(const char* msg) {
  if (msg) throw std::invalid_argument(msg);
}

template <typename T>
T get(const py::dict& d, const char* k, T def) {
  if (d.contains(k)) {
    py::object o = d[k];
    if (o.is_none()) return def;
    return o.cast<T>();
  }
  return def;
}

const void* getp(const py::dict& d, const char* k) {
  if (!d.contains(k)) return nullptr;
  py::object o = d[k];
  if (o.is_none()) return nullptr;
  return reinterpret_cast<const void*>(o.cast<uintptr_t>());
}

hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

// head-on-load fields (conv_params.h HeadGrad), hg_* keys of a conv / wgrad dict
HeadGrad head_grad(const py::dict& d) {
  HeadGrad h{};
  h.prob = (const float*)getp(d, "hg_prob");
  h.t = getp(d, "hg_t");
  h.sums = (const float*)getp(d, "hg_sums");
  h.w = (const float*)getp(d, "hg_w");
  h.bits = (const uint8_t*)getp(d, "hg_bits");
  h.gscale = (const float*)getp(d, "hg_gscale");
  h.inv_total = get<float>(d, "hg_inv_total", 0.f);
  h.bce_w = get<float>(d, "hg_bce_w", 0.f);
  h.fa = (const float*)getp(d, "hg_fa");
  h.fc = (const float*)getp(d, "hg_fc");
  return h;
}

ConvFwdParams conv_params(const py::dict& d) {
  ConvFwdParams p{};
  p.N = get<int>(d, "N", 1);
  p.OD = get<int>(d, "OD", 1);
  p.OH = get<int>(d, "OH", 1);
  p.OW = get<int>(d, "OW", 1);
  p.ID = get<int>(d, "ID", 1);
  p.IH = get<int>(d, "IH", 1);
  p.IW = get<int>(d, "IW", 1);
  p.KD = get<int>(d, "KD", 1);
  p.KH = get<int>(d, "KH", 1);
  p.KW = get<int>(d, "KW", 1);
  p.stride = get<int>(d, "stride", 1);
  p.pad = get<int>(d, "pad", 0);
  p.C1 = get<int>(d, "C1", 0);
  p.C2 = get<int>(d, "C2", 0);
  p.up1 = get<int>(d, "up1", 1);
  p.src1 = getp(d, "src1");
  p.src2 = getp(d, "src2");
  p.wgt = getp(d, "wgt");
  p.bias = (const float*)getp(d, "bias");
  p.Cout = get<int>(d, "Cout", 0);
  p.relu = get<int>(d, "relu", 0);
  p.out_scale = get<float>(d, "out_scale", 1.f);
  p.drop_rate = get<float>(d, "drop_rate", 0.f);
  p.seed = get<uint32_t>(d, "seed", 0u);
  p.salt = get<uint32_t>(d, "salt", 0u);
  p.drop_idx0 = get<unsigned long long>(d, "drop_idx0", 0ull);
  p.rev = get<int>(d, "rev", 0);
  p.win_pf = get<int>(d, "win_pf", 0);
  p.win_cp = get<int>(d, "win_cp", 0);
  p.dst1 = const_cast<void*>(getp(d, "dst1"));
  p.dst2 = const_cast<void*>(getp(d, "dst2"));
  p.D1 = get<int>(d, "D1", p.Cout);
  p.mask1 = getp(d, "mask1");
  p.mask2 = getp(d, "mask2");
  p.mask_scale1 = get<float>(d, "mask_scale1", 1.f);
  p.mask_scale2 = get<float>(d, "mask_scale2", 1.f);
  p.shuffle = get<int>(d, "shuffle", 0);
  p.stats = (float*)getp(d, "stats");
  p.nz = getp(d, "nz");
  p.na = (const float*)getp(d, "na");
  p.nc = (const float*)getp(d, "nc");
  p.ncs = get<int>(d, "ncs", 0);
  p.npix = get<int>(d, "npix", 0);
  p.nd_rate = get<float>(d, "nd_rate", 0.f);
  p.nd_salt = get<uint32_t>(d, "nd_salt", 0u);
  p.pool_dst = const_cast<void*>(getp(d, "pool_dst"));
  p.pool_code = (uint32_t*)const_cast<void*>(getp(d, "pool_code"));
  p.relu_bits = (uint8_t*)const_cast<void*>(getp(d, "relu_bits"));
  p.mask_bits = get<int>(d, "mask_bits", 0);
  p.route_gy = getp(d, "route_gy");
  p.xform = get<int>(d, "xform", 0);
  p.xcs = get<int>(d, "xcs", 0);
  p.xa = (const float*)getp(d, "xa");
  p.xb = (const float*)getp(d, "xb");
  p.xc = (const float*)getp(d, "xc");
  p.xz = getp(d, "xz");
  p.s2d = get<int>(d, "s2d", 0);
  p.ut.x = getp(d, "ut_x");
  p.ut.w = getp(d, "ut_w");
  p.ut.b = (const float*)getp(d, "ut_b");
  p.ut.C = get<int>(d, "ut_C", 0);
  p.ut.kpad = get<int>(d, "ut_kpad", 0);
  p.fw.x = getp(d, "fw_x");
  p.fw.slab = (float*)const_cast<void*>(getp(d, "fw_slab"));
  p.fw.bias_slab = (float*)const_cast<void*>(getp(d, "fw_bias_slab"));
  p.fw.Cx = get<int>(d, "fw_Cx", 0);
  p.fw.nsplit = get<int>(d, "fw_nsplit", 0);
  p.fw.split_lo = get<int>(d, "fw_split_lo", 0);
  p.xout = const_cast<void*>(getp(d, "xout"));
  p.xd_rate = get<float>(d, "xd_rate", 0.f);
  p.xd_salt = get<uint32_t>(d, "xd_salt", 0u);
  p.xd_idx0 = get<unsigned long long>(d, "xd_idx0", 0ull);
  p.x2a = (const float*)getp(d, "x2a");
  p.x2b = (const float*)getp(d, "x2b");
  p.x2cs = get<int>(d, "x2cs", 0);
  p.tile = get<int>(d, "tile", 0);
  p.head_w = (const float*)getp(d, "head_w");
  p.head_b = (const float*)getp(d, "head_b");
  p.head_logit = (float*)const_cast<void*>(getp(d, "head_logit"));
  p.head_t = getp(d, "head_t");
  p.head_ws = (float*)const_cast<void*>(getp(d, "head_ws"));
  p.head_nostore = get<int>(d, "head_nostore", 0);
  p.hg = head_grad(d);
  if (!p.src1 || !p.wgt || (!p.dst1 && !(p.head_nostore && p.head_w)))
    throw std::invalid_argument("conv_fwd: src1/wgt/dst1 required");
  check_msg(conv_fwd_prepare(p));
  return p;
}

WgradParams wgrad_params(const py::dict& d) {
  WgradParams p{};
  p.N = get<int>(d, "N", 1);
  p.QD = get<int>(d, "QD", 1);
  p.QH = get<int>(d, "QH", 1);
  p.QW = get<int>(d, "QW", 1);
  p.AD = get<int>(d, "AD", 1);
  p.AH = get<int>(d, "AH", 1);
  p.AW = get<int>(d, "AW", 1);
  p.KD = get<int>(d, "KD", 1);
  p.KH = get<int>(d, "KH", 1);
  p.KW = get<int>(d, "KW", 1);
  p.stride = get<int>(d, "stride", 1);
  p.pad = get<int>(d, "pad", 0);
  p.M1 = get<int>(d, "M1", 0);
  p.M2 = get<int>(d, "M2", 0);
  p.upA = get<int>(d, "upA", 1);
  p.a1 = getp(d, "a1");
  p.a2 = getp(d, "a2");
  p.b = getp(d, "b");
  p.Nc = get<int>(d, "Nc", 0);
  p.splits = get<int>(d, "splits", 1);
  p.split_lo = get<int>(d, "split_lo", 0);
  p.split_n = get<int>(d, "split_n", 0);
  p.tap_groups = 1;
  p.slab = (float*)getp(d, "slab");
  p.bias_mode = get<int>(d, "bias_mode", 0);
  p.bias_slab = (float*)getp(d, "bias_slab");
  p.win = get<int>(d, "win", 0);
  p.xform = get<int>(d, "xform", 0);
  p.xcs = get<int>(d, "xcs", 0);
  p.xa = (const float*)getp(d, "xa");
  p.xb = (const float*)getp(d, "xb");
  p.xc = (const float*)getp(d, "xc");
  p.xz = getp(d, "xz");
  p.pair = get<int>(d, "pair", 0);
  p.pf = get<int>(d, "pf", 0);
  p.hg = head_grad(d);
  if (p.bias_mode && !p.bias_slab) throw std::invalid_argument("wgrad: bias_slab required");
  if (!p.a1 || !p.b || !p.slab) throw std::invalid_argument("wgrad: a1/b/slab required");
  check_msg(wgrad_check(p));
  return p;
}

F32Conv f32_conv_params(const py::dict& d) {
  F32Conv p{};
  p.N = get<int>(d, "N", 1);
  p.OD = get<int>(d, "OD", 1);
  p.OH = get<int>(d, "OH", 1);
  p.OW = get<int>(d, "OW", 1);
  p.ID = get<int>(d, "ID", 1);
  p.IH = get<int>(d, "IH", 1);
  p.IW = get<int>(d, "IW", 1);
  p.KD = get<int>(d, "KD", 1);
  p.KH = get<int>(d, "KH", 1);
  p.KW = get<int>(d, "KW", 1);
  p.stride = get<int>(d, "stride", 1);
  p.pad = get<int>(d, "pad", 0);
  p.C1 = get<int>(d, "C1", 0);
  p.C2 = get<int>(d, "C2", 0);
  p.Cout = get<int>(d, "Cout", 0);
  p.src1 = (const float*)getp(d, "src1");
  p.src2 = (const float*)getp(d, "src2");
  p.wgt = (const float*)getp(d, "wgt");
  p.bias = (const float*)getp(d, "bias");
  p.dst = (float*)const_cast<void*>(getp(d, "dst1"));
  p.relu = get<int>(d, "relu", 0);
  p.drop_rate = get<float>(d, "drop_rate", 0.f);
  p.seed = get<uint32_t>(d, "seed", 0u);
  p.salt = get<uint32_t>(d, "salt", 0u);
  p.drop_idx0 = get<unsigned long long>(d, "drop_idx0", 0ull);
  p.mask = (const float*)getp(d, "mask1");
  p.mask_scale = get<float>(d, "mask_scale1", 1.f);
  p.shuffle = get<int>(d, "shuffle", 0);
  p.ldw = get<int>(d, "ldw", p.Cout);
  check_msg(unet::f32_conv_check(p));
  return p;
}

F32Wgrad f32_wgrad_params(const py::dict& d) {
  F32Wgrad p{};
  p.N = get<int>(d, "N", 1);
  p.QD = get<int>(d, "QD", 1);
  p.QH = get<int>(d, "QH", 1);
  p.QW = get<int>(d, "QW", 1);
  p.AD = get<int>(d, "AD", 1);
  p.AH = get<int>(d, "AH", 1);
  p.AW = get<int>(d, "AW", 1);
  p.KD = get<int>(d, "KD", 1);
  p.KH = get<int>(d, "KH", 1);
  p.KW = get<int>(d, "KW", 1);
  p.stride = get<int>(d, "stride", 1);
  p.pad = get<int>(d, "pad", 0);
  p.M1 = get<int>(d, "M1", 0);
  p.M2 = get<int>(d, "M2", 0);
  p.Nc = get<int>(d, "Nc", 0);
  p.a1 = (const float*)getp(d, "a1");
  p.a2 = (const float*)getp(d, "a2");
  p.b = (const float*)getp(d, "b");
  p.slab = (float*)const_cast<void*>(getp(d, "slab"));
  p.splits = get<int>(d, "splits", 1);
  check_msg(unet::f32_wgrad_check(p));
  return p;
}

// Kernel launchers of one element-type build.  dtype 0 = bf16 (namespace unet),
// 1 = fp16 (namespace unet_f16); host-only helpers (prepare / pick / check) are
// element-type independent and always come from the bf16 build.
#define UNET_KERNEL_FNS(X) \
  X(conv_fwd_launch) \
  X(wgrad_launch) \
  X(wgrad_reduce_launch) \
  X(multi_reduce_launch) \
  X(colsum_launch) \
  X(cast_input_launch) \
  X(gather_batch_launch) \
  X(maxpool2_fwd_launch) \
  X(norm_pool_launch) \
  X(maxpool2_bwd_launch) \
  X(maxpool2_bwd_norm_launch) \
  X(upsample2_bwd_launch) \
  X(upsample2_fwd_launch) \
  X(head_fwd_launch) \
  X(head_bwd_launch) \
  X(head_wsum_grad_launch) \
  X(head_dy_launch) \
  X(partial_reduce_launch) \
  X(head_finish_launch) \
  X(norm_head_launch) \
  X(norm_head_loss_launch) \
  X(head_norm_coef_launch) \
  X(head_norm_bwd_launch) \
  X(norm_moments_launch) \
  X(moments_collect_launch) \
  X(bn_stats_launch) \
  X(gn_stats_launch) \
  X(norm_rows_launch) \
  X(bn_finalize_launch) \
  X(gn_finalize_launch) \
  X(norm_apply_launch) \
  X(norm_bwd_apply_launch) \
  X(tconv_compose_launch) \
  X(tconv_chain_launch) \
  X(adam_pack_launch)

struct KernelApi {
#define UNET_DECL(f) decltype(&unet::f) f;
  UNET_KERNEL_FNS(UNET_DECL)
#undef UNET_DECL
};

#define UNET_BF16(f) &unet::f,
#define UNET_F16(f) &unet_f16::f,
const KernelApi kApi[2] = {{UNET_KERNEL_FNS(UNET_BF16)}, {UNET_KERNEL_FNS(UNET_F16)}};
#undef UNET_BF16
#undef UNET_F16

const KernelApi* api(int dtype) {
  if (dtype != 0 && dtype != 1) throw std::invalid_argument("dtype must be 0 (bf16) or 1 (fp16)");
  return &kApi[dtype];
}

using Launcher = std::function<hipError_t(hipStream_t)>;

// generic memory-bound ops: (kind, pointer args, int args, float args)
// seedp: the owning plan's per-step dropout seed (nullptr for immediate calls: the
// seed is then the op's last int argument); seed_devp: the plan's device seed pointer
// (set for HIP-graph capture, where kernel arguments are frozen at capture time)
Launcher make_generic(const KernelApi* A, const std::string& kind, const std::vector<uintptr_t>& P,
                      const std::vector<long long>& I, const std::vector<double>& F, const uint32_t* seedp = nullptr,
                      const uint32_t* const* seed_devp = nullptr) {
  auto need = [&](size_t np, size_t ni, size_t nf) {
    if (P.size() < np || I.size() < ni || F.size() < nf)
      throw std::invalid_argument("generic op '" + kind + "': wrong argument count");
  };
  auto vp = [&](int i) { return reinterpret_cast<void*>(P[i]); };
  if (kind == "cast_input") {
    need(2, 3, 0);
    const float* x = (const float*)vp(0);
    void* y = vp(1);
    int a = I[0], b = I[1], c = I[2];
    return [=](hipStream_t s) { return A->cast_input_launch(x, a, b, c, y, s); };
  }
  if (kind == "gather_batch") {
    // ptrs: x_all, y_all, idx (int64, device), xb, tb   ints: B, P, Cin, Cpad
    need(5, 4, 0);
    const float *xa = (const float*)vp(0), *ya = (const float*)vp(1);
    const long long* ix = (const long long*)vp(2);
    void *xb = vp(3), *tb = vp(4);
    int B = I[0], P_ = I[1], cin = I[2], cpad = I[3];
    if (cin > cpad || cpad > 64) throw std::invalid_argument("gather_batch: Cin <= Cpad <= 64");
    return [=](hipStream_t s) { return A->gather_batch_launch(xa, ya, ix, B, P_, cin, cpad, xb, tb, s); };
  }
  if (kind == "pool_fwd") {
    // ptrs: x, y[, code]
    need(2, 6, 0);
    void *x = vp(0), *y = vp(1), *code = P.size() > 2 ? vp(2) : nullptr;
    int n = I[0], d = I[1], h = I[2], w = I[3], c = I[4], d3 = I[5];
    if (c % 8) throw std::invalid_argument("pool: C % 8");
    if ((long long)n * d * h * w * c >= (1LL << 31)) throw std::invalid_argument("pool: too many elements");
    return [=](hipStream_t s) { return A->maxpool2_fwd_launch(x, n, d, h, w, c, d3, y, code, s); };
  }
  if (kind == "norm_pool") {
    // ptrs: z, fa, fc, y, pooled y, code   ints: N, D, H, W, C, dims3, cstride
    need(6, 7, 0);
    const void* z = vp(0);
    const float *fa = (const float*)vp(1), *fc = (const float*)vp(2);
    void *y = vp(3), *py = vp(4), *code = vp(5);
    int n = I[0], d = I[1], h = I[2], w = I[3], c = I[4], d3 = I[5], cs = I[6];
    if (c % 8 || (cs != 0 && cs != c)) throw std::invalid_argument("norm_pool: C % 8, cstride 0 or C");
    if ((long long)n * d * h * w * c >= (1LL << 31)) throw std::invalid_argument("norm_pool: too many elements");
    return [=](hipStream_t s) { return A->norm_pool_launch(z, fa, fc, cs, n, d, h, w, c, d3, y, py, code, s); };
  }
  if (kind == "pool_bwd") {
    // ptrs: x, dy, skip, dx[, code]  (code non-null: argmax codes of pool_fwd, x unused)
    need(4, 6, 0);
    void *x = vp(0), *dy = vp(1), *sk = vp(2), *dx = vp(3), *code = P.size() > 4 ? vp(4) : nullptr;
    int n = I[0], d = I[1], h = I[2], w = I[3], c = I[4], d3 = I[5];
    if (c % 8) throw std::invalid_argument("pool: C % 8");
    if ((long long)n * d * h * w * c >= (1LL << 31)) throw std::invalid_argument("pool: too many elements");
    return [=](hipStream_t s) { return A->maxpool2_bwd_launch(x, code, dy, sk, n, d, h, w, c, d3, dx, s); };
  }
  if (kind == "pool_bwd_norm") {
    // ptrs: code, dy, skip, z, dx, rows   ints: N, D, H, W, C, dims3, nbp
    need(6, 7, 0);
    void *code = vp(0), *dy = vp(1), *sk = vp(2), *z = vp(3), *dx = vp(4);
    float* rows = (float*)vp(5);
    int n = I[0], d = I[1], h = I[2], w = I[3], c = I[4], d3 = I[5], nbp = I[6];
    if (c % 8 || 256 % (c / 8)) throw std::invalid_argument("pool_bwd_norm: C % 8, 256 % (C / 8)");
    if ((long long)n * d * h * w * c >= (1LL << 31)) throw std::invalid_argument("pool: too many elements");
    return [=](hipStream_t s) { return A->maxpool2_bwd_norm_launch(code, dy, sk, z, n, d, h, w, c, d3, nbp, dx, rows, s); };
  }
  if (kind == "ups_fwd") {
    // ptrs: low-res x, full-res y; ints: N, D, H, W (low resolution), C, dims3
    need(2, 6, 0);
    void *x = vp(0), *y = vp(1);
    int n = I[0], d = I[1], h = I[2], w = I[3], c = I[4], d3 = I[5];
    if (c % 8) throw std::invalid_argument("ups_fwd: C % 8");
    if ((long long)n * d * h * w * c * (d3 ? 8 : 4) >= (1LL << 31)) throw std::invalid_argument("ups_fwd: too large");
    return [=](hipStream_t s) { return A->upsample2_fwd_launch(x, n, d, h, w, c, d3, y, s); };
  }
  if (kind == "ups_bwd") {
    need(3, 6, 0);
    void *du = vp(0), *mk = vp(1), *dl = vp(2);
    int n = I[0], d = I[1], h = I[2], w = I[3], c = I[4], d3 = I[5];
    if (c % 8) throw std::invalid_argument("ups_bwd: C % 8");
    return [=](hipStream_t s) { return A->upsample2_bwd_launch(du, mk, n, d, h, w, c, d3, dl, s); };
  }
  if (kind == "wgrad_reduce") {
    // ptrs: slab, out[, stage]   ints: splits, taps, Mtot, Mout, Nc[, rg, rkeep]
    need(2, 5, 1);
    const float* slab = (const float*)vp(0);
    float* out = (float*)vp(1);
    float* stage = P.size() > 2 ? (float*)vp(2) : nullptr;
    int sp = I[0], taps = I[1], mt = I[2], mo = I[3], nc = I[4];
    int rg = I.size() > 5 ? (int)I[5] : 0, rk = I.size() > 6 ? (int)I[6] : 0;
    float sc = (float)F[0];
    if (nc % 4) throw std::invalid_argument("wgrad_reduce: Nc % 4");
    const bool identity = (mo == mt) && (rg == rk);
    if (!stage && !(identity && sp <= 16))
      throw std::invalid_argument("wgrad_reduce: stage buffer required for >16 splits or row remap");
    return [=](hipStream_t s) { return A->wgrad_reduce_launch(slab, sp, taps, mt, mo, nc, rg, rk, sc, out, stage, s); };
  }
  if (kind == "tconv_compose") {
    // ptrs: Wt master [4][C][K], Wa master [3][3][Ca][O], out [K][rowstride]   ints: C, K, O, Ca, rowstride
    need(3, 5, 0);
    const float *wt = (const float*)vp(0), *wa = (const float*)vp(1);
    void* out = vp(2);
    int C = I[0], K = I[1], O = I[2], Ca = I[3], rs = I[4];
    check_msg(tconv_fused_check(C, K, O, Ca));
    if (rs < 36 * O) throw std::invalid_argument("tconv_compose: rowstride < 36 O");
    return [=](hipStream_t s) { return A->tconv_compose_launch(wt, wa, C, K, O, Ca, rs, out, s); };
  }
  if (kind == "tconv_chain") {
    // ptrs: H [16][O][K], Bs [16][O], Wa master, dWt [4][C][K], dbt [C]
    //       [, Wt master, bt master, skip-row gradient [9][Ca - C][O], dWa [9][Ca][O]]   ints: C, K, O, Ca
    if (P.size() != 5 && P.size() != 9) throw std::invalid_argument("tconv_chain: 5 or 9 pointers");
    need((int)P.size(), 4, 0);
    const float *hs = (const float*)vp(0), *bs = (const float*)vp(1), *wa = (const float*)vp(2);
    float *dwt = (float*)vp(3), *dbt = (float*)vp(4);
    const float* wt = P.size() == 9 ? (const float*)vp(5) : nullptr;
    const float* bt = P.size() == 9 ? (const float*)vp(6) : nullptr;
    const float* skg = P.size() == 9 ? (const float*)vp(7) : nullptr;
    float* dwa = P.size() == 9 ? (float*)vp(8) : nullptr;
    int C = I[0], K = I[1], O = I[2], Ca = I[3];
    check_msg(tconv_fused_check(C, K, O, Ca));
    if (dwa && (!wt || !bt || (Ca > C && !skg))) throw std::invalid_argument("tconv_chain: dWa needs Wt, bt, skip rows");
    return [=](hipStream_t s) {
      return A->tconv_chain_launch(hs, bs, wa, C, K, O, Ca, dwt, dbt, wt, bt, skg, dwa, s);
    };
  }
  if (kind == "multi_reduce") {
    // ptrs: job table (device, ReduceJob[njobs])   ints: njobs, total1, total2
    need(1, 3, 0);
    const void* jobs = vp(0);
    int nj = (int)I[0];
    long long t1 = I[1], t2 = I[2];
    return [=](hipStream_t s) { return A->multi_reduce_launch(jobs, nj, t1, t2, s); };
  }
  if (kind == "colsum") {
    need(2, 3, 0);
    void* x = vp(0);
    float* part = (float*)vp(1);
    int rows = I[0], c = I[1], blocks = I[2];
    if (c % 8 || c > 2048) throw std::invalid_argument("colsum: C % 8 / C > 2048");
    return [=](hipStream_t s) { return A->colsum_launch(x, rows, c, blocks, part, s); };
  }
  if (kind == "head_finish") {
    need(4, 1, 0);
    float* prob = (float*)vp(0);
    const void* t = vp(1);
    float *part = (float*)vp(2), *sums = (float*)vp(3);
    int P_ = I[0];
    return [=](hipStream_t s) { return A->head_finish_launch(prob, t, P_, part, sums, s); };
  }
  if (kind == "norm_head") {
    // ptrs: z, fa, fc, w, b, y, logit   ints: P, C, cstride, npix
    need(7, 4, 0);
    const void* z = vp(0);
    const float *fa = (const float*)vp(1), *fc = (const float*)vp(2), *w = (const float*)vp(3),
                *bb = (const float*)vp(4);
    void* y = vp(5);
    float* lg = (float*)vp(6);
    int P_ = I[0], C = I[1], cs = I[2], np_ = I[3];
    check_msg(head_check(C));
    if ((cs != 0 && cs != C) || np_ <= 0) throw std::invalid_argument("norm_head: cstride 0 or C, npix > 0");
    return [=](hipStream_t s) { return A->norm_head_launch(z, fa, fc, cs, np_, w, bb, P_, C, y, lg, s); };
  }
  if (kind == "norm_head_loss") {
    // ptrs: z, fa, fc, w, b, t, y (0: not stored), prob, partial, sums
    // ints: N, npix, C, cstride   (partial: hn_partial_floats(N, npix, C) floats)
    need(10, 4, 0);
    const void *z = vp(0), *t = vp(5);
    const float *fa = (const float*)vp(1), *fc = (const float*)vp(2), *w = (const float*)vp(3),
                *bb = (const float*)vp(4);
    void* y = vp(6);
    float *prob = (float*)vp(7), *part = (float*)vp(8), *sums = (float*)vp(9);
    int n = I[0], np_ = I[1], C = I[2], cs = I[3];
    check_msg(head_check(C));
    if ((cs != 0 && cs != C) || np_ <= 0 || n <= 0) throw std::invalid_argument("norm_head_loss: cstride 0 or C");
    return [=](hipStream_t s) {
      return A->norm_head_loss_launch(z, fa, fc, cs, n, np_, w, bb, t, y, C, prob, part, sums, s);
    };
  }
  if (kind == "head_norm_coef") {
    // ptrs: partial, sums, w, fa, fc, rows, gw, gb [, gscale_ptr]   ints: N, npix, C, cstride
    // floats: inv_total, bce_w, gscale    (rows: N * hn_blocks_per_sample x 2 x C)
    need(8, 4, 3);
    const float *part = (const float*)vp(0), *sums = (const float*)vp(1), *w = (const float*)vp(2),
                *fa = (const float*)vp(3), *fc = (const float*)vp(4);
    float *rows = (float*)vp(5), *gw = (float*)vp(6), *gb = (float*)vp(7);
    const float* gsp = P.size() > 8 ? (const float*)vp(8) : nullptr;
    int n = I[0], np_ = I[1], C = I[2], cs = I[3];
    check_msg(head_check(C));
    if (cs != 0 && cs != C) throw std::invalid_argument("head_norm_coef: cstride 0 or C");
    float it = (float)F[0], bw = (float)F[1], gs = (float)F[2];
    return [=](hipStream_t s) {
      return A->head_norm_coef_launch(part, n, np_, C, sums, w, fa, fc, cs, it, bw, gs, gsp, rows, gw, gb, s);
    };
  }
  if (kind == "head_norm_bwd") {
    // ptrs: z, prob, t, sums, w, fa, fc, ca, cb, cc, dz [, gscale_ptr]   ints: N, P, C, cstride
    // floats: inv_total, bce_w, gscale
    need(11, 4, 3);
    const void *z = vp(0), *t = vp(2);
    const float *prob = (const float*)vp(1), *sums = (const float*)vp(3), *w = (const float*)vp(4),
                *fa = (const float*)vp(5), *fc = (const float*)vp(6), *ca = (const float*)vp(7),
                *cb = (const float*)vp(8), *cc = (const float*)vp(9);
    void* dz = vp(10);
    const float* gsp = P.size() > 11 ? (const float*)vp(11) : nullptr;
    int n = I[0], np_ = I[1], C = I[2], cs = I[3];
    check_msg(norm_check(C, 0));
    if (cs != 0 && cs != C) throw std::invalid_argument("head_norm_bwd: cstride 0 or C");
    float it = (float)F[0], bw = (float)F[1], gs = (float)F[2];
    return [=](hipStream_t s) {
      return A->head_norm_bwd_launch(z, prob, t, sums, w, fa, fc, ca, cb, cc, cs, n, np_, C, it, bw, gs, gsp, dz, s);
    };
  }
  if (kind == "partial_reduce") {
    need(2, 2, 0);
    const float* part = (const float*)vp(0);
    float* out = (float*)vp(1);
    int nb = I[0], width = I[1];
    return [=](hipStream_t s) { return A->partial_reduce_launch(part, nb, width, out, s); };
  }
  if (kind == "head_fwd") {
    need(7, 2, 0);
    void* x = vp(0);
    const float *w = (const float*)vp(1), *b = (const float*)vp(2);
    void* t = vp(3);
    float *prob = (float*)vp(4), *part = (float*)vp(5), *sums = (float*)vp(6);
    int P_ = I[0], C = I[1];
    check_msg(head_check(C));
    return [=](hipStream_t s) { return A->head_fwd_launch(x, w, b, t, P_, C, prob, part, sums, s); };
  }
  if (kind == "head_bwd") {
    need(9, 2, 3);
    void* x = vp(0);
    const float* w = (const float*)vp(1);
    const float* prob = (const float*)vp(2);
    void* t = vp(3);
    const float* sums = (const float*)vp(4);
    void* dx = vp(5);
    float *part = (float*)vp(6), *gw = (float*)vp(7), *gb = (float*)vp(8);
    int P_ = I[0], C = I[1];
    // optional 10th pointer: device float loss scale (overrides floats[2])
    const float* gsp = P.size() > 9 ? (const float*)vp(9) : nullptr;
    float it = (float)F[0], bw = (float)F[1], gs = (float)F[2];
    check_msg(head_check(C));
    return [=](hipStream_t s) {
      return A->head_bwd_launch(x, w, prob, t, sums, P_, C, it, bw, gs, gsp, dx, part, gw, gb, s);
    };
  }
  if (kind == "head_dy") {
    // ptrs: relu bits, w, prob, t, sums, dx [, device loss scale]   ints: P, C   floats: inv_total, bce_w, gscale
    need(6, 2, 3);
    void *bits = vp(0), *t = vp(3), *dx = vp(5);
    const float *w = (const float*)vp(1), *prob = (const float*)vp(2), *sums = (const float*)vp(4);
    const float* gsp = P.size() > 6 ? (const float*)vp(6) : nullptr;
    const int P_ = (int)I[0], C = (int)I[1];
    const float it = (float)F[0], bw = (float)F[1], gs = (float)F[2];
    check_msg(head_check(C));
    return [=](hipStream_t s) { return A->head_dy_launch(bits, w, prob, t, sums, P_, C, it, bw, gs, gsp, dx, s); };
  }
  if (kind == "head_wsum_grad") {
    // ptrs: rows (head_ws), sums, gw, gb [, device loss scale]   ints: nrows   floats: inv_total, bce_w, gscale
    need(4, 1, 3);
    const float *rows = (const float*)vp(0), *sums = (const float*)vp(1);
    float *gw = (float*)vp(2), *gb = (float*)vp(3);
    const float* gsp = P.size() > 4 ? (const float*)vp(4) : nullptr;
    const int nr = (int)I[0];
    const float it = (float)F[0], bw = (float)F[1], gs = (float)F[2];
    return [=](hipStream_t s) { return A->head_wsum_grad_launch(rows, nr, sums, it, bw, gs, gsp, gw, gb, s); };
  }
  if (kind == "norm_moments") {
    // ptrs: A, B, partial, S   ints: N, P, C    (S[n][2][C] = per-sample sums of A and A*B)
    need(4, 3, 0);
    void *a = vp(0), *b = vp(1);
    float *part = (float*)vp(2), *S = (float*)vp(3);
    int n = I[0], np = I[1], c = I[2];
    check_msg(norm_check(c, 0));
    return [=](hipStream_t s) { return A->norm_moments_launch(a, b, n, np, c, part, S, s); };
  }
  if (kind == "bn_finalize") {
    // ptrs: S, gamma, run_mean, run_var, mean, rstd, ca, cb, cc, dgamma, dbeta, partial[, beta, fa, fc]
    // ints: N, C, mode   floats: count, eps, momentum   (partial: sample_slices(N) * 2 * C floats of
    // workspace; fa / fc: forward modes also write the relu-input coefficients gamma r, beta - mu gamma r)
    need(12, 3, 3);
    const float* bt = P.size() > 14 ? (const float*)vp(12) : nullptr;
    float* fa = P.size() > 14 ? (float*)vp(13) : nullptr;
    float* fc = P.size() > 14 ? (float*)vp(14) : nullptr;
    const float* S = (const float*)vp(0);
    const float* gm = (const float*)vp(1);
    float *rm = (float*)vp(2), *rv = (float*)vp(3), *mu = (float*)vp(4), *rs = (float*)vp(5);
    float *ca = (float*)vp(6), *cb = (float*)vp(7), *cc = (float*)vp(8), *dg = (float*)vp(9), *db = (float*)vp(10);
    int n = I[0], c = I[1], mode = I[2];
    float* pt = (float*)vp(11);
    float cnt = (float)F[0], eps = (float)F[1], mom = (float)F[2];
    if (mode != 2 && !pt) throw std::invalid_argument("bn_finalize: partial workspace required");
    return [=](hipStream_t s) {
      return A->bn_finalize_launch(S, n, c, cnt, mode, gm, eps, mom, rm, rv, mu, rs, ca, cb, cc, dg, db, pt, bt, fa, fc,
                                   s);
    };
  }
  if (kind == "gn_finalize") {
    // ptrs: S, gamma, mean, rstd, ca, cb, cc, dgamma, dbeta, partial[, beta, fa, fc]
    // ints: N, C, G, P, mode   floats: eps
    need(10, 5, 1);
    const float* bt = P.size() > 12 ? (const float*)vp(10) : nullptr;
    float* fa = P.size() > 12 ? (float*)vp(11) : nullptr;
    float* fc = P.size() > 12 ? (float*)vp(12) : nullptr;
    const float* S = (const float*)vp(0);
    const float* gm = (const float*)vp(1);
    float *mu = (float*)vp(2), *rs = (float*)vp(3), *ca = (float*)vp(4), *cb = (float*)vp(5), *cc = (float*)vp(6);
    float *dg = (float*)vp(7), *db = (float*)vp(8);
    int n = I[0], c = I[1], g = I[2], np = I[3], mode = I[4];
    float* pt = (float*)vp(9);
    float eps = (float)F[0];
    check_msg(norm_check(c, g));
    if (mode == 1 && !pt) throw std::invalid_argument("gn_finalize: partial workspace required");
    return [=](hipStream_t s) {
      return A->gn_finalize_launch(S, n, c, g, np, mode, gm, eps, mu, rs, ca, cb, cc, dg, db, pt, bt, fa, fc, s);
    };
  }
  if (kind == "bn_stats") {
    // ptrs: rows, gamma, beta, run_mean, run_var, mean, rstd, fa, fc, ca, cb, cc, dgamma, dbeta, slices
    // ints: R, C, mode   floats: count, eps, momentum
    need(15, 3, 3);
    std::vector<float*> q(15);
    for (int i = 0; i < 15; ++i) q[i] = (float*)vp(i);
    int R = I[0], c = I[1], mode = I[2];
    float cnt = (float)F[0], eps = (float)F[1], mom = (float)F[2];
    if (c % 8) throw std::invalid_argument("bn_stats: C % 8");
    return [=](hipStream_t s) {
      return A->bn_stats_launch(q[0], R, c, cnt, mode, q[1], q[2], eps, mom, q[3], q[4], q[5], q[6], q[7], q[8], q[9],
                                q[10], q[11], q[12], q[13], q[14], s);
    };
  }
  if (kind == "gn_stats") {
    // ptrs: rows, gamma, beta, mean, rstd, fa, fc, ca, cb, cc, dgamma, dbeta, work
    // ints: N, rps, C, G, P, mode   floats: eps
    need(13, 6, 1);
    std::vector<float*> q(13);
    for (int i = 0; i < 13; ++i) q[i] = (float*)vp(i);
    int n = I[0], rps = I[1], c = I[2], g = I[3], np = I[4], mode = I[5];
    float eps = (float)F[0];
    check_msg(norm_check(c, g));
    return [=](hipStream_t s) {
      return A->gn_stats_launch(q[0], n, rps, c, g, np, mode, q[1], q[2], eps, q[3], q[4], q[5], q[6], q[7], q[8], q[9],
                                q[10], q[11], q[12], s);
    };
  }
  if (kind == "norm_rows") {
    // ptrs: A, B, rows   ints: N, P, C   (rows[N * norm_blocks_per_sample][2][C])
    need(3, 3, 0);
    void *a = vp(0), *b = vp(1);
    float* rows = (float*)vp(2);
    int n = I[0], np = I[1], c = I[2];
    check_msg(norm_check(c, 0));
    return [=](hipStream_t s) { return A->norm_rows_launch(a, b, n, np, c, rows, s); };
  }
  if (kind == "stat_collect") {
    // ptrs: partial rows, S   ints: N, C, nbp   (S[n][2][C] = sum of rows n*nbp .. n*nbp + nbp - 1)
    need(2, 3, 0);
    const float* part = (const float*)vp(0);
    float* S = (float*)vp(1);
    int n = I[0], c = I[1], nbp = I[2];
    return [=](hipStream_t s) { return A->moments_collect_launch(part, n, c, nbp, S, s); };
  }
  if (kind == "norm_apply") {
    // ptrs: z, mean, rstd, gamma, beta, y   ints: N, P, C, cstride, relu, salt[, seed[, n0]]   floats: drop_rate
    // (n0: first sample of the launch in the whole batch -- dropout hash indices)
    need(6, 6, 1);
    void* z = vp(0);
    const float *mu = (const float*)vp(1), *rs = (const float*)vp(2), *gm = (const float*)vp(3),
                *bt = (const float*)vp(4);
    void* y = vp(5);
    int n = I[0], np = I[1], c = I[2], cs = I[3], relu = I[4];
    uint32_t salt = (uint32_t)I[5], seed0 = I.size() > 6 ? (uint32_t)I[6] : 0u;
    const int n0 = I.size() > 7 ? (int)I[7] : 0;
    float dr = (float)F[0];
    check_msg(norm_check(c, 0));
    return [=](hipStream_t s) {
      return A->norm_apply_launch(z, n, np, c, mu, rs, cs, gm, bt, relu, dr, seedp ? *seedp : seed0,
                               seed_devp ? *seed_devp : nullptr, salt, n0, y, s);
    };
  }
  if (kind == "norm_bwd_apply") {
    // ptrs: g, z, ca, cb, cc, dz   ints: N, P, C, cstride
    need(6, 4, 0);
    void *g = vp(0), *z = vp(1);
    const float *ca = (const float*)vp(2), *cb = (const float*)vp(3), *cc = (const float*)vp(4);
    void* dz = vp(5);
    int n = I[0], np = I[1], c = I[2], cs = I[3];
    check_msg(norm_check(c, 0));
    return [=](hipStream_t s) { return A->norm_bwd_apply_launch(g, z, n, np, c, ca, cb, cc, cs, dz, s); };
  }
  if (kind == "memset") {
    need(1, 1, 0);
    void* p = vp(0);
    size_t bytes = (size_t)I[0];
    return [=](hipStream_t s) { return unet_types::dry_dispatch() ? hipSuccess : hipMemsetAsync(p, 0, bytes, s); };
  }
  // fp32 path (f32.hip; element-type independent, from the bf16 build)
  auto fp = [&](int i) { return reinterpret_cast<float*>(P[i]); };
  if (kind == "f32_pool_fwd" || kind == "f32_ups_fwd") {
    // ptrs: x, y   ints: N, D, H, W (input resolution; ups: the low one), C, dims3
    need(2, 6, 0);
    const float* x = fp(0);
    float* y = fp(1);
    int n = I[0], dd = I[1], hh = I[2], ww = I[3], c = I[4], d3 = I[5];
    if (kind == "f32_pool_fwd") return [=](hipStream_t s) { return unet::f32_pool_fwd_launch(x, n, dd, hh, ww, c, d3, y, s); };
    return [=](hipStream_t s) { return unet::f32_ups_launch(x, nullptr, n, dd, hh, ww, c, d3, 0, y, s); };
  }
  if (kind == "f32_pool_bwd") {
    // ptrs: x (pool input), dy (pooled gradient), skip (or 0), dx   ints: N, D, H, W, C, dims3
    need(4, 6, 0);
    const float *x = fp(0), *dy = fp(1), *sk = fp(2);
    float* dx = fp(3);
    int n = I[0], dd = I[1], hh = I[2], ww = I[3], c = I[4], d3 = I[5];
    return [=](hipStream_t s) { return unet::f32_pool_bwd_launch(x, dy, sk, n, dd, hh, ww, c, d3, dx, s); };
  }
  if (kind == "f32_ups_bwd") {
    // ptrs: full-resolution gradient, low-resolution mask (or 0), low-resolution gradient
    // ints: N, D, H, W (low resolution), C, dims3
    need(3, 6, 0);
    const float *g = fp(0), *mk = fp(1);
    float* dl = fp(2);
    int n = I[0], dd = I[1], hh = I[2], ww = I[3], c = I[4], d3 = I[5];
    return [=](hipStream_t s) { return unet::f32_ups_launch(g, mk, n, dd, hh, ww, c, d3, 1, dl, s); };
  }
  if (kind == "f32_head_fwd") {
    // ptrs: x, w, b, t (or 0), prob, partial, sums   ints: P, C
    need(7, 2, 0);
    const float *x = fp(0), *w = fp(1), *b = fp(2), *t = fp(3);
    float *pr = fp(4), *pa = fp(5), *su = fp(6);
    int np = I[0], c = I[1];
    return [=](hipStream_t s) { return unet::f32_head_fwd_launch(x, w, b, t, np, c, pr, pa, su, s); };
  }
  if (kind == "f32_head_bwd") {
    // ptrs: x, w, prob, t, sums, dx (or 0), partial, gw, gb   ints: P, C   floats: inv_total, bce_w
    need(9, 2, 2);
    const float *x = fp(0), *w = fp(1), *pr = fp(2), *t = fp(3), *su = fp(4);
    float *dx = fp(5), *pa = fp(6), *gw = fp(7), *gb = fp(8);
    int np = I[0], c = I[1];
    float it = (float)F[0], bw = (float)F[1];
    return [=](hipStream_t s) { return unet::f32_head_bwd_launch(x, w, pr, t, su, np, c, it, bw, dx, pa, gw, gb, s); };
  }
  if (kind == "f32_colsum") {
    // ptrs: x [rows][C], partial [blocks][C], out [C]   ints: rows, C, blocks
    need(3, 3, 0);
    const float* x = fp(0);
    float *pa = fp(1), *out = fp(2);
    long long rows = I[0];
    int c = I[1], nb = I[2];
    if (c % 4 || c <= 0 || c > 1024 || nb < 1) throw std::invalid_argument("f32_colsum: C % 4 == 0, C <= 1024, blocks >= 1");
    return [=](hipStream_t s) { return unet::f32_colsum_launch(x, rows, c, nb, pa, out, s); };
  }
  if (kind == "f32_transpose") {
    // ptrs: src [T][A][B], dst [T][B][A] (tap order reversed if flip)   ints: T, A, B, flip
    need(2, 4, 0);
    const float* src = fp(0);
    float* dst = fp(1);
    int t = I[0], a = I[1], b = I[2], fl = I[3];
    return [=](hipStream_t s) { return unet::f32_transpose_launch(src, t, a, b, fl, dst, s); };
  }
  throw std::invalid_argument("unknown generic op '" + kind + "'");
}

int head_blocks_py(int P) { return head_blocks(P); }

thread_local bool g_dry = false;

// sets dry dispatch for the current thread while alive (Plan::check_dispatch)
struct DryScope {
  DryScope() { g_dry = true; }
  ~DryScope() { g_dry = false; }
};

class Plan {
 public:
  explicit Plan(int dtype = 0) : A_(api(dtype)) {}
  int add_conv_fwd(const py::dict& d) {
    ConvFwdParams p = conv_params(d);
    const bool seeded = p.drop_rate > 0.f || p.nd_rate > 0.f || p.xd_rate > 0.f;
    const uint32_t* seedp = &seed_;
    const uint32_t* const* seed_devp = &seed_dev_;
    const KernelApi* A = A_;
    ops_.push_back([p, seeded, seedp, seed_devp, A](hipStream_t s) mutable {
      if (seeded) {
        p.seed = *seedp;
        p.seed_ptr = *seed_devp;
      }
      return A->conv_fwd_launch(p, s);
    });
    names_.push_back(get<std::string>(d, "name", "conv_fwd"));
    return (int)ops_.size() - 1;
  }
  int add_wgrad(const py::dict& d) {
    WgradParams p = wgrad_params(d);
    const KernelApi* A = A_;
    ops_.push_back([p, A](hipStream_t s) { return A->wgrad_launch(p, s); });
    names_.push_back(get<std::string>(d, "name", "wgrad"));
    return (int)ops_.size() - 1;
  }
  int add_f32_conv(const py::dict& d) {
    F32Conv p = f32_conv_params(d);
    const bool seeded = p.drop_rate > 0.f;
    const uint32_t* seedp = &seed_;
    const uint32_t* const* seed_devp = &seed_dev_;
    ops_.push_back([p, seeded, seedp, seed_devp](hipStream_t s) mutable {
      if (seeded) {
        p.seed = *seedp;
        p.seed_ptr = *seed_devp;
      }
      return unet::f32_conv_launch(p, s);
    });
    names_.push_back(get<std::string>(d, "name", "f32_conv"));
    return (int)ops_.size() - 1;
  }
  int add_f32_wgrad(const py::dict& d) {
    F32Wgrad p = f32_wgrad_params(d);
    ops_.push_back([p](hipStream_t s) { return unet::f32_wgrad_launch(p, s); });
    names_.push_back(get<std::string>(d, "name", "f32_wgrad"));
    return (int)ops_.size() - 1;
  }
  int add_generic(const std::string& kind, const std::vector<uintptr_t>& P, const std::vector<long long>& I,
                  const std::vector<double>& F, const std::string& name) {
    ops_.push_back(make_generic(A_, kind, P, I, F, &seed_, &seed_dev_));
    names_.push_back(name.empty() ? kind : name);
    return (int)ops_.size() - 1;
  }
  // Dry dispatch of ops [begin, end) (conv_params.h dry_dispatch): every launcher resolves
  // its kernel instantiation and returns its status without launching -- no GPU needed.
  // Returns (op index, name, error) of every op whose launcher has no kernel for its
  // parameters (e.g. a combination conv_fwd_prepare accepts that launch_win never built).
  std::vector<std::tuple<int, std::string, std::string>> check_dispatch(int begin, int end) {
    if (begin < 0 || end > (int)ops_.size() || begin > end) throw std::out_of_range("Plan.check_dispatch: bad range");
    std::vector<std::tuple<int, std::string, std::string>> bad;
    DryScope dry;
    for (int i = begin; i < end; ++i) {
      hipError_t e = ops_[i](nullptr);
      if (e != hipSuccess) bad.emplace_back(i, names_[i], hipGetErrorName(e));
    }
    return bad;
  }
  void set_seed(uint32_t s) { seed_ = s; }
  // device address of a uint32 seed: dropout kernels read it at run time (graph mode)
  void set_seed_ptr(uintptr_t p) { seed_dev_ = reinterpret_cast<const uint32_t*>(p); }
  int size() const { return (int)ops_.size(); }
  std::vector<std::string> names() const { return names_; }
  void run(int begin, int end, uintptr_t stream) {
    if (begin < 0 || end > (int)ops_.size() || begin > end) throw std::out_of_range("Plan.run: bad range");
    hipStream_t s = as_stream(stream);
    for (int i = begin; i < end; ++i) {
      hipError_t e = ops_[i](s);
      if (e != hipSuccess)
        throw std::runtime_error("Plan op " + std::to_string(i) + " (" + names_[i] + "): " + hipGetErrorString(e));
    }
  }

 private:
  const KernelApi* A_;
  std::vector<Launcher> ops_;
  std::vector<std::string> names_;
  uint32_t seed_ = 0;
  const uint32_t* seed_dev_ = nullptr;
};

}  // namespace

namespace unet_types {
bool dry_dispatch() { return g_dry; }
}  // namespace unet_types

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) HIP kernels and launch-plan executor for the UNet trainer";
  // dtype: 0 = bf16 activations / weight copies, 1 = fp16
  m.def("conv_fwd", [](const py::dict& d, uintptr_t stream, int dtype) {
    ConvFwdParams p = conv_params(d);
    check(api(dtype)->conv_fwd_launch(p, as_stream(stream)), "conv_fwd");
  }, py::arg("params"), py::arg("stream"), py::arg("dtype") = 0);
  // workgroups of a row-window conv launch (0 for other kernels): sizes per-block
  // partial buffers of fused epilogues (the fused head); raises if the dict is invalid
  m.def("conv_fwd_grid", [](const py::dict& d) { return unet::conv_fwd_grid(conv_params(d)); }, py::arg("params"));
  // kernel / tile id a conv launch dispatches to (conv_fwd.hip conv_fwd_pick; tests)
  m.def("conv_fwd_pick", [](const py::dict& d) { return unet::conv_fwd_pick(conv_params(d)); }, py::arg("params"));
  // (rows, pixels per tile) of the per-tile statistics the conv's epilogue writes
  // (rows 0: no statistics epilogue for this shape -> separate moments pass)
  m.def("conv_stat_tiles", [](const py::dict& d) {
    int rows = 0, px = 0;
    unet::conv_stat_tiles(conv_params(d), &rows, &px);
    return py::make_tuple(rows, px);
  }, py::arg("params"));
  // validates a weight-gradient dict before its slabs exist (planning): raises like "wgrad"
  m.def("wgrad_validate", [](const py::dict& d0) {
    py::dict d = d0.attr("copy")();           // (a new dict: the caller's is left as is)
    if (!d.contains("slab") || d["slab"].is_none()) d["slab"] = py::int_(256);
    if (!d.contains("bias_slab") || d["bias_slab"].is_none()) d["bias_slab"] = py::int_(256);
    (void)wgrad_params(d);
  }, py::arg("params"));
  m.def("wgrad", [](const py::dict& d, uintptr_t stream, int dtype) {
    WgradParams p = wgrad_params(d);
    check(api(dtype)->wgrad_launch(p, as_stream(stream)), "wgrad");
  }, py::arg("params"), py::arg("stream"), py::arg("dtype") = 0);
  m.def("generic", [](const std::string& kind, const std::vector<uintptr_t>& P, const std::vector<long long>& I,
                      const std::vector<double>& F, uintptr_t stream, int dtype) {
    check(make_generic(api(dtype), kind, P, I, F)(as_stream(stream)), kind.c_str());
  }, py::arg("kind"), py::arg("ptrs"), py::arg("ints"), py::arg("floats"), py::arg("stream"), py::arg("dtype") = 0);
  m.def("adam_pack", [](uintptr_t w, uintptr_t g, uintptr_t mm, uintptr_t v, int n_total, uintptr_t segs, int nseg,
                        double lr_t, double b1, double b2, double eps, double gscale, int do_adam, uintptr_t arena,
                        uintptr_t stream, uintptr_t scalars, int dtype) {
    // scalars: optional device float[2] = {lr_t, gscale} read by the kernel (HIP-graph replay)
    check_msg(adam_check(nseg));
    check(api(dtype)->adam_pack_launch((float*)w, (const float*)g, (float*)mm, (float*)v, n_total, (const void*)segs, nseg,
                           (float)lr_t, (float)b1, (float)b2, (float)eps, (float)gscale, do_adam,
                           (const float*)scalars, (void*)arena, as_stream(stream)),
          "adam_pack");
  }, py::arg("w"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("n_total"), py::arg("segs"), py::arg("nseg"),
     py::arg("lr_t"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("gscale"), py::arg("do_adam"),
     py::arg("arena"), py::arg("stream"), py::arg("scalars") = 0, py::arg("dtype") = 0);
  m.def("f32_conv", [](const py::dict& d, uintptr_t stream) {
    F32Conv p = f32_conv_params(d);
    check(unet::f32_conv_launch(p, as_stream(stream)), "f32_conv");
  }, py::arg("params"), py::arg("stream") = 0);
  m.def("f32_wgrad", [](const py::dict& d, uintptr_t stream) {
    F32Wgrad p = f32_wgrad_params(d);
    check(unet::f32_wgrad_launch(p, as_stream(stream)), "f32_wgrad");
  }, py::arg("params"), py::arg("stream") = 0);
  m.def("f32_head_blocks", &unet::f32_head_blocks);
  m.def("f32_wgrad_tile", [](int M1, int M2, int Nc) {
    int bm, bn;
    unet::f32_wgrad_tile(M1, M2, Nc, &bm, &bn);
    return py::make_tuple(bm, bn);
  });
  m.def("head_blocks", &head_blocks_py);
  m.def("norm_blocks_per_sample", &norm_blocks_per_sample);
  m.def("sample_slices", &sample_slices);
  m.def("row_slices", &row_slices);
  m.def("hn_blocks_per_sample", &hn_blocks_per_sample);
  m.def("hn_partial_floats", &hn_partial_floats);
  m.def("wgrad_reduce_stage_floats", &wgrad_reduce_stage_floats);
  // QW > 0 describes a 3x3 (KT 9) or 3x3x3 (KT 27) stride-1 'same' conv on a QD x QH x QW
  // grid (QH, QD default to QW: square / cubic levels), a row-window candidate
  m.def(
      "wgrad_pick",
      [](int M1, int M2, int Nc, int KT, int QW, int upA, int win, int QH, int QD, int xform) {
        WgradParams p{};
        p.xform = xform;
        p.M1 = M1;
        p.M2 = M2;
        p.Nc = Nc;
        p.KD = 1;
        p.KH = 1;
        p.KW = KT;
        p.upA = upA;
        p.win = win;
        p.bias_mode = 1;
        if (QH <= 0) QH = QW;
        if (QW > 0 && (KT == 9 || KT == 27)) {   // 3x3 (x3) stride-1 'same' conv
          p.KH = p.KW = 3;
          p.KD = KT == 27 ? 3 : 1;
          p.QD = p.AD = KT == 27 ? (QD > 0 ? QD : QW) : 1;
          p.QW = p.AW = QW;
          p.QH = p.AH = QH;
          p.stride = 1;
          p.pad = 1;
        } else if (QW > 0 && KT == 4) {   // 2x2 stride-2 transposed conv (QW = coarse width)
          p.KH = p.KW = 2;
          p.QD = p.AD = 1;
          p.QW = p.QH = QW;
          p.AW = p.AH = 2 * QW;
          p.stride = 2;
          p.pad = 0;
          p.bias_mode = 2;
        } else if (QW > 0 && KT == 16) {  // composite tconv slab: 4x4 taps, stride 2, pad 1
          p.KH = p.KW = 4;
          p.QD = p.AD = 1;
          p.QW = p.QH = QW;
          p.AW = p.AH = 2 * QW;
          p.stride = 2;
          p.pad = 1;
          p.bias_mode = 2;
        }
        WgradCfg c = wgrad_pick(p);
        return py::make_tuple(c.BM, c.BN, c.NTAP, c.smallc);
      },
      py::arg("M1"), py::arg("M2"), py::arg("Nc"), py::arg("KT"), py::arg("QW") = 0, py::arg("upA") = 1,
      py::arg("win") = -1, py::arg("QH") = 0, py::arg("QD") = 0, py::arg("xform") = 0);
  m.def("packseg_bytes", []() { return (int)sizeof(PackSeg); });
  m.def("reduce_job_bytes", []() { return (int)sizeof(ReduceJob); });
  m.def("reduce_groups", &reduce_groups);
  m.def("crc32c", [](py::buffer b, uint32_t crc) {
    py::buffer_info info = b.request();
    const size_t n = (size_t)info.size * (size_t)info.itemsize;
    uint32_t r;
    {
      py::gil_scoped_release rel;
      r = crc32c_extend(crc, (const uint8_t*)info.ptr, n);
    }
    return r;
  }, py::arg("data"), py::arg("crc") = 0u);
  m.def("gather_rows", [](uintptr_t src, uintptr_t idx, int64_t n, int64_t row_bytes, uintptr_t dst, int threads) {
    py::gil_scoped_release rel;
    gather_rows((const uint8_t*)src, (const int64_t*)idx, n, row_bytes, (uint8_t*)dst, threads);
  });
  m.def("device_sync", []() { check(hipDeviceSynchronize(), "hipDeviceSynchronize"); });
  py::class_<Plan>(m, "Plan")
      .def(py::init<int>(), py::arg("dtype") = 0)
      .def("add_conv_fwd", &Plan::add_conv_fwd)
      .def("add_wgrad", &Plan::add_wgrad)
      .def("add_f32_conv", &Plan::add_f32_conv)
      .def("add_f32_wgrad", &Plan::add_f32_wgrad)
      .def("add_generic", &Plan::add_generic, py::arg("kind"), py::arg("ptrs"), py::arg("ints"),
           py::arg("floats"), py::arg("name") = "")
      .def("check_dispatch", &Plan::check_dispatch)
      .def("set_seed", &Plan::set_seed)
      .def("set_seed_ptr", &Plan::set_seed_ptr)
      .def("size", &Plan::size)
      .def("names", &Plan::names)
      .def("run", &Plan::run, py::call_guard<py::gil_scoped_release>());
}
