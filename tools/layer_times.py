"""Per-launch timing of the native training step (one HIP event pair per plan
entry, each entry replayed ``--reps`` times in isolation) with achieved
TFLOP/s for the conv / wgrad GEMMs.  Usage on the GPU box:

    PYTHONPATH=. python tools/layer_times.py --batch 256 --img 128 --out profiles/layer_times.md
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from unet_distributed_amd.config import Config  # noqa: E402
from unet_distributed_amd.data.datasets import synthetic_brats  # noqa: E402
from unet_distributed_amd.models import reference  # noqa: E402
from unet_distributed_amd.models.spec import spec_from_config  # noqa: E402
from unet_distributed_amd.runtime.native_engine import NativeUNet  # noqa: E402
from unet_distributed_amd.runtime.params import FlatParams  # noqa: E402


def layer_flops(spec, B, img, dims, e=None, names=()):
    """GEMM FLOPs per plan-entry name (fwd:, dgrad:, dgrad_skip:, wgrad:), attributed to
    the launch that does them: a concat conv's data gradient split into its u and skip
    halves, the u-row weight gradient chained into the transposed conv's composite
    weight gradient (tconv_wa), data + weight gradient in one fused launch (dw_fused), and
    a layer's work split over several launches of one name (halves) divided among them."""
    out = {}
    tcon = {}                                   # concat conv -> its transposed conv
    for l in spec.layers:
        if l.kind == "tconv":
            for c in spec.layers:
                if c.kind == "conv" and c.skip_from is not None and c.level == l.level:
                    tcon[c.name] = l
    wa = getattr(e, "_wa_chain_of", {}) if e is not None else {}
    fused = set(getattr(e, "fusions", {}).get("dw_fused", ())) if e is not None else set()
    for l in spec.layers:
        s = img >> (l.level - 1)
        pix = B * s ** dims
        if l.kind == "conv":
            f = 2.0 * pix * l.cout * l.cin * 3 ** dims
            out["fwd:" + l.name] = f
            cs = l.cin - tcon[l.name].cout if l.name in tcon else 0       # skip channels
            fw = f * cs / l.cin if l.name in wa else f
            if l.name in wa:
                out["wgrad:" + wa[l.name]] = out.get("wgrad:" + wa[l.name], 0.0) + f - fw
            fd = 0.0
            if l.level > 1 or l.skip_from is not None or l.cin > 8:
                fd = f
                if "dgrad_skip:" + l.name in names:
                    fd = f * (l.cin - cs) / l.cin
                    out["dgrad_skip:" + l.name] = f * cs / l.cin
            if l.name in fused and "wgrad:" + l.name not in names:
                fd += fw
            else:
                out["wgrad:" + l.name] = fw
            if fd:
                out["dgrad:" + l.name] = fd
        elif l.kind == "tconv":
            s2 = img >> l.level
            f = 2.0 * B * s2 ** dims * l.cin * l.cout * 2 ** dims
            out["fwd:" + l.name] = f
            out["wgrad:" + l.name] = out.get("wgrad:" + l.name, 0.0) + f
            out["dgrad:" + l.name] = f
    for n in set(names):
        k = list(names).count(n)
        if k > 1 and n in out:
            out[n] /= k
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=128)
    ap.add_argument("--in_channels", type=int, default=4)
    ap.add_argument("--dims", type=int, default=2)
    ap.add_argument("--upsampling", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--norm", default="none", choices=["none", "batch", "group"])
    ap.add_argument("--groups", type=int, default=8)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp16"])
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = Config(batch_size=a.batch, img_size=a.img, in_channels=a.in_channels, dims=a.dims,
                 use_upsampling=a.upsampling, norm=a.norm, groups=a.groups, dtype=a.dtype)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=1))
    e = NativeUNet(spec, flat, a.batch, a.img, dev, dtype=a.dtype)
    x, y = synthetic_brats(min(a.batch, 64), a.img, a.in_channels, a.dims, seed=0)
    reps = (a.batch + 63) // 64
    x = torch.from_numpy(x).repeat((reps,) + (1,) * (x.ndim - 1))[:a.batch].to(dev)
    y = torch.from_numpy(y).repeat((reps,) + (1,) * (y.ndim - 1))[:a.batch].to(dev)
    e.load_batch(x, y)
    for _ in range(3):
        e.forward(1)
        e.backward()
    torch.cuda.synchronize()
    names = e.plan.names()
    fl = layer_flops(spec, a.batch, a.img, a.dims, e, names)
    s = torch.cuda.current_stream().cuda_stream
    rows = []
    total = 0.0
    for i, n in enumerate(names):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e.plan.run(i, i + 1, s)
        st.record()
        for _ in range(a.reps):
            e.plan.run(i, i + 1, s)
        en.record()
        torch.cuda.synchronize()
        ms = st.elapsed_time(en) / a.reps
        total += ms
        f = fl.get(n)
        rows.append((i, n, ms, f / ms / 1e9 if f else None))
    # whole step for comparison
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.reps):
        e.forward(1)
        e.backward()
    en.record()
    torch.cuda.synchronize()
    step = st.elapsed_time(en) / a.reps
    lines = ["# Per-launch times, native step, %dD UNet %dx%d in_ch=%d, batch %d, norm %s, %s (1x MI355X)" %
             (a.dims, a.img, a.img, a.in_channels, a.batch, a.norm, a.dtype), "",
             "sum of isolated launches %.3f ms; back-to-back step %.3f ms (%.0f img/s fwd+bwd only)"
             % (total, step, a.batch / step * 1e3), "",
             "| # | launch | ms | TFLOP/s |", "|---|---|---|---|"]
    for i, n, ms, tf in rows:
        lines.append("| %d | `%s` | %.4f | %s |" % (i, n, ms, "%.0f" % tf if tf else ""))
    # per-kind rollup
    kinds = {}
    for _, n, ms, _ in rows:
        k = n.split(":")[0]
        kinds[k] = kinds.get(k, 0.0) + ms
    lines += ["", "| kind | ms | % |", "|---|---|---|"]
    for k, v in sorted(kinds.items(), key=lambda kv: -kv[1]):
        lines.append("| %s | %.3f | %.1f |" % (k, v, 100 * v / total))
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
