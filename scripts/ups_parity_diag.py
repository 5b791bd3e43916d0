"""Why does the 1-channel upsampling-decoder step sit further from the fp32 oracle than the
other configs (total gradient cosine distance 0.0062 vs ~1.5e-4)?  Compare, per
batch size, the native bf16 step and ATen's own bf16 (autocast) step against the exact
fp32 step on the CPU; and the native fp32 executor as a control.  Prints one JSON line per
(config, path)."""
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from unet_distributed_amd.config import Config  # noqa: E402
from unet_distributed_amd.data.datasets import synthetic_brats  # noqa: E402
from unet_distributed_amd.models import reference  # noqa: E402
from unet_distributed_amd.models.spec import spec_from_config  # noqa: E402
from unet_distributed_amd.runtime.backends import NativeBackend, TorchBackend  # noqa: E402
from unet_distributed_amd.runtime.params import FlatParams  # noqa: E402

dev = torch.device("cuda:0")


def cosd(a, b):
    a, b = a.double().reshape(-1), b.double().reshape(-1)
    return 1.0 - (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def run(kw, seed=77):
    cfg = Config(**kw)
    spec = spec_from_config(cfg)
    B = cfg.batch_size
    x, y = synthetic_brats(B, cfg.img_size, cfg.in_channels, cfg.dims, seed=5)
    init = reference.init_params(spec, seed=3)
    ref = FlatParams(spec)
    ref.load_dict(init)
    tb = TorchBackend(spec, ref, Config(**dict(kw, dtype="fp32")), "cpu", B)
    tb.fwd_bwd(torch.from_numpy(x), torch.from_numpy(y), seed=seed)
    out = []
    for path, dt, backend in (("native bf16", "bf16", "native"), ("ATen bf16 (GPU)", "bf16", "torch"),
                              ("native fp32", "fp32", "native")):
        f = FlatParams(spec, device=dev)
        f.load_dict(init)
        c = Config(**dict(kw, dtype=dt, backend=backend))
        be = NativeBackend(spec, f, c, dev, B) if backend == "native" else TorchBackend(spec, f, c, dev, B)
        be.fwd_bwd(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev), seed=seed)
        torch.cuda.synchronize()
        g = f.grad.cpu()
        worst = max(((cosd(g[o:o + n], ref.grad[o:o + n]), name) for name, _, o, n in f.entries
                     if ref.grad[o:o + n].norm() > 0), key=lambda t: t[0])
        ratio = max(((abs(g[o:o + n].norm().item() / ref.grad[o:o + n].norm().item() - 1), name)
                     for name, _, o, n in f.entries if ref.grad[o:o + n].norm() > 0), key=lambda t: t[0])
        out.append(dict(config=kw, path=path, total_cos_dist=cosd(g, ref.grad), worst_cos=worst, worst_ratio=ratio,
                        sums=[round(v, 3) for v in be.sums().tolist()], ref_sums=[round(v, 3) for v in tb.sums().tolist()]))
        print(json.dumps(out[-1]), flush=True)
    return out


if __name__ == "__main__":
    for kw in (dict(batch_size=2, img_size=64, in_channels=1, use_upsampling=True),
               dict(batch_size=8, img_size=64, in_channels=1, use_upsampling=True),
               dict(batch_size=2, img_size=64, in_channels=1),
               dict(batch_size=2, img_size=64, in_channels=4)):
        run(kw)
