"""Per-layer gradient cosine: native bf16 vs fp32, and ATen bf16-autocast vs fp32 (noise floor)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unet_distributed_amd.config import Config
from unet_distributed_amd.data.datasets import synthetic_brats
from unet_distributed_amd.models import reference
from unet_distributed_amd.models.spec import spec_from_config
from unet_distributed_amd.runtime.backends import NativeBackend, TorchBackend
from unet_distributed_amd.runtime.params import FlatParams
dev = torch.device("cuda")
norm = sys.argv[1] if len(sys.argv) > 1 else "batch"
kw = dict(batch_size=4, img_size=64, in_channels=4, norm=norm, groups=8)
cfg = Config(**kw)
spec = spec_from_config(cfg)
x, y = synthetic_brats(4, 64, 4, 2, seed=5)
x, y = torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev)
init = reference.init_params(spec, seed=3)
def run(kind, dtype):
    f = FlatParams(spec, device=dev); f.load_dict(init)
    c = Config(**dict(kw, dtype=dtype))
    be = NativeBackend(spec, f, c, dev, 4) if kind == "native" else TorchBackend(spec, f, c, dev, 4)
    be.fwd_bwd(x, y, seed=77)
    torch.cuda.synchronize()
    return f
f32, fb, fn = run("torch", "fp32"), run("torch", "bf16"), run("native", "bf16")
fh = run("native", "fp16")
cos = lambda a, b: (a.double() @ b.double() / (a.double().norm() * b.double().norm() + 1e-30)).item()
for name, shape, off, n in f32.entries:
    g0 = f32.grad[off:off + n]
    if g0.norm() < 1e-6:
        continue
    print("%-28s native-bf16 %.4f  aten-bf16 %.4f  native-fp16 %.4f" % (
        name, cos(fn.grad[off:off + n], g0), cos(fb.grad[off:off + n], g0), cos(fh.grad[off:off + n], g0)))
