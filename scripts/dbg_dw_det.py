"""Debug: run-to-run determinism of the native step with the fused data + weight gradient,
and which gradients differ between two option sets."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from test_gpu_model import _setup  # noqa: E402

dev = torch.device("cuda:0")


def run(engine, hip_graph=True):
    os.environ["UNET_ENGINE"] = engine
    spec, cfg, x, y, fn, nb, ft, tb = _setup(dev, batch_size=4, img_size=128, in_channels=4, loss="dice_bce",
                                             hip_graph=hip_graph)
    for seed in (77, 78):
        nb.fwd_bwd(x, y, seed=seed)
    torch.cuda.synchronize()
    return fn, fn.grad.clone()


for eng_a, eng_b in [("head_onload=1", "head_onload=1"), ("head_onload=0", "head_onload=1"),
                     ("head_onload=0,dw_fuse=0", "head_onload=1,dw_fuse=0"),
                     ("dw_fuse=0", "dw_fuse=1")]:
    fn, ga = run(eng_a)
    _, gb = run(eng_b)
    bad = [(name, (ga[off:off + n] - gb[off:off + n]).abs().max().item())
           for name, shape, off, n in fn.entries if not torch.equal(ga[off:off + n], gb[off:off + n])]
    print(eng_a, "vs", eng_b, "differ:", bad[:8], flush=True)
