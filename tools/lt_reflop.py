"""Recompute the TFLOP/s column of a tools/layer_times.py table in place with the
current FLOP attribution (layer_flops), taking the launch names from the table itself
and the planner's fusions from a dry-run engine of the table's configuration.

    python tools/lt_reflop.py profiles/r6_layer_times*.md
"""
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from layer_times import layer_flops  # noqa: E402
from unet_distributed_amd.config import Config  # noqa: E402
from unet_distributed_amd.models.spec import spec_from_config  # noqa: E402
from unet_distributed_amd.runtime.native_engine import NativeUNet  # noqa: E402
from unet_distributed_amd.runtime.params import FlatParams  # noqa: E402

HDR = re.compile(r"(\d)D UNet (\d+)x\d+ in_ch=(\d+), batch (\d+), norm (\w+), (\w+)")
ROW = re.compile(r"\| (\d+) \| `(\S+)` \| ([\d.]+) \| ([\d.]*) \|")


def reflop(path):
    lines = open(path).read().split("\n")
    m = next(HDR.search(l) for l in lines if HDR.search(l))
    dims, img, cin, B, norm, dt = int(m[1]), int(m[2]), int(m[3]), int(m[4]), m[5], m[6]
    cfg = Config(batch_size=B, img_size=img, in_channels=cin, dims=dims, norm=norm, dtype=dt)
    spec = spec_from_config(cfg)
    e = NativeUNet(spec, FlatParams(spec), B, img, "cpu", dry_run=True, dtype=dt)
    names = [r[2] for r in (ROW.match(l) for l in lines) if r]
    fl = layer_flops(spec, B, img, dims, e, names)
    out = []
    for l in lines:
        r = ROW.match(l)
        if r:
            f = fl.get(r[2])
            l = "| %s | `%s` | %s | %s |" % (r[1], r[2], r[3], "%.0f" % (f / float(r[3]) / 1e9) if f else "")
        out.append(l)
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    for p in sys.argv[1:]:
        reflop(p)
        print("rewrote", p)
