"""GEMM FLOPs per image of one training step (forward + data + weight gradients) of a UNet
config, for the TF/s column of the config tables (profiles/r5_configs.md).  The first
layer has no data gradient; the Mask head and elementwise work are not counted."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from unet_distributed_amd.models.spec import UNetSpec  # noqa: E402


def step_flops_per_image(img=128, in_channels=4, dims=2, use_upsampling=False, norm="none"):
    spec = UNetSpec(in_channels=in_channels, dims=dims, use_upsampling=use_upsampling, norm=norm)
    total = 0.0
    for l in spec.layers:
        if l.kind == "conv":
            pix = (img >> (l.level - 1)) ** dims
            f = 2.0 * pix * l.cin * l.cout * 3 ** dims
            total += f * (2 if l.name == spec.layers[0].name else 3)
        elif l.kind == "tconv":
            pix = (img >> l.level) ** dims
            total += 3 * 2.0 * pix * l.cin * l.cout * 2 ** dims
    return total


if __name__ == "__main__":
    print("%.3f GFLOP/img" % (step_flops_per_image() / 1e9))
