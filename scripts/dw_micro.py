"""Isolated timings of the fused data + weight gradient (conv_dw.hip) at the benched
level-1 shape (2D, 128 wide, 32 -> 32 channels, per-GPU batch 1024) for each operand
source: plain dY (XF 0), norm backward on load (XF 2), the normalised head (XF 3) and
the norm-free head (XF 4).  Usage on the GPU box: python scripts/dw_micro.py [N] [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unet_distributed_amd import native  # noqa: E402


def ptr(t):
    return int(t.data_ptr())


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    H = W = 128
    P = N * H * W
    C = native.require()
    dev = torch.device("cuda")
    s = int(torch.cuda.current_stream().cuda_stream)
    bf = torch.bfloat16
    g = torch.randn(N, H, W, 32, device=dev).to(bf)
    z = torch.randn(N, H, W, 32, device=dev).to(bf)
    x = torch.randn(N, H, W, 32, device=dev).to(bf)
    zd = torch.randn(N, H, W, 32, device=dev).to(bf)
    out = torch.empty(N, H, W, 32, device=dev, dtype=bf)
    bits = torch.randint(0, 255, (P * 4,), device=dev, dtype=torch.uint8)
    prob = torch.rand(P, device=dev)
    t = (torch.rand(P, device=dev) > 0.5).to(bf)
    sums = torch.tensor([100.0, 200.0, 300.0, 0.0], device=dev)
    co = [torch.rand(32, device=dev) for _ in range(7)]
    wp = torch.randn(32, 9 * 32 + 32, device=dev).to(bf)
    slab = torch.zeros(512, 9, 32, 32, device=dev)
    bslab = torch.zeros(512, 32, device=dev)
    st = torch.zeros(N * H // 2, 2, 32, device=dev)
    base = dict(N=N, OH=H, OW=W, IH=H, IW=W, KH=3, KW=3, pad=1, C1=32, src1=ptr(g), wgt=ptr(wp), Cout=32, relu=0,
                dst1=ptr(out), fw_x=ptr(x), fw_slab=ptr(slab), fw_bias_slab=ptr(bslab), fw_Cx=32, fw_nsplit=512)
    norm = dict(nz=ptr(zd), na=ptr(co[0]), nc=ptr(co[1]), ncs=0, npix=H * W, stats=ptr(st))
    xf2 = dict(xform=2, xa=ptr(co[2]), xb=ptr(co[3]), xc=ptr(co[4]), xz=ptr(z), xcs=0)
    hg = dict(hg_prob=ptr(prob), hg_t=ptr(t), hg_sums=ptr(sums), hg_w=ptr(co[5]), hg_inv_total=1.0 / P)
    variants = {
        "XF0 dgrad bits": dict(base, mask1=ptr(bits), mask_bits=1),
        "XF0 dgrad-norm": dict(base, **norm),
        "XF2 dgrad-norm": dict(base, **norm, **xf2),
        "XF3 dgrad-norm": dict(base, **norm, **xf2, **hg, src1=ptr(z), hg_fa=ptr(co[5]), hg_fc=ptr(co[6])),
        "XF4 dgrad bits": dict(base, mask1=ptr(bits), mask_bits=1, **hg, hg_bits=ptr(bits)),
    }
    for name, d in variants.items():
        for _ in range(3):
            C.conv_fwd(d, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            C.conv_fwd(d, s)
        e1.record()
        torch.cuda.synchronize()
        print("| %s | %.4f |" % (name, e0.elapsed_time(e1) / reps))


if __name__ == "__main__":
    main()
