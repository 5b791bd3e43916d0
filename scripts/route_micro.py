"""Isolated timings of the skip-half data gradient with and without the fused pool
backward in its epilogue (conv_epilogue.h route_gy) at the benched shapes: 2D level 1
(128 wide, 32 -> 32, per-GPU batch 1024: the persistent prefetching window), 2D level 2
(64 wide, 64 -> 64: the chunk-pipelined window) and 3D level 1 (128^3, 32 -> 32, batch 8:
the 128-wide chunk-pipelined window).  Usage on the GPU box: python scripts/route_micro.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unet_distributed_amd import native  # noqa: E402


def ptr(t):
    return int(t.data_ptr())


def shape_variants(N, D, H, W, C, cp):
    dev = torch.device("cuda")
    bf = torch.bfloat16
    P = N * D * H * W
    kd = 3 if D > 1 else 1
    kpad = -(-(kd * 9 * C) // 64) * 64
    keep = []

    def t(x):
        keep.append(x)
        return ptr(x)
    g = t(torch.randn(P, C, device=dev).to(bf))
    out = t(torch.empty(P, C, device=dev, dtype=bf))
    wp = t(torch.randn(C, kpad, device=dev).to(bf))
    bits = t(torch.randint(0, 255, (P * C // 8,), device=dev, dtype=torch.uint8))
    pg = t(torch.randn(P // (8 if D > 1 else 4), C, device=dev).to(bf))
    code = t(torch.randint(0, 2 ** 31 - 1, (P // (8 if D > 1 else 4) * C // 8,), device=dev, dtype=torch.int32))
    base = dict(N=N, OD=D, OH=H, OW=W, ID=D, IH=H, IW=W, KD=kd, KH=3, KW=3, stride=1, pad=1, tile=0, win_pf=8,
                win_cp=cp, C1=C, src1=g, wgt=wp, Cout=C, relu=0, dst1=out, D1=C)
    v = {"no mask": dict(base), "mask bits": dict(base, mask1=bits, mask_bits=1),
         "mask bits + pool route": dict(base, mask1=bits, mask_bits=1, route_gy=pg, pool_code=code)}
    return v, keep


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    C = native.require()
    s = int(torch.cuda.current_stream().cuda_stream)
    print("| shape | variant | ms |\n|---|---|---|")
    for label, shp in (("2D L1 b1024 128^2 32ch", (1024, 1, 128, 128, 32, 1)),
                       ("2D L2 b1024 64^2 64ch", (1024, 1, 64, 64, 64, 1)),
                       ("3D L1 b8 128^3 32ch", (8, 128, 128, 128, 32, 2))):
        variants, keep = shape_variants(*shp)
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
            print("| %s | %s | %.4f |" % (label, name, e0.elapsed_time(e1) / reps), flush=True)
        del keep
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
