"""Isolated timings of the level-1 row-window data-gradient launch (2D, 128 wide,
32 -> 32 channels, per-GPU batch 1024) under epilogue variants: which part of the
kernel (halo DMA + MFMAs vs mask / pool-route epilogue vs head-on-load fill) sets its
time.  Usage on the GPU box: python scripts/win_micro.py [N]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unet_distributed_amd import native  # noqa: E402


def ptr(t):
    return int(t.data_ptr())


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    H = 128
    C = native.require()
    dev = torch.device("cuda")
    s = int(torch.cuda.current_stream().cuda_stream)
    dz = torch.randn(N, H, H, 32, device=dev).bfloat16()
    w = torch.randn(32, 9 * 32, device=dev).bfloat16()
    out = torch.empty(N, H, H, 32, device=dev, dtype=torch.bfloat16)
    bits = torch.randint(0, 255, (N * H * H * 4,), device=dev, dtype=torch.uint8)
    act = torch.randn(N, H, H, 32, device=dev).bfloat16()
    pooled = torch.randn(N, H // 2, H // 2, 32, device=dev).bfloat16()
    codes = torch.randint(0, 2 ** 31 - 1, (N * (H // 2) ** 2 * 4,), device=dev, dtype=torch.int32)
    bias = torch.zeros(32, device=dev)
    base = dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=32, src1=ptr(dz), wgt=ptr(w), Cout=32,
                dst1=ptr(out))
    variants = {
        "dgrad no mask": dict(base),
        "dgrad mask bits": dict(base, mask1=ptr(bits), mask_bits=1),
        "dgrad mask 16-bit": dict(base, mask1=ptr(act)),
        "dgrad bits + pool route": dict(base, mask1=ptr(bits), mask_bits=1, route_gy=ptr(pooled),
                                        pool_code=ptr(codes)),
        "fwd bias relu": dict(base, bias=ptr(bias), relu=1),
        "fwd bias relu + bits": dict(base, bias=ptr(bias), relu=1, relu_bits=ptr(bits)),
    }
    gbytes = 2 * N * H * H * 32 * 2 / 1e9
    print("| variant | ms | TB/s (1 read + 1 write of a 32-ch tensor) |")
    print("|---|---|---|")
    for name, d in variants.items():
        for _ in range(3):
            C.conv_fwd(d, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            C.conv_fwd(d, s)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print("| %s | %.4f | %.2f |" % (name, ms, gbytes / ms))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
