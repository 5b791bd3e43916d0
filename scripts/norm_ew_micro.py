"""Bandwidth of the BatchNorm / GroupNorm streaming passes (norm_bwd_apply: dz = a g + b z + c,
norm_apply: y = relu(A z + B)) at the bench's level shapes (batch 1024, 128x128 2D UNet), against
a torch bf16 elementwise op that moves the same bytes.  Grid width from UNET_NORM_EW_BPS (one
setting per process).  Prints one JSON line per (op, shape)."""
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from unet_distributed_amd import native  # noqa: E402

dev = torch.device("cuda:0")
C = native.require()


def ptr(t):
    return int(t.data_ptr())


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    bps = os.environ.get("UNET_NORM_EW_BPS", "default")
    N = 1024
    st = int(torch.cuda.current_stream().cuda_stream)
    for P, Cc in ((16384, 32), (4096, 64), (1024, 128)):
        g = torch.randn(N, P, Cc, device=dev).bfloat16()
        z = torch.randn(N, P, Cc, device=dev).bfloat16()
        dz = torch.empty_like(z)
        ca, cb, cc = [torch.randn(Cc, device=dev) for _ in range(3)]
        gam, bet = torch.rand(Cc, device=dev) + 0.5, torch.randn(Cc, device=dev)
        mean, rstd = torch.randn(Cc, device=dev), torch.rand(Cc, device=dev) + 0.5
        gb = g.numel() * 2 / 1e9

        t_bwd = timeit(lambda: C.generic("norm_bwd_apply", [ptr(g), ptr(z), ptr(ca), ptr(cb), ptr(cc), ptr(dz)],
                                         [N, P, Cc, 0], [], st))
        t_app = timeit(lambda: C.generic("norm_apply", [ptr(z), ptr(mean), ptr(rstd), ptr(gam), ptr(bet), ptr(dz)],
                                         [N, P, Cc, 0, 1, 0, 0], [0.0], st))
        t_tadd = timeit(lambda: torch.add(g, z, out=dz))
        t_tcopy = timeit(lambda: dz.copy_(z))
        # correctness of the pass at this grid
        C.generic("norm_bwd_apply", [ptr(g), ptr(z), ptr(ca), ptr(cb), ptr(cc), ptr(dz)], [N, P, Cc, 0], [], st)
        ref = (ca * g[:8].float() + cb * z[:8].float() + cc)
        err = ((dz[:8].float() - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps(dict(bps=bps, P=P, C=Cc, err=err,
                              norm_bwd_apply=dict(ms=round(t_bwd, 4), TBs=round(3 * gb / t_bwd, 2)),
                              norm_apply=dict(ms=round(t_app, 4), TBs=round(2 * gb / t_app, 2)),
                              torch_add=dict(ms=round(t_tadd, 4), TBs=round(3 * gb / t_tadd, 2)),
                              torch_copy=dict(ms=round(t_tcopy, 4), TBs=round(2 * gb / t_tcopy, 2)))), flush=True)
        del g, z, dz
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
