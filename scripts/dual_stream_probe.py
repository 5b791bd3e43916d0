"""Probe: does running the weight-gradient launches (wgrad / bsum / reduce, which are
off the backward critical path) on a second stream, concurrently with the dgrad
chain, shorten the native backward on MI355X -- eagerly and under HIP-graph replay?

    python scripts/dual_stream_probe.py --batch 256 --img 128
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

SIDE = ("wgrad:", "bsum:", "reduce:")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=128)
    ap.add_argument("--in_channels", type=int, default=4)
    ap.add_argument("--dims", type=int, default=2)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    cfg = Config(batch_size=a.batch, img_size=a.img, in_channels=a.in_channels, dims=a.dims)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev)
    flat.load_dict(reference.init_params(spec, seed=1))
    e = NativeUNet(spec, flat, a.batch, a.img, dev)
    x, y = synthetic_brats(a.batch, a.img, a.in_channels, a.dims, seed=0)
    e.load_batch(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev))
    e.forward(1)
    torch.cuda.synchronize()
    names = e.plan.names()
    b0, b1 = e.fwd_end, e.plan.size()
    main_s = torch.cuda.current_stream()
    side_s = torch.cuda.Stream()

    def single(s):
        e.plan.run(b0, b1, s.cuda_stream)

    def dual(ms, ss):
        i = b0
        while i < b1:
            j = i
            on_side = names[i].startswith(SIDE)
            while j < b1 and names[j].startswith(SIDE) == on_side:
                j += 1
            if on_side:
                ss.wait_stream(ms)
                e.plan.run(i, j, ss.cuda_stream)
            else:
                e.plan.run(i, j, ms.cuda_stream)
            i = j
        ms.wait_stream(ss)

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(a.reps):
            fn()
        en.record()
        torch.cuda.synchronize()
        return st.elapsed_time(en) / a.reps

    ref = flat.grad.clone()
    single(main_s)
    torch.cuda.synchronize()
    ref.copy_(flat.grad)
    t_single = timeit(lambda: single(main_s))
    t_dual = timeit(lambda: dual(main_s, side_s))
    torch.cuda.synchronize()
    same_eager = torch.equal(ref, flat.grad)

    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        single(torch.cuda.current_stream())
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        cs = torch.cuda.current_stream()
        side2 = torch.cuda.Stream()
        side2.wait_stream(cs)
        dual(cs, side2)
    t_g1 = timeit(g1.replay)
    t_g2 = timeit(g2.replay)
    torch.cuda.synchronize()
    same_graph = torch.equal(ref, flat.grad)
    print("backward eager: single %.3f ms, dual %.3f ms (grads identical %s)" % (t_single, t_dual, same_eager))
    print("backward graph: single %.3f ms, dual %.3f ms (grads identical %s)" % (t_g1, t_g2, same_graph))


if __name__ == "__main__":
    main()
