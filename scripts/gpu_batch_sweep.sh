#!/bin/bash
# Per-GPU micro-batch sweep of the headline bench (128x128x4 bf16): 64 .. 2048, plus the
# device memory each needs (torch.cuda.max_memory_allocated from a 1-step probe).
# Writes gpurun_out/batch_sweep.md.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bsweep
for b in 64 128 256 512 1024 2048; do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 --per_gpu_batch $b > gpurun_out/bsweep/b$b.log 2>&1 || { tail -5 gpurun_out/bsweep/b$b.log; exit 1; }
done
timeout -k 10 240 python - <<'PY' > gpurun_out/bsweep/mem.txt || exit 1
import torch, sys
sys.path.insert(0, ".")
from unet_distributed_amd.config import Config
from unet_distributed_amd.models import reference
from unet_distributed_amd.models.spec import spec_from_config
from unet_distributed_amd.runtime.backends import NativeBackend
from unet_distributed_amd.runtime.params import FlatParams
from unet_distributed_amd.data.datasets import synthetic_brats
dev = torch.device("cuda:0")
for b in (64, 128, 256, 512, 1024, 2048):
    torch.cuda.empty_cache(); torch.cuda.reset_peak_memory_stats()
    cfg = Config(batch_size=b, in_channels=4, img_size=128)
    spec = spec_from_config(cfg)
    flat = FlatParams(spec, device=dev); flat.load_dict(reference.init_params(spec, seed=1))
    be = NativeBackend(spec, flat, cfg, dev, b)
    be.engine.repack()
    x, y = synthetic_brats(b, 128, 4, seed=1)
    be.fwd_bwd(torch.from_numpy(x).to(dev), torch.from_numpy(y).to(dev), seed=1)
    torch.cuda.synchronize()
    print(b, torch.cuda.max_memory_allocated() / 2**30)
    del be, flat
PY
python - <<'PY'
import json
mem = dict(l.split() for l in open("gpurun_out/bsweep/mem.txt"))
out = ["# Per-GPU micro-batch sweep, bench.py 2D UNet 128x128x4 bf16 (1x MI355X)", "",
       "| per-GPU batch | images/sec | ms/step | peak device memory (GiB) |", "|---|---|---|---|"]
for b in (64, 128, 256, 512, 1024, 2048):
    r = [json.loads(l) for l in open("gpurun_out/bsweep/b%d.log" % b) if l.startswith("{")][0]
    out.append("| %d | %.0f | %.3f | %.1f |" % (b, r["value"], r["ms_per_step"], float(mem[str(b)])))
open("gpurun_out/batch_sweep.md", "w").write("\n".join(out) + "\n")
print("\n".join(out))
PY
