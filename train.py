"""Training entry point (flag-compatible with the reference's test_dist.py).

    python train.py --synthetic --in_channels 4 --batch_size 256 --epochs 1
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py --synthetic ...

See unet_distributed_amd/config.py for the flag list.
"""
import sys

from unet_distributed_amd.runtime.trainer import main

if __name__ == "__main__":
    sys.exit(main())
