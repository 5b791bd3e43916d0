"""Alias of train.py under the reference's entry-point name (`test_dist.py`).

The reference's ``--ip`` role selection is accepted and ignored: ranks come
from the torch.distributed environment (RANK / WORLD_SIZE / MASTER_ADDR).
"""
import sys

from unet_distributed_amd.runtime.trainer import main

if __name__ == "__main__":
    sys.exit(main())
