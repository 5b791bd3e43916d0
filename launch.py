"""One process per GPU launcher (see unet_distributed_amd/launch.py).

    python launch.py --nproc_per_node 8 train.py --epochs 10 --batch_size 1024
    python launch.py --hostfile inv.yml --nproc_per_node 8 train.py ...
"""
import sys

from unet_distributed_amd.launch import main

if __name__ == "__main__":
    sys.exit(main())
