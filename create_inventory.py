"""Write inv.yml from settings.WORKER_HOSTS (`create_inventory.py` of the reference)."""
import sys

from unet_distributed_amd.launch import main

if __name__ == "__main__":
    sys.exit(main(["--create_inventory", sys.argv[1] if len(sys.argv) > 1 else "inv.yml"]))
