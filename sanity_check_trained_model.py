"""Average Dice of the exported model on the test set (see unet_distributed_amd/sanity_check.py)."""
from unet_distributed_amd.sanity_check import main

if __name__ == "__main__":
    main()
