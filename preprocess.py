"""BraTS .mha -> .npy slices (see unet_distributed_amd/data/preprocess.py)."""
from unet_distributed_amd.data.preprocess import main

if __name__ == "__main__":
    main()
