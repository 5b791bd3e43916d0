"""Static configuration constants.

Mirrors the module-level constants of the reference's ``settings_dist.py``
(`settings_dist.py:1-42`) so that code written against the reference can read
the same names.  Every value can be overridden at run time by the CLI flags in
:mod:`unet_distributed_amd.config` (the reference derives its ``tf.app.flags``
defaults from these constants the same way, `test_dist.py:64-85`).

Differences from the reference, all deliberate:

* the cluster host tables default to a single-node ``127.0.0.1`` layout; on
  MI355X one process per GPU rendezvous through ``MASTER_ADDR``/``MASTER_PORT``
  (torch.distributed env://) instead of hard-coded gRPC host lists
  (`settings_dist.py:36-39`);
* paths default to locations under the current working directory instead of
  ``/home/bduser``/``/data03`` (`settings_dist.py:1-3,41`).
"""

import os

BASE = os.environ.get("UNET_DATA_BASE", os.path.join(os.getcwd(), "data"))
DATA_PATH = os.path.join(BASE, "slices")
OUT_PATH = os.path.join(BASE, "slices", "Results")
IMG_ROWS = 128
IMG_COLS = 128
RESCALE_FACTOR = 1
SLICE_BY = 5

IN_CHANNEL_NO = 1
OUT_CHANNEL_NO = 1

EPOCHS = 10

# CPU threading knobs of the reference (`settings_dist.py:14-16`). On the GPU
# path they size the host data-loader thread pool instead of MKL/OpenMP.
BLOCKTIME = 0
NUM_INTRA_THREADS = 50
NUM_INTER_THREADS = 2
BATCH_SIZE = 1024

LEARNINGRATE = 0.0005
DECAY_STEPS = 100
LR_FRACTION = 0.2
CONST_LEARNINGRATE = True

USE_UPSAMPLING = False  # True = UpSampling2D; False = Conv2DTranspose

MODEL_FN = "brainWholeTumor"

# Segmentation modes (`settings_dist.py:28-33`, `preprocess.py:287-350`):
#   1: FLAIR -> whole tumour (test Dice 0.78-0.80 in the reference)
#   2: T1c   -> enhancing tumour (0.65-0.75)
#   3: T2    -> tumour core (0.50-0.55)
#   4: [EXT] all four modalities -> whole tumour (the BASELINE 128x128x4 config)
MODE = 1

# Host tables. Kept for parity with the reference's parameter-server layout
# (`settings_dist.py:36-39`); the single-node launcher ignores them.
PS_HOSTS = []
PS_PORTS = []
WORKER_HOSTS = ["127.0.0.1"]
WORKER_PORTS = ["29500"]
GPUS_PER_NODE = int(os.environ.get("UNET_GPUS_PER_NODE", "8"))   # MI355X node: 8 GPUs on xGMI
MASTER_PORT = 29500

CHECKPOINT_DIRECTORY = os.environ.get(
    "UNET_CHECKPOINT_DIRECTORY", os.path.join(os.getcwd(), "checkpoints"))
TENSORBOARD_IMAGES = 3
