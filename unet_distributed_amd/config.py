"""CLI flag surface.

Accepts every flag the reference trainer defines with ``tf.app.flags``
(`test_dist.py:64-85`) with the same names, types and defaults, plus the
README-only spellings (`README.md:63-71`) as aliases, plus the extensions the
MI355X framework adds (dtype, norm, dims, synthetic data, ...).

Boolean flags follow absl/``tf.app.flags`` conventions so that reference
command lines keep working: ``--use_upsampling``, ``--use_upsampling=True``,
``--use_upsampling=false`` and ``--nouse_upsampling`` are all accepted.
"""

import argparse
import dataclasses
import socket
from typing import List, Optional

from . import settings


def _str2bool(v):
    if isinstance(v, bool):
        return v
    s = str(v).strip().lower()
    if s in ("1", "true", "t", "yes", "y", "on"):
        return True
    if s in ("0", "false", "f", "no", "n", "off"):
        return False
    raise argparse.ArgumentTypeError("expected a boolean, got %r" % v)


def _default_ip():
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return "127.0.0.1"


@dataclasses.dataclass
class Config:
    # --- reference flags (test_dist.py:64-85) ---
    const_learningrate: bool = settings.CONST_LEARNINGRATE
    learning_rate: float = settings.LEARNINGRATE
    lr_fraction: float = settings.LR_FRACTION
    decay_steps: int = settings.DECAY_STEPS
    is_sync: int = 1
    ip: str = "127.0.0.1"
    batch_size: int = settings.BATCH_SIZE          # GLOBAL batch, split over ranks
    epochs: int = settings.EPOCHS
    use_upsampling: bool = settings.USE_UPSAMPLING
    # --- README-only flags (README.md:63-66): host loader threads on GPU ---
    num_threads: int = settings.NUM_INTRA_THREADS
    num_inter_threads: int = settings.NUM_INTER_THREADS
    blocktime: int = settings.BLOCKTIME
    # --- extensions ---
    dtype: str = "bf16"              # fp32 | bf16 | fp16 (compute dtype)
    norm: str = "none"               # none | batch | group
    groups: int = 8                  # GroupNorm groups
    dims: int = 2                    # 2 | 3
    in_channels: int = settings.IN_CHANNEL_NO
    out_channels: int = settings.OUT_CHANNEL_NO
    img_size: int = settings.IMG_ROWS
    base_filters: int = 32
    depth: int = 4
    dropout: float = 0.2
    eval_dropout: bool = False       # reference keeps dropout on at eval (Q9)
    loss: str = "dice"               # dice | dice_bce
    bce_weight: float = 1.0
    mode: int = settings.MODE
    synthetic: bool = False
    synthetic_train: int = 2048
    synthetic_test: int = 256
    synthetic_difficulty: str = "easy"   # easy | hard (datasets.synthetic_brats)
    data_on_device: str = "auto"     # auto | on | off: keep the train set resident in HBM
    data_path: str = settings.OUT_PATH
    steps: int = 0                   # >0 overrides epochs*num_batches
    seed: int = 816
    checkpoint_dir: str = settings.CHECKPOINT_DIRECTORY
    save_model_secs: float = 60.0
    no_checkpoint: bool = False
    resume: bool = True
    bucket_mb: float = 8.0
    overlap_comm: bool = True
    backend: str = "auto"            # auto | native | torch
    device: str = "auto"             # auto | cuda | cpu
    dist_backend: str = "auto"       # auto | nccl | gloo
    dist_timeout_s: float = 300.0
    profile: bool = False
    profile_steps: str = "5,10"
    log_every: int = 10
    log_jsonl: str = ""
    tensorboard: bool = True
    export: bool = True
    fault_inject_step: int = -1
    fault_inject_rank: int = -1
    fault_inject_overflow_step: int = -1   # fp16 test hook: poison this step's gradient
    check_sync_every: int = 0        # cross-rank parameter checksum every K steps
    deterministic: bool = False      # torch path: deterministic algorithms (native path always is)
    serialize_kernels: bool = False  # debug: AMD_SERIALIZE_KERNEL=3 + HIP_LAUNCH_BLOCKING=1
    launch_tensorboard: bool = False # start `tensorboard --logdir` on the chief if installed
    hip_graph: bool = True           # native: replay the forward / Adam as HIP graphs (the bench default)
    progress: bool = True
    loss_scale: float = 0.0          # fp16 static loss scale (0 = dynamic)

    @property
    def method_up(self):
        return "upsample2D" if self.use_upsampling else "conv2DTranspose"


_BOOL_FLAGS = [f.name for f in dataclasses.fields(Config) if f.type in (bool, "bool")]

_ALIASES = {
    "learningrate": "learning_rate",   # README.md:68
}

_CHOICES = {
    "dtype": ("fp32", "bf16", "fp16"),
    "norm": ("none", "batch", "group"),
    "loss": ("dice", "dice_bce"),
    "backend": ("auto", "native", "torch"),
    "device": ("auto", "cuda", "cpu"),
    "dist_backend": ("auto", "nccl", "gloo"),
    "data_on_device": ("auto", "on", "off"),
    "synthetic_difficulty": ("easy", "hard"),
}


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(
        description="MI355X-native distributed UNet trainer "
                    "(flag-compatible with the reference test_dist.py)")
    defaults = Config()
    for f in dataclasses.fields(Config):
        name = f.name
        default = getattr(defaults, name)
        if name in _BOOL_FLAGS:
            p.add_argument("--" + name, dest=name, nargs="?", const=True,
                           default=default, type=_str2bool)
            p.add_argument("--no" + name, dest=name, action="store_false")
        else:
            kw = dict(dest=name, default=default, type=type(default))
            if name in _CHOICES:
                kw["choices"] = _CHOICES[name]
            p.add_argument("--" + name, **kw)
    for alias, target in _ALIASES.items():
        p.add_argument("--" + alias, dest=target, type=float,
                       default=argparse.SUPPRESS)
    return p


def parse_args(argv: Optional[List[str]] = None) -> Config:
    ns, unknown = build_parser().parse_known_args(argv)
    if unknown:
        raise SystemExit("unrecognised flags: %s" % " ".join(unknown))
    cfg = Config(**vars(ns))
    validate(cfg)
    return cfg


def validate(cfg: Config) -> None:
    if cfg.dims not in (2, 3):
        raise SystemExit("--dims must be 2 or 3")
    if cfg.img_size % (1 << cfg.depth) != 0:
        raise SystemExit("--img_size must be divisible by 2**depth")
    if cfg.batch_size <= 0:
        raise SystemExit("--batch_size must be positive")
    if not 0.0 <= cfg.dropout < 1.0:
        raise SystemExit("--dropout must be in [0, 1)")
