"""Rank-0 metric logging: stdout, JSONL and TensorBoard events.

Mirrors the reference's observability: the tqdm-style
progress line with (loss, dice) (`test_dist.py:456-459`), the per-epoch TEST
DATASET block (`test_dist.py:430-433`), and TensorBoard tags ``loss``,
``dice``, ``sensitivity``, ``specificity``, ``percent_complete`` and
``*_test`` (`test_dist.py:275-298,322-326`).  Adds images/sec (global) and
the learning rate.  Non-chief ranks log nothing (the reference's chief-only
summary op, Q8: no extra forward pass is run for logging).
"""

import json
import sys
import time

from .events import EventWriter


class MetricLogger:
    def __init__(self, cfg, is_chief: bool, logdir: str):
        self.cfg = cfg
        self.on = is_chief
        self.jsonl = None
        self.events = None
        if not self.on:
            return
        if cfg.log_jsonl:
            self.jsonl = open(cfg.log_jsonl, "a")
        if cfg.tensorboard and not cfg.no_checkpoint:
            try:
                self.events = EventWriter(logdir)
            except OSError:
                self.events = None
        self.t0 = time.time()
        from .. import settings
        self.max_images = int(getattr(settings, "TENSORBOARD_IMAGES", 3))

    def _emit(self, rec):
        if self.jsonl:
            self.jsonl.write(json.dumps(rec) + "\n")
            self.jsonl.flush()

    # TF 1.x uniquifies the second summary op of a name: the histograms the reference
    # adds next to the scalars (`test_dist.py:275-282`) carry the tags "<name>_1"
    HIST_TAGS = {"loss": "loss_1", "dice": "dice_1", "sensitivity": "sensitivity_1",
                 "specificity": "specificity_1"}

    def train(self, step, m, total, images=None):
        """images: optional {"predictions", "ground_truth", "images"} -> [n, H, W] arrays
        (first TENSORBOARD_IMAGES samples of the step's batch, `test_dist.py:285-287`)."""
        if not self.on:
            return
        if self.cfg.progress:
            print("step %d/%d (loss=%.4f, dice=%.4f) %.1f img/s lr=%.2e"
                  % (step, total, m["loss"], m["dice"], m["images_per_sec"], m["lr"]), flush=True)
        self._emit(dict(kind="train", step=step, time=time.time() - self.t0, **m))
        if self.events:
            self.events.scalars(step, {k: m[k] for k in ("loss", "dice", "sensitivity", "specificity",
                                                           "percent_complete", "images_per_sec")})
            for k, tag in self.HIST_TAGS.items():
                self.events.histogram(step, tag, [m[k]])
            for tag, arr in (images or {}).items():
                self.events.images(step, tag, arr, max_outputs=self.max_images)
            self.events.flush()

    def test(self, step, m, epoch, epochs, final=False):
        if not self.on:
            return
        print("\nEpoch {} of {}: TEST DATASET\nloss = {:.4f}\nDice = {:.4f}\n"
              "Sensitivity = {:.4f}\nSpecificity = {:.4f}".format(
                  epoch, epochs, m["loss"], m["dice"], m["sensitivity"], m["specificity"]), flush=True)
        self._emit(dict(kind="test_final" if final else "test", step=step, **m))
        if self.events:
            self.events.scalars(step, {"loss_test": m["loss"], "dice_test": m["dice"],
                                       "sensitivity_test": m["sensitivity"],
                                       "specificity_test": m["specificity"]})
            self.events.flush()

    def close(self):
        if self.jsonl:
            self.jsonl.close()
        if self.events:
            self.events.close()
