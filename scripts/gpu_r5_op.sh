#!/bin/bash
# Round 5 checks O + P: tconv data gradient on wide coarse rows (512^2) and the 3D first layer
# on the window kernel.
set -o pipefail
bash scripts/gpu_r5_o.sh && bash scripts/gpu_r5_p.sh
