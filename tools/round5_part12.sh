#!/bin/bash
# Round 5, twelfth call: C5 only -- leaves of <= 1 triangle (W1) and the spatial-split overlap threshold
# 1e-6 / 1e-4 of the root's area (W3 / W4) against the kept builder (W0: leaves <= 2, 1e-5), same box
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "500:r5x_ab_cornell:ROUNDS=3 VARIANTS=\"W0 W1 W3 W4\" tools/ab_run.sh --scene cornell1m"
