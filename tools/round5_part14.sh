#!/bin/bash
# Round 5, fourteenth call: the persistent traversal's occupancy on the round-5 trees (RW5 / RW7 / RW8 waves
# per SIMD vs P0's 6), same box: C5 and shade-area
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "400:r5z_ab_cornell:ROUNDS=2 VARIANTS=\"P0 RW5 RW7 RW8\" tools/ab_run.sh --scene cornell1m" \
 "300:r5z_ab_shade_area:ROUNDS=2 VARIANTS=\"P0 RW5 RW7 RW8\" tools/ab_run.sh --mode shade_area"
