#!/bin/bash
# Round 5, fifth call: BVH builder variants (B1 = binned SAH over all three axes, B2 = B1 with 32 bins,
# B3 = 32 bins on the widest axis) against the current builder (B0), same box: C5, C3, C2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "400:r5q_ab_cornell:ROUNDS=2 VARIANTS=\"B0 B1 B2 B3\" tools/ab_run.sh --scene cornell1m" \
 "400:r5q_ab_mis:ROUNDS=2 VARIANTS=\"B0 B1 B2 B3\" tools/ab_run.sh" \
 "300:r5q_ab_brdf:ROUNDS=2 VARIANTS=\"B0 B1 B2 B3\" tools/ab_run.sh --mode brdf --steps 1"
