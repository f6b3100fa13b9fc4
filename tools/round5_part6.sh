#!/bin/bash
# Round 5, sixth call: BVH builder variants, same box -- B0 current; B2 all-axes binned SAH with 32 bins;
# B4 64 bins; B5 / B6 = B2 plus an exact SAH sweep for nodes of <= 65536 / 1024 triangles
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5r_ab_brdf:ROUNDS=2 VARIANTS=\"B0 B2 B4 B5 B6\" tools/ab_run.sh --mode brdf --steps 1" \
 "450:r5r_ab_mis:ROUNDS=2 VARIANTS=\"B0 B2 B4 B5 B6\" tools/ab_run.sh" \
 "450:r5r_ab_cornell:ROUNDS=2 VARIANTS=\"B0 B2 B4 B5 B6\" tools/ab_run.sh --scene cornell1m"
