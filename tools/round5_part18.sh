#!/bin/bash
# Round 5, eighteenth call: the fp32 triangle pre-filter re-measured on the round-5 trees, same box --
# without it in k_extend_brdf (Q1) / k_mis_rays (Q2) against HEAD (Q0)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5q2_ab_brdf:ROUNDS=3 VARIANTS=\"Q0 Q1\" tools/ab_run.sh --mode brdf --steps 1" \
 "400:r5q2_ab_mis:ROUNDS=3 VARIANTS=\"Q0 Q2\" tools/ab_run.sh"
