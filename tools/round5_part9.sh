#!/bin/bash
# Round 5, ninth call: SAH-optimal 4-wide collapse (D1, MCPT_BVH4_DP) against the greedy largest-area
# collapse (D0), same box; then the GPU tests on D1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5u_ab_brdf:ROUNDS=3 VARIANTS=\"D0 D1\" tools/ab_run.sh --mode brdf --steps 1" \
 "400:r5u_ab_mis:ROUNDS=3 VARIANTS=\"D0 D1\" tools/ab_run.sh" \
 "400:r5u_ab_cornell:ROUNDS=2 VARIANTS=\"D0 D1\" tools/ab_run.sh --scene cornell1m" \
 "600:r5u_gputests_d1:MCPT_LIB_PATH=ab/libD1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
