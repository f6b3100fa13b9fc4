#!/bin/bash
# Round 5, tenth call: spatial splits in the builder (S1, MCPT_BVH_SPATIAL) against the object-split builder
# (S0), same box; then the GPU tests on S1 (golden rays, brute-force edge rays, frames vs the oracle)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5v_ab_brdf:ROUNDS=3 VARIANTS=\"S0 S1\" tools/ab_run.sh --mode brdf --steps 1" \
 "400:r5v_ab_mis:ROUNDS=3 VARIANTS=\"S0 S1\" tools/ab_run.sh" \
 "400:r5v_ab_cornell:ROUNDS=2 VARIANTS=\"S0 S1\" tools/ab_run.sh --scene cornell1m" \
 "300:r5v_ab_shade_area:ROUNDS=2 VARIANTS=\"S0 S1\" tools/ab_run.sh --mode shade_area" \
 "600:r5v_gputests_s1:MCPT_LIB_PATH=ab/libS1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
