#!/bin/bash
# Round 5, fourth call: near / far plane loads in trace4_ww (F1; F2 = F1 with k_mis_rays at 6 waves per
# SIMD) against the min / max slab form (F0), same box; GPU tests on F1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5p_ab_brdf:ROUNDS=3 VARIANTS=\"F0 F1\" tools/ab_run.sh --mode brdf --steps 1" \
 "400:r5p_ab_mis:ROUNDS=3 VARIANTS=\"F0 F1 F2\" tools/ab_run.sh" \
 "300:r5p_ab_shade:ROUNDS=2 VARIANTS=\"F0 F1\" tools/ab_run.sh --mode shade" \
 "600:r5p_gputests_f1:MCPT_LIB_PATH=ab/libF1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
