#!/bin/bash
# Round 5, third call: same-box A/B of the zero-specular pow skip (P1 vs N) and of k_extend_brdf's
# occupancy (W6 / W4 waves per SIMD vs N's 5), then the GPU tests on the P1 build
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5o_ab_brdf:ROUNDS=3 VARIANTS=\"N P1 W6 W4\" tools/ab_run.sh --mode brdf --steps 1" \
 "300:r5o_ab_mis:ROUNDS=3 VARIANTS=\"N P1\" tools/ab_run.sh" \
 "300:r5o_ab_cornell:ROUNDS=2 VARIANTS=\"N P1\" tools/ab_run.sh --scene cornell1m" \
 "600:r5o_gputests_p1:MCPT_LIB_PATH=ab/libP1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
