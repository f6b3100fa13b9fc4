#!/bin/bash
# Round 5, twenty-first call: earlier rounds' tuning knobs re-measured at HEAD, same box -- k_mis_gen at 5 waves
# per SIMD (X1; X0: no bound, 114 VGPRs / 4 waves), the cull over 8 chunk ranges (X2; X0: 6), the persistent
# traversal taking 128 pool items per atomic (X3; X0: 256)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "500:r5x2_ab_mis:ROUNDS=3 VARIANTS=\"X0 X1 X2\" tools/ab_run.sh" \
 "300:r5x2_ab_cornell:ROUNDS=2 VARIANTS=\"X0 X3\" tools/ab_run.sh --scene cornell1m"
