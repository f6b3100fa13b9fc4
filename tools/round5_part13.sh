#!/bin/bash
# Round 5, thirteenth call: LDS top levels and occupancy re-tuned for the round-5 trees, same box --
# k_extend_brdf with 85 / 5 top nodes in LDS (BT85 / BT5; T0: 21); k_mis_rays with 21 top nodes (RT21;
# T0: 85) or at 6 waves per SIMD (R6; T0: 7)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5y_ab_brdf:ROUNDS=3 VARIANTS=\"T0 BT85 BT5\" tools/ab_run.sh --mode brdf --steps 1" \
 "400:r5y_ab_mis:ROUNDS=3 VARIANTS=\"T0 RT21 R6\" tools/ab_run.sh"
