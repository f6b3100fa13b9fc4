#!/bin/bash
# Round 5, seventeenth call: occupancy knobs at HEAD, same box -- k_mis_rays at 5 waves per SIMD (K1; K0: 6) or
# with 6 LDS stack entries (K2; K0: 8); k_extend_brdf at 6 waves per SIMD (K3; K0: 5)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "400:r5k2_ab_mis:ROUNDS=3 VARIANTS=\"K0 K1 K2\" tools/ab_run.sh" \
 "300:r5k2_ab_brdf:ROUNDS=3 VARIANTS=\"K0 K3\" tools/ab_run.sh --mode brdf --steps 1"
