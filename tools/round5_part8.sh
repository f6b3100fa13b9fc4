#!/bin/bash
# Round 5, eighth call: builder knobs on top of the round-5 builder (V0), same box -- SAH leaves of at most
# 1 / 3 triangles (L1 / L3; V0: 2), an inner-node cost of 1 / 2 triangle tests in the SAH (T1 / T2; V0: 0),
# the exact sweep at every node (X1)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5t_ab_brdf:ROUNDS=2 VARIANTS=\"V0 L1 L3 T1 T2 X1\" tools/ab_run.sh --mode brdf --steps 1" \
 "450:r5t_ab_mis:ROUNDS=2 VARIANTS=\"V0 L1 L3 T1 T2 X1\" tools/ab_run.sh" \
 "450:r5t_ab_cornell:ROUNDS=2 VARIANTS=\"V0 L1 L3 T1 T2 X1\" tools/ab_run.sh --scene cornell1m"
