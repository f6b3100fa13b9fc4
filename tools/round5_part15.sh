#!/bin/bash
# Round 5, fifteenth call: Phong's pow as exp2(y log2 x) in the BRDF-only kernels (E1) against pow (E0), same
# box, C2 (E2 = E1 with the frame's constant cross products written out); then the GPU tests on E2
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5e_ab_brdf:ROUNDS=3 VARIANTS=\"E0 E1 E2\" tools/ab_run.sh --mode brdf --steps 1" \
 "600:r5e_gputests_e2:MCPT_LIB_PATH=ab/libE2.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
