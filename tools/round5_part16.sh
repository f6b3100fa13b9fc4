#!/bin/bash
# Round 5, sixteenth call: the MIS / shade kernels' Phong value and pdf through exp2(y log2 x) (M1) against
# pow (M0), same box, C3 and shade; then the GPU tests on M1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "400:r5m1_ab_mis:ROUNDS=3 VARIANTS=\"M0 M1\" tools/ab_run.sh" \
 "300:r5m1_ab_shade:ROUNDS=2 VARIANTS=\"M0 M1\" tools/ab_run.sh --mode shade" \
 "600:r5m1_gputests:MCPT_LIB_PATH=ab/libM1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
