#!/bin/bash
# Round 5, twentieth call: k_mis_combine with the children's points / normals parked in LDS across its
# barrier phase and its own inputs re-read after it (CP1: 12 spilled VGPRs -> 0) against HEAD (CP0), same
# box, C3 and C5; GPU tests on CP1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "400:r5cp_ab_mis:ROUNDS=3 VARIANTS=\"CP0 CP1\" tools/ab_run.sh" \
 "400:r5cp_ab_cornell:ROUNDS=2 VARIANTS=\"CP0 CP1\" tools/ab_run.sh --scene cornell1m" \
 "600:r5cp_gputests:MCPT_LIB_PATH=ab/libCP1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
