#!/bin/bash
# Round 5, nineteenth call: k_extend_brdf with the child's throughput parked in LDS during the traversal
# (PK1: no spills at 5 waves per SIMD; PK2: the same at 6 waves) against HEAD (PK0: 14 spilled VGPRs); GPU
# tests on PK1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5pk_ab_brdf:ROUNDS=3 VARIANTS=\"PK0 PK1 PK2\" tools/ab_run.sh --mode brdf --steps 1" \
 "600:r5pk_gputests:MCPT_LIB_PATH=ab/libPK1.so python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread"
