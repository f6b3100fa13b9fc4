#!/bin/bash
# Round 5, final confirmation of the in-tree library at the round-5 HEAD: smoke() and the GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5k_smoke:python3 -c \"import __graft_entry__ as g; g.smoke()\"" \
 "600:r5k_gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "300:r5k_bench_default:python3 bench.py"
