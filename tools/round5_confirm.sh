#!/bin/bash
# Round 5, confirmation of the in-tree library after the last host-code change: smoke() and the GPU tests
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5h_smoke:python3 -c \"import __graft_entry__ as g; g.smoke()\"" \
 "600:r5h_gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "300:r5h_bench_default:python3 bench.py"
