#!/bin/bash
# Round 5, second measurement call: GPU tests and the C2 / C3 benches on the BRDF-only sample_phong change, then the
# rocprofv3 kernel-stats and PMC passes (tools/profile_steps.sh PART=2, TAG=round5)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tools/gpu_steps.sh \
 "600:r5n_gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "240:r5n_bench_brdf:python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "300:r5n_bench_shade_area:python3 bench.py --mode shade_area --no-cpu"
rc=$?
case $rc in 124|134|137|139) exit $rc ;; esac
[ $rc -gt 128 ] && exit $rc
TAG=round5 PART=2 exec tools/profile_steps.sh
