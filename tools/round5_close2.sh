#!/bin/bash
# Round 5, closing call 2: smoke(), then HEAD (incl. k_extend_brdf's parked throughput) as the
# default -- GPU tests, every bench configuration, then the rocprofv3 kernel stats and PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
tools/gpu_steps.sh \
 "300:r5j_smoke:python3 -c \"import __graft_entry__ as g; g.smoke()\"" \
 "600:r5j_gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "300:r5j_bench_default:python3 bench.py" \
 "240:r5j_bench_brdf:python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "300:r5j_bench_shade:python3 bench.py --mode shade --no-cpu" \
 "300:r5j_bench_shade_area:python3 bench.py --mode shade_area --no-cpu" \
 "300:r5j_bench_cornell:python3 bench.py --scene cornell1m --no-cpu" \
 "300:r5j_bench_fresh:python3 bench.py --fresh-pdf --no-cpu" \
 "300:r5j_bench_fp32:python3 bench.py --precision fp32 --no-cpu" \
 "300:r5j_bench_c4:python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu" \
 "300:r5j_bench_torchrun1:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu"
rc=$?
case $rc in 124|134|137|139) exit $rc ;; esac
[ $rc -gt 128 ] && exit $rc
TAG=round5j PART=2 exec tools/profile_steps.sh
