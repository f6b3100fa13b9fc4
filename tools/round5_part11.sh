#!/bin/bash
# Round 5, eleventh call: spatial splits for trees of >= 65536 triangles (the 1 M-triangle scene) -- GPU tests,
# the C5 and C3 benches, C5's kernel stats and PMC passes
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=round5w
exec tools/gpu_steps.sh \
 "600:r5w_gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "300:r5w_bench_cornell:python3 bench.py --scene cornell1m --no-cpu" \
 "300:r5w_bench_default:python3 bench.py" \
 "300:prof_cornell:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu" \
 "150:pmc_fetch_cornell:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu --no-replay --steps 1" \
 "150:pmc_write_cornell:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}_write_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu --no-replay --steps 1" \
 "150:pmc_sq_cornell:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${T}_sq_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu --no-replay --steps 1"
