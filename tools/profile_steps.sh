#!/bin/bash
# Round-end measurement set: GPU tests, the per-config benches (one through torchrun), rocprofv3
# kernel stats and the PMC passes (HBM bytes, SQ) under gpurun_out/; TAG names the run.  Summarised
# into profiles/ by tools/summarize_profiles.py and tools/prep_hbm_bytes.py.  PART=1 runs the tests
# and the benches, PART=2 the profiles (two gpurun calls fit the 20-minute limit).
T=${TAG:-r3}
if [ "${PART:-1}" = 1 ]; then
exec tools/gpu_steps.sh \
 "600:gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "300:bench_default:python3 bench.py" \
 "240:bench_brdf:python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "300:bench_shade:python3 bench.py --mode shade --no-cpu" \
 "300:bench_shade_area:python3 bench.py --mode shade_area --no-cpu" \
 "300:bench_cornell:python3 bench.py --scene cornell1m --no-cpu" \
 "300:bench_fresh:python3 bench.py --fresh-pdf --no-cpu" \
 "300:bench_fp32:python3 bench.py --precision fp32 --no-cpu" \
 "300:bench_c4:python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu" \
 "300:bench_torchrun1:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu"
else
exec tools/gpu_steps.sh \
 "300:prof:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 bench.py --no-cpu" \
 "120:pmc_fetch:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch -o run --output-format csv -- python3 bench.py --no-cpu --no-replay --steps 2" \
 "120:pmc_write:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}_write -o run --output-format csv -- python3 bench.py --no-cpu --no-replay --steps 2" \
 "120:pmc_sq:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${T}_sq -o run --output-format csv -- python3 bench.py --no-cpu --no-replay --steps 2" \
 "300:prof_brdf:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_brdf -o run --output-format csv -- python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "120:pmc_fetch_brdf:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch_brdf -o run --output-format csv -- python3 bench.py --mode brdf --steps 1 --no-cpu --no-replay" \
 "120:pmc_write_brdf:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}_write_brdf -o run --output-format csv -- python3 bench.py --mode brdf --steps 1 --no-cpu --no-replay" \
 "120:pmc_sq_brdf:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${T}_sq_brdf -o run --output-format csv -- python3 bench.py --mode brdf --steps 1 --no-cpu --no-replay" \
 "300:prof_cornell:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu" \
 "150:pmc_fetch_cornell:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu --no-replay --steps 1" \
 "150:pmc_write_cornell:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}_write_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu --no-replay --steps 1" \
 "150:pmc_sq_cornell:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${T}_sq_cornell -o run --output-format csv -- python3 bench.py --scene cornell1m --no-cpu --no-replay --steps 1"
fi
