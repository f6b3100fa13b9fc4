#!/bin/bash
# Round-end measurement set: GPU tests, the per-config benches (one through torchrun), rocprofv3
# kernel stats and the PMC passes (HBM bytes, SQ) under gpurun_out/; TAG names the run.  Summarised
# into profiles/ by tools/summarize_profiles.py and tools/prep_hbm_bytes.py.
T=${TAG:-r2}
exec tools/gpu_steps.sh \
 "600:gputests:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "300:bench_default:python3 bench.py" \
 "240:bench_brdf:python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "300:bench_shade:python3 bench.py --mode shade --no-cpu" \
 "300:bench_shade_area:python3 bench.py --mode shade_area --no-cpu" \
 "300:bench_cornell:python3 bench.py --scene cornell1m --no-cpu" \
 "300:bench_fresh:python3 bench.py --fresh-pdf --no-cpu" \
 "300:bench_fp32:python3 bench.py --precision fp32 --no-cpu" \
 "300:bench_c4shard:python3 bench.py --width 1600 --height 1200 --steps 2 --no-cpu" \
 "300:bench_torchrun1:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu" \
 "300:prof:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 bench.py --no-cpu" \
 "120:pmc_fetch:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmc_write:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmc_sq:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${T}_sq -o run --output-format csv -- python3 bench.py --no-cpu --steps 2"
