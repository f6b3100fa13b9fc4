#!/bin/bash
# Round-end measurement set: GPU tests, the per-config benches, rocprofv3 kernel stats and the
# PMC passes (HBM bytes, SQ) under gpurun_out/; TAG names the run (default r1h).  Summarised
# into profiles/ by tools/summarize_profiles.py and tools/prep_hbm_bytes.py.
exec tools/gpu_steps.sh \
 "900:gputests:python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "300:bench_default:python3 bench.py" \
 "240:bench_brdf:python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "300:bench_shade:python3 bench.py --mode shade --no-cpu" \
 "300:bench_cornell:python3 bench.py --scene cornell1m --no-cpu" \
 "300:prof:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG:-r1h} -o run --output-format csv -- python3 bench.py --no-cpu" \
 "120:pmc_fetch:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG:-r1h}_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmc_write:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${TAG:-r1h}_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmc_sq:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${TAG:-r1h}_sq -o run --output-format csv -- python3 bench.py --no-cpu --steps 2"
