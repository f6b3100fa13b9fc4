#!/bin/bash
# Round-3 measurement set on one gpurun box: the GPU tests, a same-box A/B of the library builds in ab/
# (tools/ab_run.sh), and for the working tree (B) and round 2 (R) the rocprofv3 kernel stats and the PMC
# passes (FETCH_SIZE; WRITE_SIZE + GRBM_GUI_ACTIVE; SQ) that tools/summarize_profiles.py turns into
# profiles/round3*_.  Each step has its own time limit; a fatal exit stops the run (tools/gpu_steps.sh).
T=${TAG:-r3}
V=${VARIANTS:-R C T B}
exec tools/gpu_steps.sh \
 "500:gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "400:ab:ROUNDS=${ROUNDS:-2} VARIANTS=\"$V\" tools/ab_run.sh" \
 "120:bench_default:python3 bench.py --no-cpu" \
 "150:prof:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T} -o run --output-format csv -- python3 bench.py --no-cpu" \
 "120:pmc_fetch:rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmc_write:rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmc_sq:rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d gpurun_out/pmc_${T}_sq -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "150:profR:MCPT_LIB_PATH=ab/libR.so rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${T}R -o run --output-format csv -- python3 bench.py --no-cpu" \
 "120:pmcR_fetch:MCPT_LIB_PATH=ab/libR.so rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${T}R_fetch -o run --output-format csv -- python3 bench.py --no-cpu --steps 2" \
 "120:pmcR_write:MCPT_LIB_PATH=ab/libR.so rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc_${T}R_write -o run --output-format csv -- python3 bench.py --no-cpu --steps 2"
