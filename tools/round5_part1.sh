#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"
exec tools/gpu_steps.sh \
 "300:r5l_ab_phong_brdf:ROUNDS=3 VARIANTS=\"S0 S1 S2\" tools/ab_run.sh --mode brdf --steps 1" \
 "300:r5l_ab_phong_mis:ROUNDS=2 VARIANTS=\"S0 S1 S2\" tools/ab_run.sh" \
 "300:r5k_ab_pk2_timing:ROUNDS=2 VARIANTS=\"C T1 T2\" tools/ab_run.sh" \
 "600:r5_gputests:python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread" \
 "300:r5_bench_default:python3 bench.py" \
 "240:r5_bench_brdf:python3 bench.py --mode brdf --steps 1 --no-cpu" \
 "300:r5_bench_shade:python3 bench.py --mode shade --no-cpu" \
 "300:r5_bench_shade_area:python3 bench.py --mode shade_area --no-cpu" \
 "300:r5_bench_cornell:python3 bench.py --scene cornell1m --no-cpu" \
 "300:r5_bench_fresh:python3 bench.py --fresh-pdf --no-cpu" \
 "300:r5_bench_fp32:python3 bench.py --precision fp32 --no-cpu" \
 "300:r5_bench_c4:python3 bench.py --config c4 --steps 1 --warmup 1 --no-cpu" \
 "300:r5_bench_torchrun1:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --no-cpu"
