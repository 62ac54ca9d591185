#!/bin/bash
# round-2: agents kernel without its private copy of the parameters; C4/HET/C3 checks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r02g.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r02g_1.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r02g_2.log 2>&1 || exit 3
timeout -k 10 200 python bench.py > gpurun_out/bench_r02g_long.log 2>&1 || exit 4
timeout -k 10 300 python tools/bench_configs.py --configs C3,HET,HS --steps 572 --warmup 20 > gpurun_out/bench_configs_r02g.log 2>&1 || exit 5
timeout -k 10 300 python tools/gpu/ma_probe.py > gpurun_out/ma_probe_r02g.log 2>&1 || exit 6
