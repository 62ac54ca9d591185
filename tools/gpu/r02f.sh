#!/bin/bash
# round-2: full GPU suite, config benches (C2, C3, HET, HS) and the fused-step probe
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r02f.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_configs.py --configs C2,C3,HET,HS --steps 572 --warmup 20 > gpurun_out/bench_configs_r02f.log 2>&1 || exit 2
timeout -k 10 300 python tools/gpu/ma_probe.py > gpurun_out/ma_probe_r02f.log 2>&1 || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cfg_f -o cfg -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs C3,HET,HS --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_cfg_f.log 2>&1 || exit 4
