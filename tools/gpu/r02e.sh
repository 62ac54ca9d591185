#!/bin/bash
# round-2 check of the fused multi-agent step: het GPU tests, config benches, rocprof kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "het" > gpurun_out/pytest_het_r02e.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_configs.py --configs HET,HETG --steps 572 --warmup 20 > gpurun_out/bench_het_r02e.log 2>&1 || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_het -o het -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs HET --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_het.log 2>&1 || exit 3
