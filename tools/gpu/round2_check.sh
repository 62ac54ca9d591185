# Round-2 check on one MI355X: new config tests first (verbose, per-test
# timeout), then the whole GPU suite, the default bench, and the self-launched
# N=2 rehearsal (bench.py starts torchrun itself; ranks share cuda:0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_cfg_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_cfg_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_cfg_$TAG.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
PGW_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 5 --batch 16384 \
  > gpurun_out/rehearse2_$TAG.log 2>&1 || { tail -20 gpurun_out/rehearse2_$TAG.log; exit 1; }
grep -o '"n_gpus": [0-9]*' gpurun_out/rehearse2_$TAG.log
