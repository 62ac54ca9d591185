# What the round-end driver runs: smoke(), pytest -m gpu, default bench.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${1:-drv}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_default_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_default_$TAG.log
