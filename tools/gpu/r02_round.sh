# Driver-like round check: smoke, GPU suite, driver-shaped bench (with CPU
# baseline and variants), rocprofv3 kernel stats of the driver-shaped bench,
# then the config benches and their kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-rnd}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-200
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_$TAG.csv
cut -d, -f1-8 gpurun_out/kernel_stats_$TAG.csv | cut -c1-200 | head -8
bash tools/gpu/prof_configs.sh cfg_$TAG
