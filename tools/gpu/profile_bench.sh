# rocprofv3 kernel-trace summary of a short bench run (+ a quick parity check first).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 286 --warmup 20 --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1 || exit $?
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_$TAG.csv
cat gpurun_out/kernel_stats_$TAG.csv | cut -c1-200 | head -20
