# Round-2 re-entry check: smoke, the whole GPU suite (verbose), the
# driver-shaped bench, the self-launched N=2 rehearsal, and a kernel trace of
# the driver-shaped bench (per-dispatch timestamps: where the short run's time
# goes between launches).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-r02b}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
PGW_BENCH_REHEARSE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 5 --batch 16384 --no-variants \
  > gpurun_out/rehearse2_$TAG.log 2>&1 || { tail -20 gpurun_out/rehearse2_$TAG.log; exit 1; }
grep -o '"n_gpus": [0-9]*' gpurun_out/rehearse2_$TAG.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_$TAG.csv
find gpurun_out/prof/$TAG -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_trace_$TAG.csv
tail -1 gpurun_out/prof_$TAG.log | cut -c1-300
