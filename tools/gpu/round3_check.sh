# Round-3 check on one MI355X: smoke, the whole GPU suite, the driver-shaped
# bench, a rocprofv3 kernel-stats run of the same bench command, and the PMC
# traffic / occupancy passes (each its own rocprofv3 --pmc run).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-r03}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-300
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_$TAG.csv
cut -d, -f1-4 gpurun_out/kernel_stats_$TAG.csv | cut -c1-120 | head -6
run_pass() {
  name=$1; shift
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$TAG/$name" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/pmc/${TAG}_$name.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run_pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit 1
run_pass p3 FETCH_SIZE || exit 1
run_pass p4 WRITE_SIZE || exit 1
python tools/gpu/pmc_summary.py $TAG > gpurun_out/pmc_$TAG.txt
python tools/gpu/pmc_traffic.py $TAG > gpurun_out/pmc_traffic_$TAG.txt 2>&1 || true
echo check-done
