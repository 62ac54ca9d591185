# Split PF kernel check: parity tests (new split test first), the short and
# long bench, and a rocprofv3 kernel-trace summary of the default bench shape.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-split}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "split or fused_equals or c4" \
  > gpurun_out/pytest_split_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_split_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_split_$TAG.log
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_s20_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_s20_$TAG.log; exit 1; }
timeout -k 10 200 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/bench_s572_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_s572_$TAG.log; exit 1; }
PGW_PF_SPLIT=0 timeout -k 10 200 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/bench_s572_onelane_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_s572_onelane_$TAG.log; exit 1; }
for f in s20 s572 s572_onelane; do python - gpurun_out/bench_${f}_$TAG.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()}, "copy %.0f" % d["stream_copy_gbs"],
      d["pf_iterations"])
PY
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 286 --warmup 20 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_$TAG.csv
cut -c1-160 gpurun_out/kernel_stats_$TAG.csv | head -8
