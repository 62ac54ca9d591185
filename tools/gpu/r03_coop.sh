# k_coord_coop probe: parity (coop == two-launch, C4 goldens), then the
# driver-shaped bench with PGW_COORD_COOP = 0 (two launches), 5 (5 waves/SIMD
# bound) and 4 (4 waves/SIMD), and a rocprofv3 kernel trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-coop}
timeout -k 10 600 python -u -m pytest tests/test_gpu_coop.py tests/test_gpu_parity.py -k "coop or c4" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
for v in 0 5 4 0 5; do
  PGW_COORD_COOP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants > gpurun_out/bench_${TAG}_$v.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$v.log; exit 1; }
  python - "$v" gpurun_out/bench_${TAG}_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("COOP=%s %.4g %.2f us/step ep %.2f us" % (sys.argv[1], d["value"], d["ms_per_step"] * 1e3, d["ms_per_step_episode"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()}, d["pf_iterations"]["mean"])
PY
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_$TAG.csv
cut -d, -f1-4 gpurun_out/kernel_stats_$TAG.csv | cut -c1-150 | head -6
