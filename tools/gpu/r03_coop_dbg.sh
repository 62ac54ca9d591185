# k_coord_coop phases: PGW_COOP_DBG=1 (block-shaped agent phase alone), 2 (+
# barrier, predictor loads, no iteration), 0 (full), and the two-launch step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dbg}; shift
for cfg in ${@:-0:x 5:1 5:2 5:0}; do
  set -- ${cfg/:/ }
  PGW_COORD_COOP=$1 PGW_COOP_DBG=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants > gpurun_out/bench_${TAG}_$1_$2.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}_$1_$2.log; exit 1; }
  python - "$cfg" gpurun_out/bench_${TAG}_$1_$2.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("COOP,DBG=%s %.4g %.2f us/step" % (sys.argv[1], d["value"], d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()})
PY
done
