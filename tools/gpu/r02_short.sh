# Short-run (driver-shaped) bench variants: cold first-episode steps vs warm
# ones vs longer runs, split vs one-lane PF.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-short}
run() { name=$1; shift; timeout -k 10 200 "$@" --no-cpu-baseline --no-variants > gpurun_out/b_${name}_$TAG.log 2>&1 || { tail -20 gpurun_out/b_${name}_$TAG.log; exit 1; }
  python - gpurun_out/b_${name}_$TAG.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()})
PY
}
run s20w5 python bench.py --steps 20 --warmup 5
run s20w300 python bench.py --steps 20 --warmup 300
run s100w5 python bench.py --steps 100 --warmup 5
run s20w5again python bench.py --steps 20 --warmup 5
PGW_PF_SPLIT=0 run s20w5one python bench.py --steps 20 --warmup 5
PGW_PF_SPLIT=0 run s20w300one python bench.py --steps 20 --warmup 300
