# Fused kernel phase costs: full, agents only (PF skipped), PF only (agents skipped).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for d in 0 2 1 3; do
  PGW_COORD_FUSED_DBG=$d timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-variants > gpurun_out/bdbg_$d.log 2>&1 || { tail -20 gpurun_out/bdbg_$d.log; exit 1; }
  python - gpurun_out/bdbg_$d.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.2f us/step" % (d["ms_per_step"] * 1e3), {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()})
PY
done
