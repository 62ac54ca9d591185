# Fast PF kernel with 32 envs per wave vs one lane per env: bit-identity test,
# long benches alternated, phase traces.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_half.log 2>&1 || { tail -30 gpurun_out/pytest_half.log; exit 1; }
tail -1 gpurun_out/pytest_half.log
for rep in 1 2; do for h in 1 0; do
  PGW_PF_HALF=$h timeout -k 10 200 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/bh_${h}_$rep.log 2>&1 || { tail -20 gpurun_out/bh_${h}_$rep.log; exit 1; }
  python - gpurun_out/bh_${h}_$rep.log $h <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("half", sys.argv[2], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()}, d["pf_iterations"])
PY
done; done
PGW_PF_HALF=1 timeout -k 10 120 python tools/gpu/pf_trace.py > gpurun_out/pf_trace_half.txt 2>&1 || { tail -20 gpurun_out/pf_trace_half.txt; exit 1; }
head -12 gpurun_out/pf_trace_half.txt
