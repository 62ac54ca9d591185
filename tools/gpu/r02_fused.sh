# Fused agents+PF kernel: variant bit-identity tests, whole GPU suite, then the
# driver-shaped and long benches with the fused kernel on and off.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-fz}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "split_pf_equals" --timeout 200 --timeout-method thread > gpurun_out/pytest_fused_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_fused_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_fused_$TAG.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for f in 1 0; do
  PGW_COORD_FUSED=$f timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants > gpurun_out/b20_f${f}_$TAG.log 2>&1 || { tail -20 gpurun_out/b20_f${f}_$TAG.log; exit 1; }
  PGW_COORD_FUSED=$f timeout -k 10 200 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/b572_f${f}_$TAG.log 2>&1 || { tail -20 gpurun_out/b572_f${f}_$TAG.log; exit 1; }
done
for f in gpurun_out/b20_f1_$TAG.log gpurun_out/b572_f1_$TAG.log gpurun_out/b20_f0_$TAG.log gpurun_out/b572_f0_$TAG.log; do python - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()})
PY
done
