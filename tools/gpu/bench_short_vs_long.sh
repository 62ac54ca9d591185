# Driver-shaped short bench (--steps 20 --warmup 5, CPU baseline first) beside
# the same without the CPU baseline and a long run: separates clock ramp /
# pipeline-fill effects from the steady state.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-x}
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_s20_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants > gpurun_out/bench_s20nocpu_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/bench_s572_$TAG.log 2>&1 || exit 1
for f in s20 s20nocpu s572; do python - gpurun_out/bench_${f}_$TAG.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()}, "copy %.0f" % d["stream_copy_gbs"])
PY
done
