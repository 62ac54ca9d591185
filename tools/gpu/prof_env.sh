# rocprofv3 kernel trace of the C4 bench under environment settings (same box):
# per-launch duration percentiles of the step's kernels and the bench's us/step.
# usage: bash tools/gpu/prof_env.sh TAG "VAR=v ..." ["VAR=v ..." ...]   (extra bench args in BENCH_ARGS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
mkdir -p gpurun_out/prof_env/$TAG
i=0
for SET in "$@"; do
  i=$((i+1)); d=gpurun_out/prof_env/$TAG/v$i
  (cd /tmp && env $SET timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 572 --warmup 20 --no-cpu-baseline --no-variants --time-steps 8 $BENCH_ARGS > $GRAFT_REPO_ROOT/$d.log 2>&1) || exit $?
  f=$(find $d -name '*kernel_trace.csv' | head -1)
  python3 - "$f" "$SET" "$d.log" <<'PY'
import csv, sys, json, numpy as np
rows = list(csv.DictReader(open(sys.argv[1])))
line = [l for l in open(sys.argv[3]) if l.startswith('{"metric"')]
us = json.loads(line[-1])["ms_per_step"] * 1e3 if line else float("nan")
print("[%s] bench us/step (under rocprof) %.2f" % (sys.argv[2], us))
names = sorted({r["Kernel_Name"].split("(")[0] for r in rows if "k_coord" in r["Kernel_Name"] or "k_step_nop" in r["Kernel_Name"]})
for nm in names:
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if r["Kernel_Name"].startswith(nm)])
    print("   %-45s n %5d p10 %.2f p50 %.2f p90 %.2f mean %.2f" % ((nm[-45:], len(d)) + tuple(np.percentile(d, [10, 50, 90])) + (d.mean(),)))
ks = sorted([r for r in rows if "k_coord" in r["Kernel_Name"]], key=lambda r: int(r["Start_Timestamp"]))
st = np.array([int(r["Start_Timestamp"]) for r in ks]); en = np.array([int(r["End_Timestamp"]) for r in ks])
per_step = np.diff(st[::2]) / 1e3
print("   device time per step (start-to-start of the step's first kernel): p10 %.2f p50 %.2f p90 %.2f" % tuple(np.percentile(per_step, [10, 50, 90])))
PY
done
