# rocprofv3 kernel trace of the C4 bench (split step) with k_coord_pf_od_list grids G (same box):
# per-launch duration percentiles of the step's two kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_lg
for G in "$@"; do
  (cd /tmp && PGW_OD_LIST_GRID=$G timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_lg/g$G -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 572 --warmup 20 --no-cpu-baseline --no-variants --time-steps 8 > $GRAFT_REPO_ROOT/gpurun_out/prof_lg/g$G.log 2>&1) || exit $?
  f=$(find gpurun_out/prof_lg/g$G -name '*kernel_trace.csv' | head -1)
  python3 - "$f" "$G" <<'PY'
import csv, sys, numpy as np
rows = list(csv.DictReader(open(sys.argv[1])))
for nm in ("k_coord_step_od", "k_coord_pf_od_list"):
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if nm in r["Kernel_Name"]])
    print("G=%s %-20s n %5d p10 %.2f p50 %.2f p90 %.2f p99 %.2f mean %.2f" % ((sys.argv[2], nm, len(d)) + tuple(np.percentile(d, [10, 50, 90, 99])) + (d.mean(),)))
PY
done
