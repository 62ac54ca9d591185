# rocprofv3 kernel stats of the C4 bench with the split step on and off (same box).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_split
for v in on off; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_split/$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 572 --warmup 20 --no-cpu-baseline --no-variants --time-steps 8 --pf-split $v > $GRAFT_REPO_ROOT/gpurun_out/prof_split/$v.log 2>&1) || exit $?
  echo "== $v"; grep -h '"metric"' gpurun_out/prof_split/$v.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('us/step %.2f' % (d['ms_per_step']*1e3))"
  f=$(find gpurun_out/prof_split/$v -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:8]: print('%-60s calls %6s avg_us %8.2f' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))"
done
