# Same-box A/B of several bench_configs configurations, alternating round-robin
# three times (no profiler), then one rocprofv3 kernel-trace pass per config.
# usage: bash tools/gpu/ab_configs_multi.sh TAG STEPS CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; STEPS=$2; shift 2
export TMPDIR=/tmp
for r in 1 2 3; do
  for C in "$@"; do
    timeout -k 10 300 python -u tools/bench_configs.py --configs $C --steps $STEPS 2>/dev/null | grep '"config"' | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$r', d['config'], 'us/step %.2f' % d['us_per_step'])" || exit 1
  done
done
for C in "$@"; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/p_$C" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --configs $C --steps $STEPS > /dev/null 2>&1 || exit 1
  cd "$GRAFT_REPO_ROOT"
  f=$(find gpurun_out/p_$C -name "*kernel_stats.csv" | head -1)
  cp "$f" "gpurun_out/kstats_${TAG}_$C.csv"
  rm -rf "gpurun_out/p_$C"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kstats_${TAG}_$C.csv')):
    if any(k in r['Name'] for k in ('k_ma_step', 'k_pf_solve_od', 'k_mc_step', 'k_coord')):
        print('$C', r['Name'].split('(')[0].replace('void pgw::', ''), r['Calls'], 'avg %.2f us min %.2f us' % (float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3))"
done
