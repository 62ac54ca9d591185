# Same-box A/B of two builds of the library on one bench_configs configuration:
# the tree's libpgw.so against abprev/libpgw.so (PGW_LIB_PATH), alternating
# three times, then one rocprofv3 kernel-trace pass each.
# usage: bash tools/gpu/ab_lib_pair.sh TAG CFG [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; STEPS=${3:-572}
export TMPDIR=/tmp
run() {   # $1 = label, $2 = library path
  PGW_LIB_PATH=$2 timeout -k 10 300 python -u tools/bench_configs.py --configs $CFG --steps $STEPS 2>/dev/null | grep '"config"' | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$r $1', d['config'], 'us/step %.2f' % d['us_per_step'])"
}
NEW=$GRAFT_REPO_ROOT/powergridworld_amd/libpgw.so
OLD=$GRAFT_REPO_ROOT/abprev/libpgw.so
for r in 1 2 3; do
  run new $NEW || exit 1
  run prev $OLD || exit 1
done
for L in new prev; do
  P=$NEW; [ $L = prev ] && P=$OLD
  cd /tmp && PGW_LIB_PATH=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/p_$L" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --configs $CFG --steps $STEPS > /dev/null 2>&1 || exit 1
  cd "$GRAFT_REPO_ROOT"
  f=$(find gpurun_out/p_$L -name "*kernel_stats.csv" | head -1)
  cp "$f" "gpurun_out/kstats_${TAG}_$L.csv"
  rm -rf "gpurun_out/p_$L"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kstats_${TAG}_$L.csv')):
    if any(k in r['Name'] for k in ('k_ma_step', 'k_pf_solve_od', 'k_mc_step', 'k_coord')):
        print('$L', r['Name'].split('(')[0].replace('void pgw::', ''), r['Calls'], 'avg %.2f us min %.2f us' % (float(r['AverageNs']) / 1e3, float(r['MinNs']) / 1e3))"
done
