# Same-box timing of the C4 step as one launch: split off (two kernels), the
# list form (PGW_STEP_LIST=1: k_coord_step_od + the list kernel), the list form
# without its list launch (PGW_STEP_NOLIST=1, timing only: exact only for steps
# whose list is empty) -- the ceiling the one-launch step (ab_inline.sh) aims at.
# usage: bash tools/gpu/ab_nolist.sh [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
STEPS=${1:-286}
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in "off 0" "on 0" "on 1"; do
    set -- $v
    PGW_STEP_LIST=1 PGW_STEP_NOLIST=$2 timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 20 --no-cpu-baseline --no-variants \
      --pf-split $1 > gpurun_out/ab/nolist_$1_$2_$r.log 2>&1 || exit $?
    grep '"metric"' gpurun_out/ab/nolist_$1_$2_$r.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('split=$1 nolist=$2', 'us/step %.2f' % (d['ms_per_step'] * 1e3), 'episode %.2f' % (d['ms_per_step_episode'] * 1e3),
      ' '.join('%s %.2f' % (n, x['avg_us']) for n, x in d['kernels'].items()))"
  done
done
