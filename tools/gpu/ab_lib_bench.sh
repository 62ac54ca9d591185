# Same-box A/B of two builds of the library on the driver-shaped bench: the
# tree's libpgw.so against abprev/libpgw.so (PGW_LIB_PATH), alternating.
# usage: bash tools/gpu/ab_lib_bench.sh [ROUNDS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=${1:-3}
for r in $(seq 1 $R); do
  for L in new prev; do
    P=$GRAFT_REPO_ROOT/powergridworld_amd/libpgw.so; [ $L = prev ] && P=$GRAFT_REPO_ROOT/abprev/libpgw.so
    PGW_LIB_PATH=$P timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-variants 2>/dev/null | grep '^{' | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
k = d['kernels']
print('$r $L', 'us/step %.2f' % (1e3 * d['ms_per_step']), 'value %.4g' % d['value'],
      ' '.join('%s %.2f' % (n, v['avg_us']) for n, v in k.items()))" || exit 1
  done
done
