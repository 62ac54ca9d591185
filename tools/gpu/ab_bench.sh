# Same-box A/B of two library builds on the C4 headline bench, alternating
# A B A B (A = the build at LIB_A, B = the tree's libpgw.so): µs per step of a
# STEPS-step region and the HIP-event kernel averages.
# usage: bash tools/gpu/ab_bench.sh TAG LIB_A [STEPS] [extra bench.py args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; LIBA=$2; STEPS=${3:-286}; shift 3 2>/dev/null; EXTRA="$*"
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export PGW_LIB_PATH=$GRAFT_REPO_ROOT/$LIBA; else unset PGW_LIB_PATH; fi
    timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 20 --no-cpu-baseline --no-variants $EXTRA \
      > gpurun_out/ab/${TAG}_$v$r.log 2>&1 || exit $?
    grep '"metric"' gpurun_out/ab/${TAG}_$v$r.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
k = d['kernels']
print('$v$r', 'us/step %.2f' % (d['ms_per_step'] * 1e3), 'episode %.2f' % (d['ms_per_step_episode'] * 1e3),
      ' '.join('%s %.2f' % (n, v['avg_us']) for n, v in k.items()))"
  done
done
