# Same-box A/B of two bench_configs configurations, alternating A B A B A B (no profiler).
# usage: bash tools/gpu/ab_configs_pair.sh A B [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
A=$1; B=$2; STEPS=${3:-572}
for r in 1 2 3; do
  for C in $A $B; do
    timeout -k 10 300 python -u tools/bench_configs.py --configs $C --steps $STEPS 2>/dev/null | grep '"config"' | python3 -c "
import sys, json
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('$r', d['config'], 'us/step %.2f' % d['us_per_step'])" || exit 1
  done
done
