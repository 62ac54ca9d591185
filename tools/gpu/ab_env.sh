# Same-box A/B of a HIP runtime environment variable on the C4 bench,
# alternating VAR=A / VAR=B: µs per step and the HIP-event kernel averages.
# usage: bash tools/gpu/ab_env.sh VAR A B [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
VAR=$1; VA=$2; VB=$3; STEPS=${4:-286}
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in "$VA" "$VB"; do
    env "$VAR=$v" timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 20 --no-cpu-baseline --no-variants \
      > gpurun_out/ab/env_${VAR}_${v}_$r.log 2>&1 || exit $?
    grep '"metric"' gpurun_out/ab/env_${VAR}_${v}_$r.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('$VAR=$v', 'us/step %.2f' % (d['ms_per_step'] * 1e3), 'episode %.2f' % (d['ms_per_step_episode'] * 1e3),
      ' '.join('%s %.2f' % (n, x['avg_us']) for n, x in d['kernels'].items()))"
  done
done
