# Same-box A/B of two bench.py argument sets on one library build, alternating
# A B A B A B: µs per step of a STEPS-step region and the HIP-event kernel
# averages.
# usage: bash tools/gpu/ab_bench_args.sh TAG "ARGS_A" "ARGS_B" [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; ARGA=$2; ARGB=$3; STEPS=${4:-286}
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then X=$ARGA; else X=$ARGB; fi
    timeout -k 10 300 python -u bench.py --steps $STEPS --warmup 20 --no-cpu-baseline --no-variants $X \
      > gpurun_out/ab/${TAG}_$v$r.log 2>&1 || exit $?
    grep '"metric"' gpurun_out/ab/${TAG}_$v$r.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
k = d['kernels']
print('$v$r', 'us/step %.2f' % (d['ms_per_step'] * 1e3), 'episode %.2f' % (d['ms_per_step_episode'] * 1e3),
      ' '.join('%s %.2f' % (n, v['avg_us']) for n, v in k.items()))"
  done
done
