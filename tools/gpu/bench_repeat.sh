# The driver-shaped bench N times on one box (full command, CPU baseline
# included), printing each headline with its host-side region diagnostics.
# usage: bash tools/gpu/bench_repeat.sh N [extra bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
N=${1:-3}; shift
for r in $(seq 1 $N); do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/bench_rep_$r.log 2>&1 || exit 1
  python3 -c "
import json
d = json.loads([l for l in open('gpurun_out/bench_rep_$r.log') if l.startswith('{')][-1])
h = d['host_region']
print('$r', 'us/step %.2f' % (1e3 * d['ms_per_step']), 'episode %.2f' % (1e3 * d['ms_per_step_episode']),
      ' '.join('%s %.2f' % (n, v['avg_us']) for n, v in d['kernels'].items()),
      '| host issue %.0f us, wait %.0f us, slowest step %.0f us at %d, median %.0f us' % (
          h['issue_us'], h['sync_wait_us'], h['step_max_us'], h['step_max_at'], h['step_median_us']))"
done
