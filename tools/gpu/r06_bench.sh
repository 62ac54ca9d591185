# Round 6: graph test, then the default bench (with variants and the CPU baseline), then rocprof stats of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_graph.py > gpurun_out/r06c_graph.log 2>&1 || { tail -40 gpurun_out/r06c_graph.log; exit 1; }
tail -3 gpurun_out/r06c_graph.log
timeout -k 10 600 python -u bench.py > gpurun_out/r06c_bench.log 2>&1 || { tail -30 gpurun_out/r06c_bench.log; exit 1; }
grep '"metric"' gpurun_out/r06c_bench.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
print('value %.4g us/step %.2f episode %.2f' % (d['value'], d['ms_per_step']*1e3, d['ms_per_step_episode']*1e3))
print('cold', json.dumps(d['episode_cold']))
for k, v in d['variants'].items(): print(k, '%.4g' % v['value'], '%.2f us' % (v['ms_per_step']*1e3))
print('roofline', json.dumps(d['roofline']))
"
