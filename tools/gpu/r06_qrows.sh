# Round 6: row records -- the PF / HET / history parity tests, then HET vs HETQ (row records off) on one box
# with rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/qrows
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pf_od.py \
  tests/test_gpu_reference_configs.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_checkpoint.py \
  tests/test_gpu_f32.py > gpurun_out/qrows/tests.log 2>&1 || { tail -60 gpurun_out/qrows/tests.log; exit 1; }
tail -3 gpurun_out/qrows/tests.log
for C in HET HETQ HET HETQ; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/qrows/$C -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_configs.py --configs $C --steps 572 > $GRAFT_REPO_ROOT/gpurun_out/qrows/$C.log 2>&1) || exit $?
  grep -h "us_per_step\|config" gpurun_out/qrows/$C.log | tail -1
  python3 -c "
import csv,glob
f=sorted(glob.glob('gpurun_out/qrows/$C/**/*kernel_stats.csv', recursive=True))[-1]
for r in csv.DictReader(open(f)):
    if 'k_pf_solve_od' in r['Name'] or 'k_ma_step' in r['Name']: print('   %-50s %6s %8.2f' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))"
done
