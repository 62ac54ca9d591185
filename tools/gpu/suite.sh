# GPU check of the committed tree: smoke, the GPU test suite, a driver-shaped
# bench line.  Stops at the first failure.  Usage: bash tools/gpu/suite.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
K=${2:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  || { echo "SMOKE FAILED rc=$?"; tail -40 gpurun_out/smoke_$TAG.log; exit 1; }
tail -2 gpurun_out/smoke_$TAG.log
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" \
  > gpurun_out/pytest_gpu_$TAG.log 2>&1; rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_gpu_$TAG.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_$TAG.log | head -30; exit $rc; }
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.log 2>&1; rc=$?
tail -c 1500 gpurun_out/bench_$TAG.log
exit $rc
