# GPU tests of a round-3 change: the named test files first (verbose), then
# the whole GPU suite.  Usage: bash tools/gpu/r03_tests.sh TAG [test files...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-t}; shift
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -3 gpurun_out/pytest_$TAG.log
fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_all_$TAG.log 2>&1 || { tail -60 gpurun_out/pytest_all_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_all_$TAG.log
