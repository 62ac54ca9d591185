set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-m}
timeout -k 10 600 python -u -m pytest tests/test_gpu_pf_general.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_pfg_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_pfg_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_pfg_$TAG.log
bash tools/gpu/r03_ev.sh $TAG
