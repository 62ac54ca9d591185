set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.log 2>&1 || true
timeout -k 10 400 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED rc=$?"; tail -40 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 286 --warmup 20 --cpu-sample-envs 1024 --cpu-sample-steps 10 > gpurun_out/bench.log 2>&1; rc=$?
tail -5 gpurun_out/bench.log
exit $rc
