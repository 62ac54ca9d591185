# Round 6: the split C4 step -- parity tests, then a same-box A/B (split on / off).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_pf_od.py tests/test_gpu_configs.py tests/test_gpu_reference_configs.py tests/test_gpu_checkpoint.py \
  "tests/test_gpu_parity.py::test_c4_fused_equals_generic_full_batch" > gpurun_out/r06b_tests.log 2>&1 || { tail -40 gpurun_out/r06b_tests.log; exit 1; }
tail -3 gpurun_out/r06b_tests.log
bash tools/gpu/ab_bench_args.sh split "--pf-split off" "--pf-split on" 286 | tee gpurun_out/r06b_ab.txt
