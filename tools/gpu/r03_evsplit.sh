# Round-3 EV split walk: its parity tests, the GPU suite, then C3 / C3L / HET
# configs with the split on (default) and off, under rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mc_ or ev or het" > gpurun_out/pytest_evsplit.log 2>&1 || { tail -60 gpurun_out/pytest_evsplit.log; exit 1; }
tail -3 gpurun_out/pytest_evsplit.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_all_evsplit.log 2>&1 || { tail -60 gpurun_out/pytest_all_evsplit.log; exit 1; }
tail -3 gpurun_out/pytest_all_evsplit.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_evs_on -o run -- python3 tools/bench_configs.py --configs C3,C3L,C3G8,HET > gpurun_out/configs_evs_on.log 2>&1 || { tail -30 gpurun_out/configs_evs_on.log; exit 1; }
cat gpurun_out/configs_evs_on.log | grep '^{'
export PGW_MC_EV_SPLIT=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_evs_off -o run -- python3 tools/bench_configs.py --configs C3,C3L > gpurun_out/configs_evs_off.log 2>&1 || { tail -30 gpurun_out/configs_evs_off.log; exit 1; }
cat gpurun_out/configs_evs_off.log | grep '^{'
