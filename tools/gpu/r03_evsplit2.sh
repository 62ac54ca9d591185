# Round-3 EV split walk (split on steps of 2+ chunks): parity tests, smoke, the
# GPU suite, the C3 A/B under rocprofv3, then the headline bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "mc_ or ev or het" > gpurun_out/pytest_evsplit2.log 2>&1 || { tail -60 gpurun_out/pytest_evsplit2.log; exit 1; }
tail -n 1 gpurun_out/pytest_evsplit2.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_evsplit2.log 2>&1 || { tail -30 gpurun_out/smoke_evsplit2.log; exit 1; }
tail -n 2 gpurun_out/smoke_evsplit2.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_all_evsplit2.log 2>&1 || { tail -60 gpurun_out/pytest_all_evsplit2.log; exit 1; }
tail -n 1 gpurun_out/pytest_all_evsplit2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_evs2_on -o run -- python3 tools/bench_configs.py --configs C3,C3G8,HET > gpurun_out/configs_evs2_on.log 2>&1 || { tail -30 gpurun_out/configs_evs2_on.log; exit 1; }
grep '^{' gpurun_out/configs_evs2_on.log
PGW_MC_EV_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_evs2_off -o run -- python3 tools/bench_configs.py --configs C3 > gpurun_out/configs_evs2_off.log 2>&1 || { tail -30 gpurun_out/configs_evs2_off.log; exit 1; }
grep '^{' gpurun_out/configs_evs2_off.log
timeout -k 10 300 python3 tools/bench_configs.py --configs C3 > gpurun_out/configs_evs2_c3plain.log 2>&1 || exit 1
grep '^{' gpurun_out/configs_evs2_c3plain.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_evsplit2.log 2>&1 || { tail -30 gpurun_out/bench_evsplit2.log; exit 1; }
tail -n 1 gpurun_out/bench_evsplit2.log
