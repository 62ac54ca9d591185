# EV rebuild check: EV / MC / heterogeneous / HS parity tests, the EV probe,
# then the config benches with rocprofv3 kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-ev}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "ev or mc or het or hs or oob or vector or reference" --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python tools/gpu/ev_probe.py > gpurun_out/ev_probe_$TAG.txt 2>&1 || { tail -20 gpurun_out/ev_probe_$TAG.txt; exit 1; }
grep vehicles gpurun_out/ev_probe_$TAG.txt
bash tools/gpu/prof_configs.sh cfg_$TAG C3,HET
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/c3c_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/tools/gpu/c3_components.py" > "$GRAFT_REPO_ROOT/gpurun_out/prof_c3c_$TAG.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof/c3c_$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_c3c_$TAG.csv
cut -d, -f1-4 gpurun_out/kernel_stats_c3c_$TAG.csv | cut -c1-120 | head -8
