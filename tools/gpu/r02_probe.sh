# PF phase traces (split and one-lane kernels) and host time of the first steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-probe}
timeout -k 10 120 python tools/gpu/pf_trace.py > gpurun_out/pf_trace_split_$TAG.txt 2>&1 || { tail -20 gpurun_out/pf_trace_split_$TAG.txt; exit 1; }
PGW_PF_SPLIT=0 timeout -k 10 120 python tools/gpu/pf_trace.py > gpurun_out/pf_trace_onelane_$TAG.txt 2>&1 || { tail -20 gpurun_out/pf_trace_onelane_$TAG.txt; exit 1; }
timeout -k 10 120 python tools/gpu/host_cold.py > gpurun_out/host_cold_$TAG.txt 2>&1 || { tail -20 gpurun_out/host_cold_$TAG.txt; exit 1; }
cat gpurun_out/pf_trace_split_$TAG.txt gpurun_out/pf_trace_onelane_$TAG.txt
grep "us per step\|construct" gpurun_out/host_cold_$TAG.txt
