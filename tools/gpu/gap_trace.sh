# Kernel-trace timeline of the bench (headline + variants): idle gaps between dispatches.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-gap}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof/$TAG -name "*kernel_trace.csv" | head -1)
python tools/gpu/gap_trace.py "$f" | tee gpurun_out/gaps_$TAG.txt
