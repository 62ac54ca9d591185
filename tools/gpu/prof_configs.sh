# bench_configs (C2, C3, HET, HS) + a rocprofv3 kernel-stats pass over the same run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-cfg}
CFGS=${2:-C2,C3,HET,HS}
timeout -k 10 300 python tools/bench_configs.py --configs $CFGS > gpurun_out/bench_configs_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_configs_$TAG.log; exit 1; }
grep "{" gpurun_out/bench_configs_$TAG.log | cut -c1-260
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --configs $CFGS > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/kernel_stats_$TAG.csv
cut -d, -f1-8 gpurun_out/kernel_stats_$TAG.csv | cut -c1-220 | head -25
