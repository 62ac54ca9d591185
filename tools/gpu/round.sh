# The round's full GPU check: smoke + GPU suite + driver-shaped bench
# (suite.sh), then a rocprofv3 kernel-trace summary of the bench, the PMC
# passes (separate runs), and the other configs.  Stops at the first failure.
# Usage: bash tools/gpu/round.sh TAG [configs]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
CFG=${2:-C2,C3,HET,HETS,HETX,HS}
bash tools/gpu/suite.sh "$TAG" || exit $?
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 286 --warmup 20 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
find gpurun_out/prof/$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_$TAG.csv
head -12 gpurun_out/kernel_stats_$TAG.csv | cut -c1-160
rm -rf gpurun_out/prof/$TAG        # (the raw trace: over gpurun's 64 MiB copy-back)
bash tools/gpu/pmc_bench.sh "$TAG" || exit $?
python tools/gpu/pmc_summary.py "$TAG" > gpurun_out/pmc_$TAG.txt 2>&1 || true
python tools/gpu/pmc_traffic.py "$TAG" > gpurun_out/pmc_traffic_$TAG.txt 2>&1 && cp profiles/pmc_traffic.json gpurun_out/pmc_traffic_$TAG.json
rm -rf gpurun_out/pmc/$TAG
timeout -k 10 600 python -u tools/bench_configs.py --configs "$CFG" --steps 286 > gpurun_out/bench_configs_$TAG.log 2>&1 || exit $?
cat gpurun_out/bench_configs_$TAG.log | cut -c1-300
