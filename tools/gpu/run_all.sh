# tests + bench + kernel-trace profile + PMC passes, stopping at the first failure
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
bash tools/gpu/profile_bench.sh "$TAG" || exit $?
bash tools/gpu/pmc_bench.sh "$TAG" || exit $?
