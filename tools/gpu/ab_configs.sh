# Same-box A/B of two library builds on tools/bench_configs.py configs,
# alternating A B A B (A = the build at LIB_A, B = the tree's libpgw.so).
# usage: bash tools/gpu/ab_configs.sh TAG LIB_A CONFIGS
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1; LIBA=$2; CFG=$3
mkdir -p gpurun_out/ab
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export PGW_LIB_PATH=$GRAFT_REPO_ROOT/$LIBA; else unset PGW_LIB_PATH; fi
    timeout -k 10 300 python -u tools/bench_configs.py --configs "$CFG" --steps 286 > gpurun_out/ab/${TAG}_$v$r.log 2>&1 || exit $?
    echo "== $v$r"; grep -o '"config": "[A-Z0-9]*"\|"us_per_step": [0-9.]*' gpurun_out/ab/${TAG}_$v$r.log | paste - -
  done
done
