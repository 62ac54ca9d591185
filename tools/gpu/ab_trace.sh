# Same-box A/B of two library builds (PGW_LIB_PATH) on the C4 step: rocprofv3
# kernel traces of tools/gpu/overlap_probe.py (synchronous step, one mode),
# alternating A B A B, each summarised by tools/gpu/kernel_timeline.py.
# usage: bash tools/gpu/ab_trace.sh TAG LIB_A MODE [STEPS]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; LIBA=$2; MODE=${3:-opendss}; STEPS=${4:-286}
mkdir -p gpurun_out/ab/$TAG
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export PGW_LIB_PATH=$GRAFT_REPO_ROOT/$LIBA; else unset PGW_LIB_PATH; fi
    d=gpurun_out/ab/$TAG/$v$r
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 $GRAFT_REPO_ROOT/tools/gpu/overlap_probe.py --modes $MODE --overlap 0 --steps $STEPS --no-timing > $GRAFT_REPO_ROOT/$d.log 2>&1) || exit $?
    echo "$v$r $(python tools/gpu/kernel_timeline.py $d/run_kernel_trace.csv)"
  done
done
