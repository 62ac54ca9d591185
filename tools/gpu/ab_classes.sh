# Same-box A/B of two library builds on the OpenDSS-rule C4 step, per step
# class (tools/gpu/od_step_classes.py): rocprofv3 kernel traces of
# od_probe.py --hist, alternating A B A B.
# usage: bash tools/gpu/ab_classes.sh TAG LIB_A [HIST]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; LIBA=$2; H=${3:-572}
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export PGW_LIB_PATH=$GRAFT_REPO_ROOT/$LIBA; else unset PGW_LIB_PATH; fi
    d=gpurun_out/abc/$TAG/$v$r; mkdir -p $d
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 $GRAFT_REPO_ROOT/tools/gpu/od_probe.py --modes opendss --steps 20 --hist $H > $GRAFT_REPO_ROOT/$d.log 2>&1) || exit $?
    echo "== $v$r"; python tools/gpu/od_step_classes.py $d/run_kernel_trace.csv $d.log || exit $?
  done
done
