# Same-box A/B of two od_probe.py argument sets on one library build, per step
# class (tools/gpu/od_step_classes.py): rocprofv3 kernel traces of
# od_probe.py --hist, alternating A B A B.
# usage: bash tools/gpu/ab_args.sh TAG "ARGS_A" "ARGS_B" [HIST]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; ARGA=$2; ARGB=$3; H=${4:-572}
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then X=$ARGA; else X=$ARGB; fi
    d=gpurun_out/aba/$TAG/$v$r; mkdir -p $d
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$d -o run -- python3 $GRAFT_REPO_ROOT/tools/gpu/od_probe.py --modes opendss --steps 20 --hist $H $X > $GRAFT_REPO_ROOT/$d.log 2>&1) || exit $?
    echo "== $v$r ($X)"; python tools/gpu/od_step_classes.py $d/run_kernel_trace.csv $d.log || exit $?
  done
done
