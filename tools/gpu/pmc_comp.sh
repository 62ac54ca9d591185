# PMC passes (each its own rocprofv3 run, --pmc only) over a python workload:
# where the component kernels' waves spend their cycles.
# usage: bash tools/gpu/pmc_comp.sh TAG script.py [args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=$1; shift
run_pass() {
  name=$1; shift
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $1 --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$TAG/$name" -o run -- python3 "$GRAFT_REPO_ROOT/$SCRIPT" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/pmc/${TAG}_$name.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
SCRIPT=$1; shift; ARGS="$*"
run_pass p1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA" || exit $?
run_pass p2 "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS" || exit $?
python tools/gpu/pmc_summary.py $TAG
