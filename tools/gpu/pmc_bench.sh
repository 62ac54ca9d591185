# PMC counter passes (each its own rocprofv3 run, --pmc only) over a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-pmc}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
run_pass() {
  name=$1; shift
  cd /tmp && timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$TAG/$name" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-variants > "$GRAFT_REPO_ROOT/gpurun_out/pmc/${TAG}_$name.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
run_pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS || exit $?
run_pass p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_THREAD_CYCLES_VALU || exit $?
run_pass p3 FETCH_SIZE || exit $?
run_pass p4 WRITE_SIZE || exit $?
echo pmc-done
