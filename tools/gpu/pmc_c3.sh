# PMC passes (each its own rocprofv3 run, --pmc only) over the C3 config bench
# (or the configs named second, e.g. C3,HET): where k_mc_step's (k_ma_step's)
# waves spend their cycles, and (passes p3 / p4) their HBM bytes.
# Usage: bash tools/gpu/pmc_c3.sh TAG [configs] [passes, default p1,p2]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-c3}
CFGS=${2:-C3}
PASSES=${3:-p1,p2}
run_pass() {
  name=$1; shift
  cd /tmp && timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$TAG/$name" -o run -- python3 "$GRAFT_REPO_ROOT/tools/bench_configs.py" --configs "$CFGS" --steps 100 --warmup 5 > "$GRAFT_REPO_ROOT/gpurun_out/pmc/${TAG}_$name.log" 2>&1
  rc=$?; cd "$GRAFT_REPO_ROOT"; return $rc
}
want() { case ",$PASSES," in *",$1,"*) return 0;; esac; return 1; }
want p1 && { run_pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA || exit $?; }
want p2 && { run_pass p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_WAIT_INST_LDS || exit $?; }
want p3 && { run_pass p3 FETCH_SIZE || exit $?; }
want p4 && { run_pass p4 WRITE_SIZE || exit $?; }
python tools/gpu/pmc_summary.py $TAG
