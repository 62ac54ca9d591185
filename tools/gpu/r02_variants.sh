# A/B of libpgw builds (powergridworld_amd/libpgw_<V>.so) on the long C4 bench,
# each run twice, interleaved with the default build.  Usage: r02_variants.sh V1 V2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cp powergridworld_amd/libpgw.so gpurun_out/libpgw_base.so
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then cp gpurun_out/libpgw_base.so powergridworld_amd/libpgw.so; else cp powergridworld_amd/libpgw_$v.so powergridworld_amd/libpgw.so; fi
    timeout -k 10 200 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/bv_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/bv_${v}_$rep.log; cp gpurun_out/libpgw_base.so powergridworld_amd/libpgw.so; exit 1; }
    python - gpurun_out/bv_${v}_$rep.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()})
PY
  done
done
cp gpurun_out/libpgw_base.so powergridworld_amd/libpgw.so
rm -f gpurun_out/libpgw_base.so
