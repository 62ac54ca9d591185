# Nontemporal action loads in k_coord_agents_std (libpgw_actnt.so) vs plain
# loads: long benches alternated, each twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
cp powergridworld_amd/libpgw.so gpurun_out/libpgw_plain.so
for rep in 1 2; do
  for v in plain actnt; do
    if [ $v = actnt ]; then cp powergridworld_amd/libpgw_actnt.so powergridworld_amd/libpgw.so; else cp gpurun_out/libpgw_plain.so powergridworld_amd/libpgw.so; fi
    timeout -k 10 200 python bench.py --steps 572 --warmup 30 --no-cpu-baseline --no-variants > gpurun_out/bnt_${v}_$rep.log 2>&1 || { tail -20 gpurun_out/bnt_${v}_$rep.log; exit 1; }
    python - gpurun_out/bnt_${v}_$rep.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], "%.3e" % d["value"], "%.2f us/step" % (d["ms_per_step"] * 1e3),
      {k: round(v["avg_us"], 2) for k, v in d["kernels"].items()}, "copy %.0f" % d["stream_copy_gbs"])
PY
  done
done
cp gpurun_out/libpgw_plain.so powergridworld_amd/libpgw.so
rm -f gpurun_out/libpgw_plain.so
