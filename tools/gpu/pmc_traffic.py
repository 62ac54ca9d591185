"""profiles/pmc_traffic.json from a pmc_bench.sh run: HBM-side bytes per launch
of each timed kernel = (2 x FETCH_SIZE + WRITE_SIZE) KB, mean over dispatches.
FETCH_SIZE x2: on gfx950 it reports half the bytes of a coalesced streaming
read (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for streaming
stores.  Usage: python tools/gpu/pmc_traffic.py TAG"""
import csv
import glob
import json
import os
import sys

NAMES = {"k_coord_agents_std": "k_coord_agents_std",
         "k_coord_pf_od<14": "k_coord_pf_od<14>",
         "k_coord_pf<14, true, false, false": "k_coord_pf<14,true,false,false>",
         "k_coord_pf_split": "k_coord_pf_split",
         "k_coord_step_od": "k_coord_step_od",
         "k_pf_solve<14, true, false, false>": "k_pf_solve<14,true,false,false>"}


def per_kernel(path, counter):
    vals = {}
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            for frag, key in NAMES.items():
                if frag in r["Kernel_Name"]:
                    vals.setdefault(key, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    tag = sys.argv[1]
    base = os.path.join("gpurun_out", "pmc", tag)
    fetch = per_kernel(os.path.join(base, "p3"), "FETCH_SIZE")
    write = per_kernel(os.path.join(base, "p4"), "WRITE_SIZE")
    path = os.path.join("profiles", "pmc_traffic.json")
    old = json.load(open(path)) if os.path.exists(path) else {}
    runs = dict(old.get("runs", {}))
    for k in old.get("bytes_per_launch", {}):             # kernels this run did not launch keep theirs
        runs.setdefault(k, old.get("source", "").split()[-1])
    for k in fetch:
        runs[k] = tag
    bpl = dict(old.get("bytes_per_launch", {}))
    bpl.update({k: (2 * fetch[k] + write.get(k, 0.0)) * 1024 for k in fetch})
    fk = dict(old.get("fetch_kb", {}))
    fk.update(fetch)
    wk = dict(old.get("write_kb", {}))
    wk.update(write)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), run per kernel in `runs`",
           "formula": "(2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes, mean per dispatch",
           "runs": runs, "bytes_per_launch": bpl, "fetch_kb": fk, "write_kb": wk}
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["bytes_per_launch"]))


if __name__ == "__main__":
    main()
