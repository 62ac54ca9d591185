"""Idle gaps between consecutive kernel dispatches in a rocprofv3 kernel trace
(kernel_trace.csv): per kernel-name pair, the median / p90 gap (us) and the
median dispatch duration -- is a step GPU-bound or waiting for the host?"""
import csv
import statistics as st
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda s: s.split("(")[0].replace("void ", "").replace("pgw::", "")[:40]
pairs, durs = {}, {}
for a, b in zip(rows, rows[1:]):
    g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
    pairs.setdefault((short(a["Kernel_Name"]), short(b["Kernel_Name"])), []).append(g)
for r in rows:
    durs.setdefault(short(r["Kernel_Name"]), []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("%-42s %6s %9s" % ("kernel", "calls", "med us"))
for k, v in sorted(durs.items(), key=lambda kv: -len(kv[1]))[:12]:
    print("%-42s %6d %9.2f" % (k, len(v), st.median(v)))
print("\n%-42s -> %-42s %6s %8s %8s" % ("prev", "next", "count", "med gap", "p90 gap"))
for (a, b), v in sorted(pairs.items(), key=lambda kv: -len(kv[1]))[:14]:
    v.sort()
    print("%-42s -> %-42s %6d %8.2f %8.2f" % (a, b, len(v), st.median(v), v[int(0.9 * (len(v) - 1))]))
