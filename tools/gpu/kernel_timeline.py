"""Per-step timeline of the C4 kernels from a rocprofv3 --kernel-trace CSV:
for consecutive (agents, PF) launches, the PF's start relative to the agents'
end and the next agents' start relative to the PF's start (overlap), and the
mean step period.  Usage: python tools/gpu/kernel_timeline.py <kernel_trace.csv>"""
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
ks = []
for r in rows:
    nm = r["Kernel_Name"]
    kind = "A" if "k_coord_agents" in nm else "P" if ("k_coord_pf" in nm) else None
    if kind:
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind))
ks.sort()
A = [k for k in ks if k[2] == "A"]
P = [k for k in ks if k[2] == "P"]
n = min(len(A), len(P))
A, P = A[-n:], P[-n:]
gap = [(P[i][0] - A[i][1]) / 1e3 for i in range(n)]                 # PF start - its agents' end
ovl = [(min(P[i][1], A[i + 1][1]) - max(P[i][0], A[i + 1][0])) / 1e3 for i in range(n - 1)]
per = [(A[i + 1][0] - A[i][0]) / 1e3 for i in range(n - 1)]
dur_a = [(a[1] - a[0]) / 1e3 for a in A]
dur_p = [(p[1] - p[0]) / 1e3 for p in P]
print("steps %d  period median %.2f us  agents %.2f us  PF %.2f us  PF start after its agents %.2f us  "
      "PF(t) / agents(t+1) overlap %.2f us (median)" % (n, statistics.median(per), statistics.median(dur_a),
                                                        statistics.median(dur_p), statistics.median(gap),
                                                        statistics.median(ovl)))
