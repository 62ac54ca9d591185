"""Per-step k_coord_pf_od durations (rocprofv3 kernel trace) by the step's
(min, max) iteration counts (od_probe.py --hist sequence): which steps cost
what.  Usage: python tools/gpu/od_step_classes.py <kernel_trace.csv> <od_probe log>"""
import collections
import csv
import statistics
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_coord_pf_od" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
seq, early = None, None
for line in open(sys.argv[2]):
    if "in order:" in line:
        seq = line.split("in order:")[1].split()
    if "in one wave:" in line:
        early = [tuple(int(x) for x in w.split("/")) for w in line.split("in one wave:")[1].split()]
assert seq, "no --hist sequence in the log"
tail = d[-len(seq):]                       # the --hist steps are the last launches
cls = collections.defaultdict(list)
for c, t in zip(seq, tail):
    cls[c].append(t)
for c in sorted(cls):
    v = cls[c]
    print("iterations (min,max)=(%s,%s)  steps %4d  PF median %.2f us  mean %.2f  min %.2f  max %.2f"
          % (c[0], c[1], len(v), statistics.median(v), statistics.mean(v), min(v), max(v)))
if early:                                  # mixed steps by the most early-stopping envs in one wave
    sub = collections.defaultdict(list)
    for c, (nw, mx), t in zip(seq, early, tail):
        if c[0] != c[1]:
            b = "1" if mx <= 1 else "2-4" if mx <= 4 else "5-12" if mx <= 12 else "13+"
            sub[(c, b)].append((t, nw))
    for (c, b) in sorted(sub):
        v = [t for t, _ in sub[(c, b)]]
        print("  (%s,%s) most early envs per wave %-4s steps %4d  PF median %.2f us  mean %.2f  waves with one "
              "(median) %d" % (c[0], c[1], b, len(v), statistics.median(v), statistics.mean(v),
                               statistics.median([n for _, n in sub[(c, b)]])))
