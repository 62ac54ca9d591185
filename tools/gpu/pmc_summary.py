"""Summarise rocprofv3 --pmc passes per kernel (mean over dispatches)."""
import collections, csv, glob, sys
tag = sys.argv[1]
for p in sorted(glob.glob('gpurun_out/pmc/%s/*' % tag)):
    f = glob.glob(p + '/*counter_collection.csv')
    if not f:
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r['Kernel_Name']
        if 'pgw' not in k:
            continue
        agg[k.split('(')[0][-28:]][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, d in agg.items():
        print(p.split('/')[-1], k, {c: round(sum(v) / len(v)) for c, v in d.items()})
