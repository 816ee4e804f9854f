"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel name, mean of each counter."""
import csv, sys, collections, glob
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        name = r.get('Kernel_Name') or r.get('Kernel-Name') or r.get('KernelName')
        agg[name[:60]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in agg.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f'   {c:32s} {sum(v)/len(v):16.1f}  (n={len(v)})')
