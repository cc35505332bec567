"""Average PMC counters per kernel over passes: python scripts/pmcsum.py DIR [filter]."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(d + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name']
        if flt not in name:
            continue
        key = (name[:60], r.get('Grid_Size', ''))
        vals[key][r['Counter_Name']].append(float(r['Counter_Value']))
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f'    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})')
