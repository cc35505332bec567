"""Average PMC counters per (kernel, grid, workgroup, LDS) over dispatches and passes.

    python scripts/pmcsum.py DIR [name-filter] [--json OUT]

DIR holds p*/run_counter_collection.csv from separate rocprofv3 --pmc passes.
FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3; the gfx950 correction of
MI355X_MICROARCH.md (FETCH_SIZE counts wide streaming reads at half their bytes)
is applied by the consumer (bench.py / DESIGN.md), not here.
"""
import collections
import csv
import glob
import json
import re
import sys

argv = sys.argv[1:]
if '--json' in argv:   # the option's value is not a positional argument
    del argv[argv.index('--json') + 1]
args = [a for a in argv if not a.startswith('--')]
d = args[0]
flt = args[1] if len(args) > 1 else ''
out = sys.argv[sys.argv.index('--json') + 1] if '--json' in sys.argv else None
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in sorted(glob.glob(d + '/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name']
        if flt not in name:
            continue
        key = (re.sub(r'\(anonymous namespace\)::', '', name).split('(')[0], r['Grid_Size'], r['Workgroup_Size'], r['LDS_Block_Size'])
        vals[key][r['Counter_Name']].append(float(r['Counter_Value']))
        durs[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
res = []
for k, cs in vals.items():
    row = {'kernel': k[0], 'grid': int(k[1]), 'wg': int(k[2]), 'lds': int(k[3]),
           'avg_us_under_pmc': sum(durs[k]) / len(durs[k])}
    print(k)
    for c, v in sorted(cs.items()):
        print(f'    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})')
        row[c] = sum(v) / len(v)
    res.append(row)
if out:
    json.dump(res, open(out, 'w'), indent=1)
