"""Per (kernel, grid) average durations from a rocprofv3 kernel_trace.csv: python scripts/ktrace.py CSV [filter]."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ''
agg = collections.defaultdict(list)
for r in rows:
    name = r['Kernel_Name']
    if flt not in name:
        continue
    key = (name[:70], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Workgroup_Size_X', ''), r.get('LDS_Block_Size', r.get('Lds_Size', '')))
    agg[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f'{k[0]:70s} grid={k[1]:>8s} wg={k[2]:>5s} lds={k[3]:>6s} n={len(v):4d} avg={sum(v) / len(v):8.1f}us')
