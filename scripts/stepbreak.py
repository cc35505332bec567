"""Per-step kernel breakdown of the last N steps of a kernel_trace.csv:
python scripts/stepbreak.py TRACE.csv [N] [step-start-kernel-substring]."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
mark = sys.argv[3] if len(sys.argv) > 3 else 'conv1_fwd_kernel'
starts = [i for i, r in enumerate(rows) if mark in r['Kernel_Name']]
first = starts[-N]
sel = rows[first:]
t0 = int(sel[0]['Start_Timestamp'])
t1 = max(int(r['End_Timestamp']) for r in sel)
agg = collections.defaultdict(lambda: [0, 0.0])
busy = 0.0
for r in sel:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    name = r['Kernel_Name'].replace('(anonymous namespace)::', '')
    name = name.split('(')[0][:60]
    key = (name, r.get('Grid_Size_X', r.get('Grid_Size', '')))
    agg[key][0] += 1
    agg[key][1] += d
    busy += d
print(f'steps={N} wall/step={(t1 - t0) / 1e3 / N:.1f}us kernel-busy/step={busy / N:.1f}us launches/step={len(sel) / N:.1f}')
for (name, grid), (n, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f'{name:60s} grid={grid:>8s} n/step={n / N:5.1f} avg={tot / n:7.1f}us per-step={tot / N:7.1f}us')
