"""Summarise a rocprofv3 kernel_stats.csv per training step: python scripts/kstats.py CSV [steps]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 13.0
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{r['Name'][:64]:64s} calls/step={int(r['Calls']) / steps:5.1f} avg={float(r['AverageNs']) / 1e3:8.1f}us "
          f"per-step={float(r['TotalDurationNs']) / steps / 1e3:8.1f}us")
print(f'total per step {tot / steps / 1e3:.1f} us, launches/step {sum(int(r["Calls"]) for r in rows) / steps:.1f}')
