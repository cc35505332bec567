"""Critical-chain view of one wsj_c3 training step from a rocprofv3 kernel trace:
    python scripts/c3_timeline.py RUN_kernel_trace.csv [--step -2] [--all]
Splits the trace into steps at conv1_bwd (the step's last SDR-independent kernel),
prints per-class busy time (last layer = the J = 32 kernels, inner = J = 16) and the
last layer's launches with their start offsets, so gaps and serialised launches on
the last layer's chain show up directly."""
import argparse
import collections
import csv


def short(name):
    n = name.replace('void (anonymous namespace)::', '').replace('(anonymous namespace)::', '')
    if n.startswith('_ZN12_GLOBAL__N_1'):
        n = n[17:].lstrip('0123456789')
    return n.split('(')[0][:38]


def cls(r):
    k = r['k']
    grid = (int(r['Grid_Size_X']), int(r['Grid_Size_Y']), int(r['Grid_Size_Z']))
    if 'sdr_seq' in k or 'sdr_stream' in k:
        return 'last' if '<32, 32' in k else 'inner'
    if 'pose' in k:
        return 'last_pose' if grid[0] == 6144 else 'inner_pose'
    if 'gxw32' in k or 'sdr_gx' in k or 'sdr_gw' in k:
        return 'last_gxw' if grid[0] == 2048 else 'inner_gxw'
    return 'other'


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('trace')
    ap.add_argument('--step', type=int, default=-2, help='which step (python index over the steps found)')
    ap.add_argument('--all', action='store_true', help='list every SDR launch, not only the last layer')
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    for r in rows:
        r['s'], r['e'] = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        r['k'] = short(r['Kernel_Name'])
    rows.sort(key=lambda r: r['s'])
    marks = [r for r in rows if 'conv1_bwd' in r['Kernel_Name']]
    if len(marks) < 2:
        raise SystemExit('fewer than two training steps in the trace')
    i = a.step % (len(marks) - 1)
    t0, t1 = marks[i]['e'], marks[i + 1]['e']
    seg = [r for r in rows if t0 <= r['s'] < t1]
    print('step %d of %d: span %.2f ms' % (i, len(marks) - 1, (t1 - t0) / 1e6))
    busy, cnt = collections.defaultdict(float), collections.Counter()
    for r in seg:
        busy[cls(r)] += (r['e'] - r['s']) / 1e3
        cnt[cls(r)] += 1
    for c in sorted(busy):
        print('  %-11s %8.0f us  %4d launches' % (c, busy[c], cnt[c]))
    iv = sorted((r['s'], r['e']) for r in seg)
    tot, cs, ce = 0, None, 0
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    print('  union busy %.2f ms' % (tot / 1e6))
    for r in seg:
        c = cls(r)
        if a.all and c != 'other' or c.startswith('last'):
            print('%9.1f %7.1f  %-10s %-30s %dx%sx%s' % ((r['s'] - t0) / 1e3, (r['e'] - r['s']) / 1e3, c,
                                                      r['k'][:30], int(r['Grid_Size_X']), r['Grid_Size_Y'],
                                                      r['Grid_Size_Z']))


if __name__ == '__main__':
    main()
