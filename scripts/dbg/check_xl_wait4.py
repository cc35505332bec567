"""Check the x_dma waits of the four-row-tile passes (route_fwd32_kernel /
route_bwd32_kernel <32,32,NW,4>) against their ISA.  There the DMA of capsule i + 2 is
issued after capsule i's barrier and waited for (xl_wait) before capsule i + 1's, so the
walk from each in-loop global_load_lds to the next s_barrier wraps around the loop's
back edge: the last 's_waitcnt vmcnt(K)' on that walk must leave at most as many
vector-memory operations in flight as the wave issued after the DMA.
    python scripts/dbg/check_xl_wait4.py ISA.s"""
import re
import sys

s = open(sys.argv[1]).read()
bad = 0
for name in re.findall(r'^(_Z\w*route_(?:fwd|bwd)32_kernelILi32ELi32ELi[248]ELi4E\w*):', s, re.M):
    body = s[s.index(name + ':'):]
    body = body[:body.index('.Lfunc_end')]
    raw = body.split('\n')
    hdr = [k for k, l in enumerate(raw) if 'Loop Header' in l and 'Depth=1' in l]
    lab = raw[hdr[0]].split(':')[0]
    ends = [k for k, l in enumerate(raw) if 'branch' in l and l.strip().endswith(lab)]
    lo, hi = min(hdr + ends), max(hdr + ends)
    lines = [l.strip() for l in raw[lo:hi + 1] if l.startswith('\t') and not l.strip().startswith(';')]
    for k, l in enumerate(lines):
        if not l.startswith('global_load_lds'):
            continue
        n, last = 0, None
        for step in range(1, len(lines)):
            l2 = lines[(k + step) % len(lines)]
            m = re.match(r's_waitcnt vmcnt\((\d+)\)$', l2)
            if m:
                last = (n, int(m.group(1)))
            if l2.startswith('s_barrier'):
                break
            if re.match(r'(buffer|global)_(load|store|atomic)', l2) and not l2.startswith('global_load_lds'):
                n += 1
        tag = f'{name[:70]} dma@{k}'
        if last is None:
            print(f'{tag}: no wait before the barrier')
            bad += 1
        elif last[1] > last[0]:
            print(f'{tag}: vmcnt({last[1]}) with {last[0]} operations after the DMA: TOO FEW')
            bad += 1
        else:
            print(f'{tag}: vmcnt({last[1]}), {last[0]} operations after the DMA: ok')
sys.exit(1 if bad else 0)
