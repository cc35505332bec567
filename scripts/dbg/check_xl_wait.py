"""Check the x_dma waits of the pipelined passes against their ISA: between each
in-loop global_load_lds (x_dma) and the barrier that publishes it, the last
's_waitcnt vmcnt(K)' (xl_wait) must leave at most as many loads in flight as the wave
issued after the DMA (else the wait lets the DMA still be in flight).
    python scripts/dbg/check_xl_wait.py ISA.s"""
import re
import sys

s = open(sys.argv[1]).read()
bad = 0
for name in re.findall(r'^(_Z\w*route_(?:fwd|bwd)32p_kernelILi32ELi32E\w*):', s, re.M):
    body = s[s.index(name + ':'):]
    body = body[:body.index('.Lfunc_end')]
    lines = [l.strip() for l in body.split('\n') if l.startswith('\t') and not l.strip().startswith(';')]
    for k, l in enumerate(lines):
        if not l.startswith('global_load_lds'):
            continue
        n, last = 0, None
        for l2 in lines[k + 1:]:
            m = re.match(r's_waitcnt vmcnt\((\d+)\)$', l2)
            if m:
                last = (n, int(m.group(1)))
            if l2.startswith('s_barrier'):
                break
            if re.match(r'(buffer|global)_(load|store|atomic)', l2):
                n += 1
        if last is None:
            print(f'{name[:64]} dma@{k}: no wait before the barrier')
            bad += 1
        elif last[1] > last[0]:
            print(f'{name[:64]} dma@{k}: vmcnt({last[1]}) with {last[0]} loads after the DMA: TOO FEW')
            bad += 1
        else:
            print(f'{name[:64]} dma@{k}: vmcnt({last[1]}), {last[0]} loads after the DMA: ok')
sys.exit(1 if bad else 0)
