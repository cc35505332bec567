"""Register/scratch/occupancy summary of a HIP source: python scripts/kres.py FILE.hip [filter]."""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
out = subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '--offload-arch=gfx950', '-std=c++17', '-fPIC', '-munsafe-fp-atomics',
                      '-c', src, '-o', '/tmp/_kres.o', '-Rpass-analysis=kernel-resource-usage'],
                     capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r'remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)', line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k[:90]:90s} V={v.get('VGPRs')} A={v.get('AGPRs')} scr={v.get('ScratchSize')} occ={v.get('Occupancy')} lds={v.get('LDS')}")
