"""Per-kernel register / LDS / occupancy summary of one csrc/*.hip file (compiler remarks).
usage: python scripts/resusage.py attn.hip [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '-fPIC', '--offload-arch=gfx950', '-mllvm',
       '-disable-promote-alloca-to-lds', '-I../../include', '-c', src, '-o', '/tmp/_ru.o',
       '-Rpass-analysis=kernel-resource-usage'] + sys.argv[2:]
out = subprocess.run(cmd, cwd='multimodal-emotion-processing_amd/csrc', capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r'remark: (.*?): (.*) \[-Rpass', line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == 'Function Name':
        cur = {'name': subprocess.run(['c++filt', v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    print('%-90s vgpr %4s agpr %3s spill %3s occ %2s lds %6s' % (
        r['name'][:90], r.get('VGPRs'), r.get('AGPRs'), r.get('VGPRs Spill'),
        r.get('Occupancy [waves/SIMD]'), r.get('LDS Size [bytes/block]')))
