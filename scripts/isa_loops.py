"""Summarise the loops of one kernel in a hipcc -S listing: instruction mix and s_waitcnt values of
every backward-branch body with MFMAs and vector loads (development aid).

    hipcc -O3 --offload-arch=gfx950 -I include --cuda-device-only -S gemm.hip -o /tmp/gemm.s
    python scripts/isa_loops.py /tmp/gemm.s k_wgrad
"""
import re
import sys


def main(path, kernel):
    L = open(path).read().split('\n')
    st = [i for i, l in enumerate(L) if re.match(r'^_Z\S*%s\S*:' % kernel, l)][0]
    en = [i for i, l in enumerate(L) if i > st and 's_endpgm' in l][0]
    L = L[st:en]
    labels = {}
    for i, l in enumerate(L):
        m = re.match(r'^(\.LBB\d+_\d+):', l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(L):
        m = re.search(r's_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)', l)
        if not (m and m.group(2) in labels and labels[m.group(2)] < i):
            continue
        body = L[labels[m.group(2)]:i + 1]
        cnt = {}
        for b in body:
            b = b.strip()
            if not b or b.startswith(';') or b.startswith('.'):
                continue
            op = b.split()[0]
            if 'mfma' in op:
                k = 'mfma'
            elif op.startswith('global_load') or op.startswith('buffer_load'):
                k = 'vload'
            elif 'waitcnt' in op:
                k = 'waitcnt'
            elif op.startswith('v_'):
                k = 'valu'
            elif op.startswith('s_'):
                k = 'salu'
            elif op.startswith('ds_'):
                k = 'ds'
            else:
                k = op
            cnt[k] = cnt.get(k, 0) + 1
        if cnt.get('mfma', 0) >= 12 and cnt.get('vload', 0) > 6:
            print(m.group(2), len(body), cnt, [b.strip() for b in body if 'waitcnt' in b][:10])


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
