"""FETCH_SIZE / WRITE_SIZE calibration table from scripts/r4_counters.sh STAGE=cal.

    python scripts/fetch_cal.py [gpurun_out/r4ctr] [profiles/r04_fetch_cal.json]

scripts/micro/fetch_cal reads / writes a KNOWN number of bytes per dispatch with one access shape
per kernel (dword, dwordx2, dwordx4, 2-byte, LDS-DMA 4 / 16 B, k_wgrad's two 128-byte row segments,
the attention's 64-byte head slices of 384 / 512-byte rows, 64-byte row stores).  Per shape this
writes counter bytes / known bytes:
  fetch_factor  = known / (FETCH_SIZE KB * 1024)   (what FETCH_SIZE must be multiplied by)
  write_factor  = known / (WRITE_SIZE KB * 1024)
  rdreq_bytes   = known / TCC_EA0_RDREQ_sum        (bytes per memory-side read request)
bench.py's traffic field uses fetch_factor of the shape each kernel's dominant loads have
(bench.FETCH_SHAPE)."""
import collections
import csv
import glob
import json
import os
import sys


def counters(path, names):
    """{kernel: {counter: mean per dispatch}} from a rocprofv3 counter_collection.csv"""
    hits = glob.glob(os.path.join(path, '**', '*counter_collection.csv'), recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in hits:
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] not in names:
                continue
            k = r['Kernel_Name'].split('(')[0].replace('void ', '').strip()
            d = acc[k][r['Counter_Name']]
            d[r['Dispatch_Id']] = d.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/r4ctr'
    dst = sys.argv[2] if len(sys.argv) > 2 else 'profiles/r04_fetch_cal.json'
    known = {}
    for line in open(os.path.join(src, 'cal_plain.log')):
        line = line.strip()
        if line.startswith('{'):
            d = json.loads(line)
            known[d['kernel']] = d
    fetch = counters(os.path.join(src, 'cal_fetch'), {'FETCH_SIZE'})
    write = counters(os.path.join(src, 'cal_write'), {'WRITE_SIZE'})
    req = counters(os.path.join(src, 'cal_req'), {'TCC_EA0_RDREQ_sum', 'TCC_EA0_RDREQ_32B_sum',
                                                  'TCC_EA0_WRREQ_sum', 'TCC_EA0_WRREQ_64B_sum'})
    rd32 = ('TCC_EA0_RDREQ_DRAM_32B_sum', 'TCC_EA0_RDREQ_GMI_32B_sum', 'TCC_EA0_RDREQ_IO_32B_sum')
    req2 = counters(os.path.join(src, 'cal_req2'), set(rd32)) if os.path.isdir(os.path.join(src, 'cal_req2')) else {}

    def find(tab, name):
        # rocprof kernel names carry the template arguments: k_rd<4> -> "k_rd<4>" or "void k_rd<4>"
        base = name.replace(' ', '')
        for k, v in tab.items():
            if k.replace(' ', '').replace('(anonymousnamespace)::', '').endswith(base):
                return v
        return {}
    out = {'source': 'scripts/micro/fetch_cal.hip via scripts/r4_counters.sh STAGE=cal', 'kernels': {}}
    for name, kd in known.items():
        e = dict(bytes=kd['bytes'], us=kd['us'], TBps=kd['TBps'])
        f, w, q = find(fetch, name), find(write, name), find(req, name)
        if f.get('FETCH_SIZE') and not name.startswith('k_wr'):     # store kernels read ~nothing
            e['fetch_kb'] = f['FETCH_SIZE']
            e['fetch_factor'] = round(kd['bytes'] / (1024 * f['FETCH_SIZE']), 4)
        if w.get('WRITE_SIZE'):
            e['write_kb'] = w['WRITE_SIZE']
            e['write_factor'] = round(kd['bytes'] / (1024 * w['WRITE_SIZE']), 4)
        for c in ('TCC_EA0_RDREQ_sum', 'TCC_EA0_RDREQ_32B_sum', 'TCC_EA0_WRREQ_sum', 'TCC_EA0_WRREQ_64B_sum'):
            if c in q:
                e[c] = q[c]
        if q.get('TCC_EA0_RDREQ_sum') and not name.startswith('k_wr'):
            e['bytes_per_rdreq'] = round(kd['bytes'] / q['TCC_EA0_RDREQ_sum'], 2)
        q2 = find(req2, name)
        if q2:
            units = sum(q2.get(c, 0.0) for c in rd32)
            e.update({c: q2[c] for c in rd32 if c in q2})
            if units and not name.startswith('k_wr'):
                e['rd32_factor'] = round(kd['bytes'] / (32 * units), 4)   # 1.0: 32 x units is exact
        out['kernels'][name] = e
    json.dump(out, open(dst, 'w'), indent=1)
    for k, e in out['kernels'].items():
        print('%-22s %6.3f TB/s  fetch x%-7s write x%-7s B/rdreq %-7s 32B-units x%s' % (
            k, e['TBps'], e.get('fetch_factor', '-'), e.get('write_factor', '-'), e.get('bytes_per_rdreq', '-'),
            e.get('rd32_factor', '-')))


if __name__ == '__main__':
    main()
