"""HBM traffic per kernel dispatch from a scripts/r4_counters.sh STAGE=traffic run.

    python scripts/r4_traffic.py <tag> <cfg> [gpurun_out/r4ctr]
        -> profiles/<tag>_kernel_stats[_<cfg>].csv   (rocprofv3 --kernel-trace --stats, verbatim)
           profiles/<tag>_pmc[_<cfg>].json          (per kernel: avg_us, reads, writes)
(no suffix for cfg3: bench.py pmc_traffic's naming).

Read bytes = 32 x (TCC_EA0_RDREQ_DRAM_32B_sum + _GMI_32B_sum + _IO_32B_sum): the DRAM-side bytes
of the read requests, in 32-byte units.  Calibrated with scripts/micro/fetch_cal.hip
(profiles/r04_fetch_cal.json): exact for whole-line (128-B) reads of every access width, dword to
dwordx4 and LDS-DMA; a 64-B request (a 64-byte head slice of a longer row) counts as 128 B -- and
the 64-B slice kernels stream at half the rate of the 128-B slice kernel, so that is what such a
read costs.  FETCH_SIZE (TCC_EA0_RDREQ x 64 B) is half the bytes of whole-line reads and exactly
the requested bytes of 64-B ones, so no single factor corrects it.  Write bytes = WRITE_SIZE x 1024
(exact for every store width measured)."""
import collections
import csv
import glob
import json
import os
import shutil
import sys

RD = ('TCC_EA0_RDREQ_DRAM_32B_sum', 'TCC_EA0_RDREQ_GMI_32B_sum', 'TCC_EA0_RDREQ_IO_32B_sum')


def short(name):
    return name.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '').strip()


def find(src, sub, name):
    hits = glob.glob(os.path.join(src, sub, '**', '*' + name), recursive=True)
    return sorted(hits, key=os.path.getsize)[-1] if hits else None


def per_dispatch(path, names):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] in names:
            acc[(short(r['Kernel_Name']), r['Dispatch_Id'])][r['Counter_Name']] += float(r['Counter_Value'])
    out = collections.defaultdict(list)
    for (k, _), cs in acc.items():
        out[k].append(cs)
    return out


def main():
    tag, cfg = sys.argv[1], sys.argv[2]
    src = sys.argv[3] if len(sys.argv) > 3 else 'gpurun_out/r4ctr'
    sfx = '' if cfg == 'cfg3' else '_' + cfg
    os.makedirs('profiles', exist_ok=True)
    stats_csv = find(src, cfg + '_trace', 'kernel_stats.csv')
    shutil.copy(stats_csv, 'profiles/%s_kernel_stats%s.csv' % (tag, sfx))
    res = {short(r['Name']): dict(calls=int(r['Calls']), avg_us=float(r['AverageNs']) / 1e3, pct=float(r['Percentage']))
           for r in csv.DictReader(open(stats_csv))}
    rd = per_dispatch(find(src, cfg + '_rd', 'counter_collection.csv'), set(RD) | {'TCC_EA0_RDREQ_sum'})
    wr = per_dispatch(find(src, cfg + '_wr', 'counter_collection.csv'), {'WRITE_SIZE'})
    for k, ds in rd.items():
        e = res.setdefault(k, {})
        e['read_bytes_per_dispatch'] = 32 * sum(sum(d.get(c, 0.0) for c in RD) for d in ds) / len(ds)
        e['rdreq_per_dispatch'] = sum(d.get('TCC_EA0_RDREQ_sum', 0.0) for d in ds) / len(ds)
    for k, ds in wr.items():
        res.setdefault(k, {})['write_bytes_per_dispatch'] = 1024 * sum(d['WRITE_SIZE'] for d in ds) / len(ds)
    for k, e in res.items():
        if 'read_bytes_per_dispatch' in e and 'write_bytes_per_dispatch' in e:
            e['hbm_bytes_per_dispatch'] = e['read_bytes_per_dispatch'] + e['write_bytes_per_dispatch']
    meta = {'method': 'reads 32 x TCC_EA0_RDREQ_{DRAM,GMI,IO}_32B_sum, writes 1024 x WRITE_SIZE, per dispatch '
                      '(scripts/r4_traffic.py; calibration profiles/r04_fetch_cal.json)'}
    json.dump(dict(res, _meta=meta), open('profiles/%s_pmc%s.json' % (tag, sfx), 'w'), indent=1, sort_keys=True)
    for k, e in sorted(res.items(), key=lambda kv: -kv[1].get('pct', 0))[:14]:
        print('%-26s %8.2f us %6.2f%%  traffic %s' % (k[:26], e.get('avg_us', 0), e.get('pct', 0),
                                                     '%.2f MB' % (e['hbm_bytes_per_dispatch'] / 1e6)
                                                     if 'hbm_bytes_per_dispatch' in e else '-'))


if __name__ == '__main__':
    main()
