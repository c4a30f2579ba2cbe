"""Summarise a rocprofv3 run (scripts/session.sh prof / traffic stages) into profiles/<tag>_*.

  python scripts/parse_prof.py <tag> [gpurun_out/prof_<workload>] [<workload>: cfg3 | cfg5 | cfg5_bf16 | ...]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats output, verbatim) and
profiles/<tag>_pmc.json: per kernel, the average dispatch duration (kernel trace) and the
average FETCH_SIZE / WRITE_SIZE per dispatch from the separate PMC passes, with HBM traffic
per dispatch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes (gfx950: FETCH_SIZE counts half the
bytes of a wide coalesced read -- MI355X_MICROARCH.md section HBM; the x2 is exact only for
16-byte-per-lane streams, other widths are uncalibrated).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def short(name):
    return name.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out/prof'
    # workload suffix (bench.py pmc_traffic): none for cfg3 fp32, else _<config>[_bf16]
    sfx = '_' + sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != 'cfg3' else ''
    # rocprofv3 -d <dir> -o run writes <dir>/<host>/<pid>_run_*.csv in some versions: find the files
    def find(sub, name):
        hits = glob.glob(os.path.join(src, sub, '**', '*' + name), recursive=True)
        return sorted(hits, key=os.path.getsize)[-1] if hits else os.path.join(src, sub, 'run_' + name)
    os.makedirs('profiles', exist_ok=True)
    shutil.copy(find('trace', 'kernel_stats.csv'), 'profiles/%s_kernel_stats%s.csv' % (tag, sfx))
    stats = {short(r['Name']): dict(calls=int(r['Calls']), avg_us=float(r['AverageNs']) / 1e3,
                                    pct=float(r['Percentage']))
             for r in csv.DictReader(open(find('trace', 'kernel_stats.csv')))}
    for ctr, sub in (('FETCH_SIZE', 'fetch'), ('WRITE_SIZE', 'write')):
        path = find(sub, 'counter_collection.csv')
        if not os.path.exists(path):
            continue
        acc = defaultdict(list)
        for r in csv.DictReader(open(path)):
            if r['Counter_Name'] == ctr:
                acc[short(r['Kernel_Name'])].append(float(r['Counter_Value']))
        for k, v in acc.items():
            stats.setdefault(k, {})[ctr.lower() + '_kb'] = sum(v) / len(v)
    for k, s in stats.items():
        if 'fetch_size_kb' in s and 'write_size_kb' in s:
            s['hbm_bytes_per_dispatch'] = (2 * s['fetch_size_kb'] + s['write_size_kb']) * 1024
    json.dump(stats, open('profiles/%s_pmc%s.json' % (tag, sfx), 'w'), indent=1, sort_keys=True)
    for k, s in sorted(stats.items(), key=lambda kv: -kv[1].get('pct', 0))[:16]:
        print('%-22s %8.2f us  %6.2f%%  traffic %s' % (k, s.get('avg_us', 0), s.get('pct', 0),
                                                     '%.2f MB' % (s['hbm_bytes_per_dispatch'] / 1e6)
                                                     if 'hbm_bytes_per_dispatch' in s else '-'))


if __name__ == '__main__':
    main()
