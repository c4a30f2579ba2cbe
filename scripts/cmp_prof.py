"""Compare a bench line's per-launch times with the rocprofv3 kernel trace of the same command.

    python scripts/cmp_prof.py <bench log (JSON line last)> <rocprofv3 -d dir> [--bf16]

rocprofv3 averages are taken over the timed step's own dispatches (the graph replays and the
eager timing steps alike), grouped by the launch -> kernel-symbol map of bench.KERNEL_OF."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main():
    log, d = sys.argv[1], sys.argv[2]
    line = json.loads([x for x in open(log).read().splitlines() if x.startswith('{')][-1])
    rows = list(csv.DictReader(open(glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True)[0])))
    stats = {}
    for r in rows:
        nm = r['Name'].replace('(anonymous namespace)::', '').replace('void ', '')
        stats[nm] = (int(r['Calls']), float(r['AverageNs']) / 1e3)
    from bench import KERNEL_OF  # noqa: E402
    for tag, sub in (('fp32', line), ('bf16', line.get('bf16'))):
        if not sub:
            continue
        print('==', tag, 'ms_per_step', sub['ms_per_step'], 'kernels_sum_ms', sub['kernels_sum_ms'])
        for k, v in sub['kernels'].items():
            pre = KERNEL_OF.get(k, k)
            hits = {n: s for n, s in stats.items() if n.startswith(pre)}
            print('  %-20s bench %7.2f us   rocprof %s' % (k, v['avg_launch_us'], '; '.join(
                '%s %d x %.2f' % (n.split('(')[0][:40], c, a) for n, (c, a) in sorted(hits.items()))))


if __name__ == '__main__':
    main()
