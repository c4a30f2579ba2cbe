"""Per-position dispatch durations of a rocprofv3 kernel trace: the step is cut at every dispatch of
a marker kernel (default k_wsplit, the first launch of a realformer step) and each position's
duration is averaged over the complete steps after the first two (warmup / capture).

  python scripts/dispatch_order.py <rocprofv3 -d dir> [marker]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name):
    return name.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')[:60]


def main():
    src = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'k_wsplit'
    hits = glob.glob(os.path.join(src, '**', '*kernel_trace.csv'), recursive=True)
    rows = []
    for path in hits:
        for r in csv.DictReader(open(path)):
            n = short(r['Kernel_Name'])
            if 'k_stamp' not in n and 'k_hbm_probe' not in n:   # bench.py's timing stamps / probe
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), n))
    rows.sort()
    steps, cur = [], None
    for s, e, n in rows:
        if marker in n:
            cur = []
            steps.append(cur)
        if cur is not None:
            cur.append((n, (e - s) / 1e3, s))
    steps = steps[2:-1] if len(steps) > 3 else steps
    if not steps:
        print('no steps found')
        return
    L = min(len(x) for x in steps)
    acc = defaultdict(list)
    for st in steps:
        for i in range(L):
            acc[i].append(st[i][1])
    tot = 0.0
    for i in range(L):
        v = sorted(acc[i])[len(acc[i]) // 2]
        tot += v
        print('%2d %-60s %9.2f us' % (i, steps[0][i][0], v))
    span = sorted((st[L - 1][2] - st[0][2]) / 1e3 for st in steps)[len(steps) // 2]
    print('steps %d, kernels/step %d, sum of medians %.1f us, first-to-last start %.1f us' % (len(steps), L, tot, span))


if __name__ == '__main__':
    main()
