"""Summarise scripts/counters.sh output: per kernel, counter totals (mean over dispatches) and
per-wave values.   python scripts/ctr_summary.py [kernel ...]"""
import collections
import csv
import glob
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out', 'ctr')


def summary(kernel, pattern=None):
    """pattern: glob of the run directories (default g*_<kernel>, scripts/counters.sh; r3_ctr.sh
    writes <tag>_g<i>)"""
    tot, n = collections.defaultdict(float), collections.Counter()
    match = kernel.replace('mep_', 'k_').replace('block_', '')
    for f in glob.glob(os.path.join(ROOT, pattern or ('g*_%s' % kernel), 'run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            if match not in r['Kernel_Name'] or 'reduce' in r['Kernel_Name']:
                continue
            key = (r['Counter_Name'], r['Dispatch_Id'])
            tot[key] += float(r['Counter_Value'])
    per = collections.defaultdict(list)
    for (c, _), v in tot.items():
        per[c].append(v)
    return {c: sum(v) / len(v) for c, v in per.items()}


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--tag':     # r3_ctr.sh runs: --tag <tag> <kernel>
        s = summary(sys.argv[3], sys.argv[2] + '_g*')
        w = s.get('SQ_WAVES', 1.0)
        print(sys.argv[2], sys.argv[3], 'waves %.0f' % w)
        for c in sorted(s):
            print('  %-28s %16.1f   per wave %12.2f' % (c, s[c], s[c] / max(w, 1)))
        sys.exit(0)
    ks = sys.argv[1:] or ['mep_block_epi_fwd', 'mep_block_epi_bwd', 'mep_wgrad', 'mep_attn_fwd', 'mep_attn_bwd']
    for k in ks:
        s = summary(k)
        if not s:
            continue
        w = s.get('SQ_WAVES', 1.0)
        print(k, 'waves %.0f' % w)
        for c in sorted(s):
            print('  %-28s %16.1f   per wave %12.2f' % (c, s[c], s[c] / max(w, 1)))
