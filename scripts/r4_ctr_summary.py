"""Per-kernel SQ counter summary of a scripts/r4_counters.sh STAGE=sq run.

    python scripts/r4_ctr_summary.py <cfg> [gpurun_out/r4ctr] [profiles/r04_kernel_stats_<cfg>.csv] [tag r04]
        -> profiles/<tag>_counters_<cfg>.txt and .json

Counters are per dispatch (rocprofv3 --pmc ... --kernel-trace; each group its own run of
`bench.py --steps 2 --warmup 1`, every launch of the step counted), averaged over the dispatches
of each kernel.  Derived per kernel:
  mfma_flops      (SQ_INSTS_VALU_MFMA_MOPS_BF16 + _F32) x 512: MFMA work ISSUED per dispatch (split
                  products included -- a 3-part fp32 product issues 6 bf16 products)
  mfma_tflops     mfma_flops / the kernel's rocprofv3 average duration (the kernel-stats CSV)
  mfma_util       mfma_tflops / the dense bf16 peak (2.5 PFLOP/s; f32 MOPS priced at 157 TF)
  mfma_busy       SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x duration x 2.4 GHz): the share of every
                  SIMD's cycles its matrix core was busy
  valu_busy       SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x duration x 2.4 GHz) (quad-cycles)
                  Both use the kernel's rocprofv3 duration at the 2.4 GHz peak clock, not
                  GRBM_GUI_ACTIVE: that counter is summed over the 8 XCDs and reads high on
                  dispatches this short (MI355X_MICROARCH.md, DVFS), which made rocprofiler's
                  MfmaUtil / VALUBusy formulas 8-11x too small here.  Under load the clock runs
                  at ~1.9-2.3 GHz, so these are lower bounds (by up to ~20%).
  per wave        VALU / MFMA / VMEM-read / LDS instructions, and the shares of a wave's cycles
                  waiting (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY) and issuing
                  (SQ_ACTIVE_INST_ANY) -- quad-cycle counters, ratios only
  lds_conflict    SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles per LDS-array cycle)
"""
import collections
import csv
import glob
import json
import os
import sys

BF16_PEAK, F32_PEAK = 2.5e15, 157.3e12
N_CU, N_SIMD = 256, 1024
CLK = 2.4e9


def short(name):
    return name.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '').split('<')[0].strip()


def load(run_dir):
    acc = collections.defaultdict(lambda: collections.defaultdict(dict))
    for f in glob.glob(os.path.join(run_dir, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            d = acc[short(r['Kernel_Name'])][r['Counter_Name']]
            d[r['Dispatch_Id']] = d.get(r['Dispatch_Id'], 0.0) + float(r['Counter_Value'])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def durations(stats_csv):
    out = {}
    if stats_csv and os.path.exists(stats_csv):
        for r in csv.DictReader(open(stats_csv)):
            k = short(r['Name'])
            out[k] = max(out.get(k, 0.0), float(r['AverageNs']) * 1e-9)
    return out


def main():
    cfg = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else 'gpurun_out/r4ctr'
    stats = sys.argv[3] if len(sys.argv) > 3 else 'profiles/r04_kernel_stats_%s.csv' % cfg
    tag = sys.argv[4] if len(sys.argv) > 4 else 'r04'
    tab = collections.defaultdict(dict)
    for g in (1, 2, 3, 4):   # g4 (optional, SQ_L2=1): the L2 group
        if g == 4 and not os.path.isdir(os.path.join(src, '%s_g4' % cfg)):
            continue
        for k, cs in load(os.path.join(src, '%s_g%d' % (cfg, g))).items():
            for c, v in cs.items():
                tab[k].setdefault(c, v)          # GRBM_GUI_ACTIVE is in two groups: keep the first
    dur = durations(stats)
    res = {}
    for k, c in tab.items():
        w = c.get('SQ_WAVES', 0.0)
        gui = c.get('GRBM_GUI_ACTIVE', 0.0)
        e = {'waves': w, 'avg_us': round(dur[k] * 1e6, 2) if k in dur else None}
        mops_b, mops_f = c.get('SQ_INSTS_VALU_MFMA_MOPS_BF16', 0.0), c.get('SQ_INSTS_VALU_MFMA_MOPS_F32', 0.0)
        e['mfma_flops'] = 512 * (mops_b + mops_f)
        if k in dur and dur[k] > 0:
            e['mfma_tflops'] = round(512 * (mops_b + mops_f) / dur[k] / 1e12, 2)
            # time the issued products need at their peaks, over the kernel's time
            e['mfma_util'] = round((512 * mops_b / BF16_PEAK + 512 * mops_f / F32_PEAK) / dur[k], 4)
        if k in dur and dur[k] > 0:
            cyc = N_SIMD * dur[k] * CLK
            if 'SQ_VALU_MFMA_BUSY_CYCLES' in c:
                e['mfma_busy'] = round(c['SQ_VALU_MFMA_BUSY_CYCLES'] / cyc, 4)
            if 'SQ_ACTIVE_INST_VALU' in c:
                e['valu_busy'] = round(c['SQ_ACTIVE_INST_VALU'] * 4 / cyc, 4)
        if gui and k in dur and dur[k] > 0:
            e['grbm_clock_ghz'] = round(gui / 8 / dur[k] / 1e9, 2)   # reads high on short dispatches
        if w:
            for name, ctr in (('valu', 'SQ_INSTS_VALU'), ('mfma', 'SQ_INSTS_MFMA'), ('vmem_rd', 'SQ_INSTS_VMEM_RD'),
                              ('vmem_wr', 'SQ_INSTS_VMEM_WR'), ('lds', 'SQ_INSTS_LDS'), ('salu', 'SQ_INSTS_SALU')):
                if ctr in c:
                    e[name + '_per_wave'] = round(c[ctr] / w, 1)
        wc = c.get('SQ_WAVE_CYCLES', 0.0)
        if wc:
            for name, ctr in (('wait', 'SQ_WAIT_ANY'), ('issue_stall', 'SQ_WAIT_INST_ANY'), ('active', 'SQ_ACTIVE_INST_ANY'),
                              ('valu_active', 'SQ_ACTIVE_INST_VALU'), ('lds_active', 'SQ_ACTIVE_INST_LDS')):
                if ctr in c:
                    e[name + '_frac'] = round(c[ctr] / wc, 4)
        if c.get('SQ_LDS_IDX_ACTIVE'):
            e['lds_conflict'] = round(c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE'], 4)
        if c.get('TCC_HIT_sum', 0.0) + c.get('TCC_MISS_sum', 0.0) > 0:
            e['l2_hit'] = round(c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']), 4)
            e['l2_req_per_dispatch'] = c.get('TCC_REQ_sum')
        e['raw'] = {kk: round(v, 1) for kk, v in sorted(c.items())}
        res[k] = e
    os.makedirs('profiles', exist_ok=True)
    json.dump(res, open('profiles/%s_counters_%s.json' % (tag, cfg), 'w'), indent=1, sort_keys=True)
    order = sorted(res, key=lambda k: -(res[k]['avg_us'] or 0))
    lines = ['# %s SQ counters' % tag + ', %s bench workload (scripts/r4_counters.sh, scripts/r4_ctr_summary.py); '
             'durations: %s' % (cfg, os.path.basename(stats)),
             '%-18s %8s %7s %8s %7s %7s %7s %7s %7s %7s %6s %6s %6s %6s %6s %8s' % (
                 'kernel', 'avg_us', 'waves', 'TFLOP/s', 'mfmaU', 'mfmaBz', 'valuBz', 'VALU/w', 'MFMA/w', 'VMEM/w',
                 'wait', 'stall', 'activ', 'ldsCf', 'l2hit', 'l2reqM')]
    for k in order:
        e = res[k]
        f = lambda x, fmt='%7.3f': (fmt % x) if isinstance(x, (int, float)) else '%7s' % '-'   # noqa: E731
        lines.append('%-18s %8s %7d %8s %7s %7s %7s %7s %7s %7s %6s %6s %6s %6s %6s %8s' % (
            k[:18], f(e['avg_us'], '%8.2f'), e['waves'], f(e.get('mfma_tflops'), '%8.1f'), f(e.get('mfma_util')),
            f(e.get('mfma_busy')), f(e.get('valu_busy')), f(e.get('valu_per_wave'), '%7.0f'),
            f(e.get('mfma_per_wave'), '%7.0f'), f(e.get('vmem_rd_per_wave'), '%7.0f'), f(e.get('wait_frac'), '%6.2f'),
            f(e.get('issue_stall_frac'), '%6.2f'), f(e.get('active_frac'), '%6.2f'), f(e.get('lds_conflict'), '%6.3f'),
            f(e.get('l2_hit'), '%6.3f'), f(e['l2_req_per_dispatch'] / 1e6 if e.get('l2_req_per_dispatch') else None, '%8.2f')))
    open('profiles/%s_counters_%s.txt' % (tag, cfg), 'w').write('\n'.join(lines) + '\n')
    print('\n'.join(lines))


if __name__ == '__main__':
    main()
