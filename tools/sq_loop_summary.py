#!/usr/bin/env python3
"""Per-launch SQ counters of the device loop's streaming pass (k_step_loop) and the other loop
kernels, from tools/gpu_round2.sh's sq / sq2 passes.  Usage: tools/sq_loop_summary.py OUTDIR"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for sub in ('sq', 'sq2'):
    for f in glob.glob(os.path.join(d, sub, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            kern = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void bpe::', '').replace('bpe::', '')
            agg[(kern, r['Counter_Name'])][r['Dispatch_Id']] += float(r['Counter_Value'])
rows = {}
for (kern, c), v in sorted(agg.items()):
    vals = list(v.values())
    rows.setdefault(kern, {})[c] = (sum(vals) / len(vals), len(vals))
for kern, cs in sorted(rows.items()):
    print(kern)
    for c, (m, n) in sorted(cs.items()):
        print('  %-24s %14.6g  (mean of %d launches)' % (c, m, n))
    if 'SQ_WAVE_CYCLES' in cs and 'SQ_INSTS_VALU' in cs:
        w = cs['SQ_WAVES'][0] if 'SQ_WAVES' in cs else 1
        print('  -> VALU/wave %.0f, SALU/wave %.0f, LDS/wave %.0f' % (
            cs['SQ_INSTS_VALU'][0] / w, cs.get('SQ_INSTS_SALU', (0,))[0] / w,
            cs.get('SQ_INSTS_LDS', (0,))[0] / w))
    if 'SQ_WAVE_CYCLES' in cs and 'SQ_WAIT_ANY' in cs:
        wc = cs['SQ_WAVE_CYCLES'][0]
        print('  -> wait_any %.1f%%, wait_inst_any %.1f%% of wave cycles' % (
            100 * cs['SQ_WAIT_ANY'][0] / wc, 100 * cs.get('SQ_WAIT_INST_ANY', (0,))[0] / wc))
    if 'SQ_ACTIVE_INST_VALU' in cs and 'SQ_WAVE_CYCLES' in cs:
        print('  -> active VALU %.1f%% of wave cycles' % (100 * cs['SQ_ACTIVE_INST_VALU'][0] / cs['SQ_WAVE_CYCLES'][0]))
