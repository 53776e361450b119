#!/usr/bin/env python3
"""Per-chunk instruction mix of the k_step kernels from a tools/profile_sq.sh (or profile.sh) run."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
chunks = float(sys.argv[2]) if len(sys.argv) > 2 else 4194304
for f in sorted(glob.glob(os.path.join(d, 'trace', '**', '*kernel_stats.csv'), recursive=True)):
    for r in csv.DictReader(open(f)):
        print('%-40s calls %4s avg %.1f us' % (r['Name'][:40], r['Calls'], float(r['AverageNs']) / 1e3))
for f in sorted(glob.glob(os.path.join(d, '*', '**', '*counter_collection.csv'), recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if 'k_step' not in r['Kernel_Name']:
            continue
        kern = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void bpe::', '')
        agg[(kern, r['Counter_Name'])][r['Dispatch_Id']] += float(r['Counter_Value'])
    for (kern, c), v in sorted(agg.items()):
        vals = list(v.values())
        m = sum(vals) / len(vals)
        print('%-22s %-22s %12.4g  per-chunk %8.2f' % (kern, c, m, m / chunks))
