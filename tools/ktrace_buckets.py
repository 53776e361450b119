#!/usr/bin/env python3
"""Average duration of each of the busiest kernels per bucket of consecutive launches, from a
rocprofv3 kernel_trace.csv (how a kernel's cost moves over a run).
Usage: tools/ktrace_buckets.py TRACE.csv [bucket] [n_kernels]"""
import csv
import sys
from collections import defaultdict

path = sys.argv[1]
bucket = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
top = int(sys.argv[3]) if len(sys.argv) > 3 else 4
d = defaultdict(list)
for r in csv.DictReader(open(path)):
    d[r['Kernel_Name'][:40]].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
names = sorted(d, key=lambda k: -sum(d[k]))[:top]
for k in names:
    v = d[k]
    avg = ['%.0f' % (sum(v[i:i + bucket]) / len(v[i:i + bucket]) / 1e3) for i in range(0, len(v), bucket)]
    print('%-40s n=%-6d us/launch per %d: %s' % (k, len(v), bucket, ' '.join(avg)))
