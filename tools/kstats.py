#!/usr/bin/env python3
"""Prints a rocprofv3 kernel_stats.csv as name / calls / avg us / total ms, and a bench line's
ms_per_step and breakdown.  Usage: tools/kstats.py KSTATS.csv [BENCH.jsonl]"""
import csv
import json
import sys

for x in csv.DictReader(open(sys.argv[1])):
    print('%-52s %7s %10.2f %10.2f' % (x['Name'][:52], x['Calls'], float(x['AverageNs']) / 1e3,
                                       float(x['TotalDurationNs']) / 1e6))
if len(sys.argv) > 2:
    d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    print('value %.4g ms_per_step %.4f' % (d['value'], d['ms_per_step']), d['breakdown_ms_per_step'])
