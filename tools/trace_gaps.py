#!/usr/bin/env python3
"""Per-kernel durations and the idle gaps before each kernel, from a rocprofv3 kernel trace
(--kernel-trace --output-format csv).  The gap before a launch = its start minus the end of the
previous kernel on the same queue: the GPU-side cost of a kernel boundary (dispatch, end-of-kernel
release) that no single kernel's duration shows.

Usage: python tools/trace_gaps.py TRACE_DIR [OUT.json] [--from-kernel NAME_SUBSTRING]
(--from-kernel: only the launches after the first one whose name holds the substring, i.e. the
timed loop and not the setup)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace('(anonymous namespace)::', '').split('(')[0]
    n = n.replace('void ', '').replace('bpe::', '')
    return n[:80]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    start_at = None
    if '--from-kernel' in sys.argv:
        start_at = sys.argv[sys.argv.index('--from-kernel') + 1]
        args = [a for a in args if a != start_at]
    files = glob.glob(os.path.join(args[0], '**', '*kernel_trace.csv'), recursive=True)
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), short(r['Kernel_Name']),
                             r.get('Queue_Id', '0')))
    rows.sort()
    if start_at:
        i0 = next((i for i, r in enumerate(rows) if start_at in r[2]), 0)
        rows = rows[i0:]
    dur = defaultdict(list)
    gap = defaultdict(list)
    last_end = {}
    for s, e, n, q in rows:
        dur[n].append(e - s)
        if q in last_end:
            g = s - last_end[q]
            if 0 <= g < 200000:   # (a host sync or a batch boundary is not a kernel boundary)
                gap[n].append(g)
        last_end[q] = max(e, last_end.get(q, 0))
    span = (rows[-1][1] - rows[0][0]) if rows else 0
    out = {'launches': len(rows), 'span_ms': span / 1e6, 'kernels': {}}
    for n in sorted(dur, key=lambda k: -sum(dur[k])):
        d, g = dur[n], gap[n]
        ds = sorted(d)
        out['kernels'][n] = {'calls': len(d), 'avg_us': sum(d) / len(d) / 1e3, 'total_ms': sum(d) / 1e6,
                             'median_us': ds[len(ds) // 2] / 1e3, 'p90_us': ds[9 * len(ds) // 10] / 1e3,
                             'avg_gap_before_us': (sum(g) / len(g) / 1e3) if g else None,
                             'total_gap_ms': sum(g) / 1e6}
    out['busy_ms'] = sum(v['total_ms'] for v in out['kernels'].values())
    # the time some kernel runs (the union of the intervals: kernels of several queues overlap)
    u, cur_s, cur_e = 0, None, None
    for s, e, _n, _q in rows:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                u += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        u += cur_e - cur_s
    out['union_busy_ms'] = u / 1e6
    out['gaps_ms'] = sum(v['total_gap_ms'] for v in out['kernels'].values())
    txt = json.dumps(out, indent=1)
    if len(args) > 1:
        with open(args[1], 'w') as f:
            f.write(txt)
    print('launches %d  span %.1f ms  busy %.1f ms (union %.1f ms)  gaps %.1f ms'
          % (len(rows), out['span_ms'], out['busy_ms'], out['union_busy_ms'], out['gaps_ms']))
    for n, v in list(out['kernels'].items())[:14]:
        print('%-60s %6d  %9.2f us  gap %s' % (n[:60], v['calls'], v['avg_us'],
                                               '%.2f us' % v['avg_gap_before_us'] if v['avg_gap_before_us'] is not None else '-'))


if __name__ == '__main__':
    main()
