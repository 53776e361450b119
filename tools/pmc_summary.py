#!/usr/bin/env python3
"""Summarises a tools/gpu_round.sh output directory into profiles/: per-kernel average duration
(rocprofv3 --kernel-trace --stats) and per-launch HBM traffic of the streaming kernel from the
separate FETCH_SIZE / WRITE_SIZE passes.

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled;
WRITE_SIZE is exact for 16 B/lane streaming stores and is taken as is.

Usage: python tools/pmc_summary.py gpurun_out/TAG profiles/TAG_pmc.json"""
import csv
import collections
import glob
import json
import os
import sys

# the merge pass, the dominant kernel of the bench: the device loop's pass, or (host-driven
# iterations) k_step<MERGE_XY>
KERNELS = ('k_step_loop<0>', 'bpe::k_step_loop', 'k_step<1, 0>')


def per_launch(path, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] == counter:
                vals[r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void bpe::', '')].append(float(r['Counter_Value']))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    src, dst = sys.argv[1], sys.argv[2]
    fetch, n_f = per_launch(os.path.join(src, 'fetch'), 'FETCH_SIZE')
    write, n_w = per_launch(os.path.join(src, 'write'), 'WRITE_SIZE')
    want = (sys.argv[3],) if len(sys.argv) > 3 else KERNELS   # (a kernel named on the command line)
    KERNEL = next((k for k in want if k in fetch), want[0])
    out = {'source': src, 'kernel': KERNEL}
    if KERNEL in fetch:
        out['fetch_bytes_per_launch'] = 2 * fetch[KERNEL] * 1024      # KiB, x2 (gfx950 wide reads)
        out['write_bytes_per_launch'] = write.get(KERNEL, 0.0) * 1024
        out['traffic_bytes_per_launch'] = out['fetch_bytes_per_launch'] + out['write_bytes_per_launch']
        out['launches_counted'] = n_f[KERNEL]
    stats = {}
    for f in glob.glob(os.path.join(src, 'trace', '**', '*kernel_stats.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            stats[r['Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void bpe::', '')] = {
                'calls': int(r['Calls']), 'avg_ns': float(r['AverageNs']), 'pct': float(r['Percentage'])}
    out['kernel_stats'] = stats
    bench = os.path.join(src, 'bench.jsonl')
    if os.path.exists(bench):
        for line in open(bench):
            if line.startswith('{'):
                out['bench'] = json.loads(line)
    os.makedirs(os.path.dirname(dst) or '.', exist_ok=True)
    json.dump(out, open(dst, 'w'), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != 'bench'}, indent=1))


if __name__ == '__main__':
    main()
