#!/usr/bin/env python3
"""Where a skewed-corpus iteration spends its time (bpe_synth_zipf corpus): wall-clock of
find_next_merge (host path: selection, heavy check, exact pass) and apply_merge at a given merge
depth.  Usage: python tools/zipf_probe.py [MiB] [depth] [reps]"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    pkg = importlib.import_module('bpe-tokenizer_amd')
    e = pkg.Engine(0)
    e.add_latin1(pkg.synth_zipf(mib << 20, seed=12345), sample_bytes=1 << 20)
    t0 = time.perf_counter()
    e.merge_until(0, 2, depth)
    t_run = time.perf_counter() - t0
    e.reset_stats()
    e.stats_enable(True)
    nt = e.num_tokens()
    find, apply_ = [], []
    for i in range(reps):
        t0 = time.perf_counter()
        m = e.find_next_merge(0, 2)
        t1 = time.perf_counter()
        e.apply_merge(m[0], m[1], nt + i)
        t2 = time.perf_counter()
        find.append(t1 - t0)
        apply_.append(t2 - t1)
    print(json.dumps({'mib': mib, 'depth': depth, 'run_s': t_run,
                      'find_ms': [round(x * 1e3, 3) for x in find],
                      'apply_ms': [round(x * 1e3, 3) for x in apply_], 'stats': e.stats()}),
          flush=True)


if __name__ == '__main__':
    main()
