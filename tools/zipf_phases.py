#!/usr/bin/env python3
"""Where the skewed-corpus run (bench.py --corpus zipf: 1 GiB of Zipf(1.1) words, 8000 merges)
spends its merges: per chunk of merges the wall time and the stats counters' deltas (merge passes
in the maintained state (fused_passes), exact passes, compactions, host iterations of the device
loop), so the table-state stretches and the maintained state's rebuilds show where they happen.
Usage: python tools/zipf_phases.py [MiB] [merges] [chunk]"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    total = int(sys.argv[2]) if len(sys.argv) > 2 else 8000
    chunk = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    pkg = importlib.import_module('bpe-tokenizer_amd')
    e = pkg.Engine(0)
    e.add_latin1(pkg.synth_zipf(mib << 20, seed=12345), sample_bytes=1 << 20)
    e.stats_enable(True)
    keys = ('fused_passes', 'exact_passes', 'cold_rebuilds', 'compactions', 'loop_host', 'tie_passes',
            'iterations')
    prev = {k: 0 for k in keys}
    done = 0
    t_all = time.perf_counter()
    while done < total:
        t0 = time.perf_counter()
        got = e.merge_until(0, 2, min(chunk, total - done))
        dt = time.perf_counter() - t0
        done += len(got)
        st = e.stats()
        d = {k: st[k] - prev[k] for k in keys}
        prev = {k: st[k] for k in keys}
        print(json.dumps(dict({'merges': done, 'ms_per_merge': round(dt * 1e3 / max(1, len(got)), 4),
                               'last_w': got[-1][2] if got else None}, **d)), flush=True)
        if not got:
            break
    print(json.dumps({'total_s': round(time.perf_counter() - t_all, 2), 'merges': done}), flush=True)


if __name__ == '__main__':
    main()
