#!/usr/bin/env python3
"""What the stats event spans cost the device loop: alternating blocks of C3 merges with stats off
and on, wall time per merge of each (GPU box).  Usage: python tools/stats_overhead.py [MiB] [blk]"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    blk = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    pkg = importlib.import_module('bpe-tokenizer_amd')
    e = pkg.Engine(0)
    e.add_latin1(pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0), sample_bytes=1 << 20)
    e.merge_until(0, 2, 5)
    out = {'off': [], 'on': []}
    for r in range(6):
        on = r % 2 == 1
        e.stats_enable(on)
        t0 = time.perf_counter()
        got = e.merge_until(0, 2, blk)
        dt = time.perf_counter() - t0
        out['on' if on else 'off'].append(round(dt * 1e3 / len(got), 4))
    print(json.dumps({'ms_per_merge': out}), flush=True)


if __name__ == '__main__':
    main()
