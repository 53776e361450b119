#!/usr/bin/env python3
"""Apply-only replay on the C3 corpus (restoreMerge runs / batch encoding, bpe_apply_merges): trains
N merges with mergeUntil on one engine, then replays the log on a fresh engine holding the same
corpus and reports the time per replayed merge (one apply-only streaming pass each) next to the
time per mergeUntil iteration.  Usage: python tools/replay_bench.py [MiB] [N]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module('bpe-tokenizer_amd')


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 500
    data = pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0)
    e = pkg.Engine(0)
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    e.recount()
    t0 = time.perf_counter()
    log = e.merge_until(0, 2, n)
    train_s = time.perf_counter() - t0
    live = e.corpus_size()[1]
    e.close()
    abc = [(a, b, nt + i) for i, (a, b, _) in enumerate(log)]
    f = pkg.Engine(0)
    f.add_latin1(data, sample_bytes=1 << 20)
    f.apply_merges(abc[:5], count_after=False)   # warm-up (first launches)
    t0 = time.perf_counter()
    rep = f.apply_merges(abc[5:], count_after=False)
    replay_s = time.perf_counter() - t0
    assert rep == [w for _, _, w in log[5:]]
    assert f.corpus_size()[1] == live
    tokens = mib << 20
    print(json.dumps({
        'corpus_mib': mib, 'merges': len(log),
        'merge_until_ms_per_merge': train_s * 1e3 / len(log),
        'replay_ms_per_merge': replay_s * 1e3 / (len(log) - 5),
        'replay_GBps_alg': 4 * tokens / (replay_s / (len(log) - 5)) / 1e9,
    }), flush=True)


if __name__ == '__main__':
    main()
