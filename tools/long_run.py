#!/usr/bin/env python3
"""Full-length C3 run: mergeUntil on the 1 GiB synthetic corpus for N merges, printing the
per-window wall time, stream-pass time, exact/tie passes and W every `--every` merges.
Usage: python tools/long_run.py [--mib 1024] [--merges 8000] [--every 500]"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module('bpe-tokenizer_amd')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--mib', type=int, default=1024)
    ap.add_argument('--alphabet', type=int, default=256)
    ap.add_argument('--merges', type=int, default=8000)
    ap.add_argument('--every', type=int, default=500)
    args = ap.parse_args()
    A = args.alphabet
    data = pkg.synth_latin1(args.mib << 20, seed=12345, A=A, base=0 if A == 256 else 0x20)
    e = pkg.Engine(0)
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    del data
    e.stats_enable(True)
    done = 0
    t_all = time.perf_counter()
    while done < args.merges:
        k = min(args.every, args.merges - done)
        e.reset_stats()
        t0 = time.perf_counter()
        got = e.merge_until(0, 2, k)
        dt = time.perf_counter() - t0
        st = e.stats()
        done += len(got)
        print(json.dumps({
            'merges': done, 'wall_ms_per_merge': dt * 1e3 / max(1, len(got)),
            'pass_ms': st['step_ms'] / max(1, st['step_timed']),
            'launches': st['step_launches'], 'select_ms': st['select_ms'] / max(1, len(got)),
            'exact_passes': st['exact_passes'], 'tie_passes': st['tie_passes'],
            'compactions': st['compactions'], 'live': st['live_tokens'] / max(1, st['iterations']),
            'W_first': got[0][2] if got else None, 'W_last': got[-1][2] if got else None,
            'pair_scans_per_s': st['live_tokens'] / dt}), flush=True)
        if len(got) < k:
            break
    print(json.dumps({'total_s': time.perf_counter() - t_all, 'merges': done}), flush=True)


if __name__ == '__main__':
    main()
