#!/usr/bin/env python3
"""The maintained state's selection on the zipf C3 corpus: mergeUntil timed over N merges after a
warmup, with the cold table's size (stats cold_used).  Run with and without BPE_SEL_FULL=1 (every
selection a full scan) to compare the block-maxima selection with the full one.
Usage: python tools/zipf_sel.py [MiB] [warmup] [merges]"""
import importlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 2000
    pkg = importlib.import_module('bpe-tokenizer_amd')
    e = pkg.Engine(0)
    e.add_latin1(pkg.synth_zipf(mib << 20, seed=12345), sample_bytes=1 << 20)
    e.stats_enable(True)
    e.merge_until(0, 2, warm)
    e.reset_stats()
    e.stats_enable(True)
    e.merge_until(0, 2, 1)
    b0 = e.stats()['sel_blocks']
    t0 = time.perf_counter()
    got = e.merge_until(0, 2, n)
    dt = time.perf_counter() - t0
    st = e.stats()
    print(json.dumps({'mib': mib, 'warmup': warm, 'merges': len(got), 'ms_per_merge': 1e3 * dt / len(got),
                      'sel_full': bool(os.environ.get('BPE_SEL_FULL')), 'cold_used': st['cold_used'],
                      'fused_passes': st['fused_passes'], 'blocks_per_sel': (st['sel_blocks'] - b0) / max(1, len(got)),
                      'cold_blocks': st['cold_used'] // 1024, 'loop_host': st['loop_host'],
                      'select_ms_per_iter': st['select_ms'] / max(1, st['step_timed']),
                      'merges_hash': hash(tuple(map(tuple, got)))}), flush=True)


if __name__ == '__main__':
    main()
