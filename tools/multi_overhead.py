#!/usr/bin/env python3
"""Per-merge cost of the sharded rank loop's exchange with host-copy all-reduces (BPE_REDUCE_HOST:
n shards on one device, the exchange through pinned host buffers), against one context on the
same corpus.  Two corpora: the uniform C3 stream (the table state: 81 920-bin tables exchanged
every merge) and the zipf words (the maintained state: delta rows).  The shards share one GPU, so
their streaming passes run one after another: the overhead per merge is
    t_multi - t_single   (the n shards' passes together stream the same bytes as the one corpus).

Usage: python tools/multi_overhead.py [MiB] [shards] [merges] [OUT.json]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module('bpe-tokenizer_amd')


def timed(e, pre, n):
    # (merge_until returns after its last batch's host sync: nothing is left in flight)
    e.merge_until(0, 2, pre)
    e.stats_enable(True)
    e.reset_stats()
    t0 = time.perf_counter()
    got = e.merge_until(0, 2, n)
    dt = time.perf_counter() - t0
    return got, dt, e.stats()


def run(kind, mib, shards, n, pre):
    data = pkg.synth_zipf(mib << 20, seed=12345) if kind == 'zipf' else \
        pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0)
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    g1, t1, s1 = timed(one, pre, n)
    one.close()
    multi = pkg.Engine(devices=[0] * shards, reduce='host')
    multi.add_latin1(data, sample_bytes=1 << 20)
    del data
    gm, tm, sm = timed(multi, pre, n)
    multi.close()
    assert gm == g1, 'sharded merges differ'
    return {'corpus': kind, 'MiB': mib, 'shards': shards, 'merges_timed': len(g1), 'after_merges': pre,
            'single_ms_per_merge': t1 * 1e3 / max(1, len(g1)),
            'multi_ms_per_merge': tm * 1e3 / max(1, len(gm)),
            'overhead_ms_per_merge': (tm - t1) * 1e3 / max(1, len(g1)),
            'multi_fused_passes': sm['fused_passes'], 'multi_loop_host': sm['loop_host'],
            'single_step_ms': s1['step_ms'] / max(1, s1['step_timed']),
            'multi_step_ms_slowest_shard': sm['step_ms'] / max(1, sm['step_timed'])}


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    shards = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 300
    out = {'what': 'host-copy exchange over %d shards on one MI355X vs one context (tools/multi_overhead.py)'
                   % shards, 'runs': []}
    for kind, pre in (('latin1', 20), ('zipf', 1500)):
        r = run(kind, mib, shards, n, pre)
        print(json.dumps(r), flush=True)
        out['runs'].append(r)
    if len(sys.argv) > 4:
        with open(sys.argv[4], 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
