#!/usr/bin/env python3
"""Progress of a sharded run on one device (shards exchanging through the device kernel): the C5
stream over S shards merged in chunks, printing per chunk the time, the index entries (builds),
hand-offs and merges on the index, for the streaming or the incremental mode.  auto: the mode left
to the engine (the stream, switching to the incremental mode past BPE_AUTO_PIX_VOCAB ids); stream:
the stream set by the caller, which the engine keeps (no switch).
Usage: python tools/multi_pix_probe.py MiB shards merges chunk [auto|stream|incremental]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mib, shards, total, chunk = (int(x) for x in sys.argv[1:5])
    mode = sys.argv[5] if len(sys.argv) > 5 else 'incremental'
    pkg = importlib.import_module('bpe-tokenizer_amd')
    data = pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0)
    e = pkg.Engine(devices=[0] * shards, reduce='host')
    _, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    del data
    if mode != 'auto':
        e.set_mode(mode)
    e.stats_enable(True)
    done = 0
    prev = (0, 0)
    t_all = time.perf_counter()
    while done < total:
        k = min(chunk, total - done)
        t0 = time.perf_counter()
        got = e.merge_until(0, 2, k)
        dt = time.perf_counter() - t0
        done += len(got)
        st = e.stats()
        # (this chunk's exchange per iteration, each shard)
        dx, di = st['xchg_bytes'] - prev[0], st['xchg_iters'] - prev[1]
        prev = (st['xchg_bytes'], st['xchg_iters'])
        print(json.dumps({'merges': done, 'chunk_xchg_bytes_per_iter': dx / shards / max(1, di), 'chunk_s': round(dt, 3), 'ms_per_merge': dt * 1e3 / max(1, len(got)),
                          'last_w': got[-1][2] if got else None, 'pix_merges': st['pix_merges'],
                          'pix_builds': st['pix_builds'], 'pix_host': st['pix_host'],
                          'loop_host': st['loop_host'],
                          # (the exchange each shard all-reduces per iteration, over the run so far)
                          'xchg_bytes_per_iter': st['xchg_bytes'] / shards / max(1, st['xchg_iters'])}),
              flush=True)
        if len(got) < k:
            break
    print(json.dumps({'total_s': time.perf_counter() - t_all, 'merges': done, 'mode': mode,
                      'shards': shards, 'corpus_mib': mib}), flush=True)


if __name__ == '__main__':
    main()
