#!/usr/bin/env python3
"""Per-iteration cost of the multi-rank protocol (bpe-tokenizer_amd/sharded.py) measured with one
rank: the same corpus merged by ShardedTrainer's exchange (all-reduce over RCCL with world size 1,
heavy check, selection, apply: ShardedTrainer.step), by the device-resident rank loop
(ShardedTrainer.run_rank_loop: RCCL all-reduces on the engine's stream, no host sync per
iteration) and by the engine's single-GPU mergeUntil.
Usage: python tools/sharded_overhead.py [MiB] [iterations]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29531')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    pkg = importlib.import_module('bpe-tokenizer_amd')
    sharded = importlib.import_module('bpe-tokenizer_amd.sharded')
    data = pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0)
    eng = pkg.Engine(0)
    cmap, nt, _ = eng.add_latin1(data, sample_bytes=1 << 20)
    tr = sharded.ShardedTrainer(sharded.GpuShard(eng, 0), 0, 1, dist, nt, mib << 20)
    tr.world = 2   # (force the exchange protocol; the collectives still run over the one rank)
    for _ in range(5):
        tr.step(0, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms = [tr.step(0, 2) for _ in range(n)]
    torch.cuda.synchronize()
    proto = (time.perf_counter() - t0) / n
    e3 = pkg.Engine(0)
    e3.add_latin1(data, sample_bytes=1 << 20)
    tr3 = sharded.ShardedTrainer(sharded.GpuShard(e3, 0), 0, 1, dist, nt, mib << 20)
    tr3.world = 2
    tr3.run_rank_loop(5, 0, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms3 = tr3.run_rank_loop(n, 0, 2)
    torch.cuda.synchronize()
    rloop = (time.perf_counter() - t0) / n
    e2 = pkg.Engine(0)
    e2.add_latin1(data, sample_bytes=1 << 20)
    e2.merge_until(0, 2, 5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ms2 = e2.merge_until(0, 2, n)
    loop = (time.perf_counter() - t0) / n
    assert [tuple(m) for m in ms] == [tuple(m) for m in ms2], 'protocol and loop disagree'
    assert [tuple(m) for m in ms3] == [tuple(m) for m in ms2], 'rank loop and loop disagree'
    print(json.dumps({'corpus_mib': mib, 'iterations': n, 'protocol_ms_per_merge': proto * 1e3,
                      'rank_loop_ms_per_merge': rloop * 1e3,
                      'device_loop_ms_per_merge': loop * 1e3}), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
