#!/usr/bin/env python3
"""Per-iteration cost of the multi-GPU exchange, measured on one GPU with its RCCL legs live
(SURVEY.md §8(e)).  The same C3-stream corpus is merged by:
  device_loop   the engine's single-context mergeUntil (no exchange at all);
  rank_loop     ShardedTrainer(rank_loop=True) over a 1-rank RCCL process group (torch.distributed
                'nccl' = RCCL), the one-process-per-GPU path bench.py's N>1 leg takes: per iteration
                an RCCL all-reduce(SUM) of the exchange buffer and an all-reduce(MAX) of the tie
                words on the engine's stream, issued from C++ by one bpe_rank_loop_rccl call per
                batch (the engine's own communicator, made from a broadcast unique id);
  rank_loop_py  the same with the all-reduces as torch.distributed calls from Python and the
                three rank-loop C-ABI calls per iteration (BPE_RANK_LOOP=python; round 4's path);
  multi_rccl    bpe_create_multi(devices=[0], reduce='rccl'): ncclCommInitAll over one device and
                grouped ncclAllReduce calls from C++ (the drop-in's BPE_DEVICES path);
  protocol      ShardedTrainer.step: the host protocol of every iteration (table all-reduce,
                heavy check, selection, tie all-reduce; a host round trip per merge).
All four must give the same merges.  Prints one JSON line.
Usage: python tools/sharded_overhead.py [MiB] [iterations]"""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(f):
    import torch
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = f()
    torch.cuda.synchronize()
    return r, time.perf_counter() - t0


def main():
    import torch
    import torch.distributed as dist
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    warm = 5
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29531')
    torch.cuda.set_device(0)
    dist.init_process_group('nccl', rank=0, world_size=1, device_id=torch.device('cuda', 0))
    pkg = importlib.import_module('bpe-tokenizer_amd')
    sharded = importlib.import_module('bpe-tokenizer_amd.sharded')
    data = pkg.synth_latin1(mib << 20, seed=12345, A=256, base=0)
    out = {'corpus_mib': mib, 'iterations': n, 'backend': dist.get_backend()}

    e = pkg.Engine(0)
    e.add_latin1(data, sample_bytes=1 << 20)
    e.merge_until(0, 2, warm)
    want, t = timed(lambda: e.merge_until(0, 2, n))
    out['device_loop_ms_per_merge'] = t / n * 1e3
    e.close()

    for key, how in (('rank_loop', 'native'), ('rank_loop_py', 'python')):
        os.environ['BPE_RANK_LOOP'] = how
        tr = sharded.ShardedTrainer.synthetic(device=0, rank=0, world=1, bytes_per_rank=mib << 20,
                                              sample_bytes=1 << 20, seed=12345, alphabet=256, base=0,
                                              dist=dist, rank_loop=True)
        assert tr.exchange
        tr.run(warm, 0, 2)
        assert tr._native == (how == 'native')
        got, t = timed(lambda: tr.run(n, 0, 2))
        assert [tuple(m) for m in got] == want, '%s and device loop disagree' % key
        out[key + '_ms_per_merge'] = t / n * 1e3
        tr.engine.close()
    os.environ.pop('BPE_RANK_LOOP')

    m = pkg.Engine(devices=[0], reduce='rccl')
    m.add_latin1(data, sample_bytes=1 << 20)
    m.merge_until(0, 2, warm)
    got, t = timed(lambda: m.merge_until(0, 2, n))
    assert got == want, 'multi-context RCCL loop and device loop disagree'
    out['multi_rccl_ms_per_merge'] = t / n * 1e3
    m.close()

    tr = sharded.ShardedTrainer.synthetic(device=0, rank=0, world=1, bytes_per_rank=mib << 20,
                                          sample_bytes=1 << 20, seed=12345, alphabet=256, base=0,
                                          dist=dist, rank_loop=True)
    for _ in range(warm):
        tr.step(0, 2)
    k = min(n, 100)
    got, t = timed(lambda: [tr.step(0, 2) for _ in range(k)])
    assert [tuple(x) for x in got] == want[:k], 'host protocol and device loop disagree'
    out['protocol_ms_per_merge'] = t / k * 1e3
    out['protocol_iterations'] = k
    out['rank_loop_overhead_ms'] = out['rank_loop_ms_per_merge'] - out['device_loop_ms_per_merge']
    out['rank_loop_py_overhead_ms'] = out['rank_loop_py_ms_per_merge'] - out['device_loop_ms_per_merge']
    out['multi_rccl_overhead_ms'] = out['multi_rccl_ms_per_merge'] - out['device_loop_ms_per_merge']
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
