"""Two ranks sharing the GPU (gloo collectives on host copies): GpuShard + the export / select /
tie-position C ABI + the exchange protocol, against a single engine on the whole corpus."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def worker(rank, world, port, q):
    import importlib
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sharded = importlib.import_module('bpe-tokenizer_amd.sharded')
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        tr = sharded.ShardedTrainer.synthetic(device=0, rank=rank, world=world,
                                              bytes_per_rank=3 << 20, sample_bytes=1 << 20,
                                              seed=777, alphabet=40, base=60, dist=dist)
        for _ in range(60):
            if tr.step(0, 2) is None:
                break
        ids, off = tr.engine.read_corpus()
        q.put((rank, tr.merges, ids.tolist(), off.tolist()))
    finally:
        dist.destroy_process_group()


def test_two_ranks_on_one_gpu_match_single_engine():
    import importlib
    import torch.multiprocessing as mp
    from bpe_amd import pkg
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, rest) for r, *rest in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = pkg.synth_latin1(6 << 20, seed=777, A=40, base=60)
    e = pkg.Engine(0)
    e.add_latin1(data, sample_bytes=1 << 20)
    want = e.merge_until(0, 2, 60)
    assert [tuple(m) for m in res[0][0]] == want
    assert [tuple(m) for m in res[1][0]] == want
    ids, off = e.read_corpus()
    n0 = len(res[0][1])
    assert res[0][1] + res[1][1] == ids.tolist()
