"""One-rank-per-GPU driver of the merge loop (mergeUntil, core.ts:365-383) over a corpus sharded at
sample boundaries.

Pairs never cross samples (core.ts:265-267), so rank r owns a contiguous run of whole samples and
counts its pairs locally; the only exchange per iteration is the pair-count table (an all-reduce
over RCCL/xGMI) plus, when several pairs tie on (W, a+b), an all-reduce(MAX) of their last counted
positions (rule R3).  Every rank then applies the same merge to its shard.

world == 1 is the plain single-GPU loop.
"""
import importlib

import numpy as np

pkg = importlib.import_module('bpe-tokenizer_amd')


def first_appearance(data, alphabet_size=256):
    """Position of the first occurrence of every byte value (-1 if absent).  Scans in blocks and
    stops once `alphabet_size` distinct values have been seen."""
    first = np.full(256, -1, np.int64)
    seen = 0
    step = 1 << 16
    for s in range(0, len(data), step):
        u, idx = np.unique(data[s:s + step], return_index=True)
        new = first[u] < 0
        first[u[new]] = idx[new] + s
        seen += int(new.sum())
        if seen >= alphabet_size:
            break
    return first


class ShardedTrainer:
    def __init__(self, engine, rank, world, dist, n_tokens, live_global):
        self.engine = engine
        self.rank = rank
        self.world = world
        self.dist = dist
        self.n_tokens = n_tokens          # token_table.length (next new id, core.ts:315)
        self.live = live_global           # live corpus tokens over all ranks
        self.merges = []

    @classmethod
    def synthetic(cls, device, rank, world, bytes_per_rank, sample_bytes, seed, alphabet, base,
                  dist=None):
        """Rank r holds bytes [r*B, (r+1)*B) of one xorshift32 corpus stream."""
        data = pkg.synth_latin1(bytes_per_rank, seed=seed, A=alphabet, base=base,
                                skip=rank * bytes_per_rank)
        eng = pkg.Engine(device)
        if world == 1:
            cmap, nt, _ = eng.add_latin1(data, sample_bytes=sample_bytes)
            return cls(eng, rank, world, dist, nt, bytes_per_rank)
        # global first-appearance order (core.ts:186-199) across the shards, in corpus order
        import torch
        first = first_appearance(data, alphabet)
        key = np.where(first >= 0, rank * (1 << 40) + first, np.iinfo(np.int64).max)
        t = torch.tensor(key, dtype=torch.int64, device='cuda')
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        gkey = t.cpu().numpy()
        order = [int(ch) for ch in np.argsort(gkey, kind='stable') if gkey[ch] != np.iinfo(np.int64).max]
        cmap = np.full(256, -1, np.int32)
        for i, ch in enumerate(order):
            cmap[ch] = i
        for i in range(len(order)):
            eng.set_token_len16(i, 1)
        eng.add_latin1(data, sample_bytes=sample_bytes, char_to_id=cmap, n_tokens=len(order))
        return cls(eng, rank, world, dist, len(order), bytes_per_rank * world)

    def live_tokens_global(self):
        return self.live

    def find_next_merge(self, max_length=0, min_weight=0):
        if self.world == 1:
            return self.engine.find_next_merge(max_length, min_weight)
        raise NotImplementedError('multi-rank exchange')

    def step(self, max_length=0, min_weight=0):
        """One findNextMerge + applyMerge on every rank; returns (a, b, W) or None."""
        m = self.find_next_merge(max_length, min_weight)
        if m is None:
            return None
        a, b, w = m
        self.engine.apply_merge(a, b, self.n_tokens)
        self.n_tokens += 1
        self.live -= w
        self.merges.append(m)
        return m
