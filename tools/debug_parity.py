#!/usr/bin/env python3
"""Step-by-step divergence finder (GPU box, test infrastructure): runs the small golden cases
through the engine one merge at a time and, at the first difference from the oracle, prints the
corpus before the step, both choices, and the hot-table counts that differ."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'oracle'))
from bpe_amd import pkg  # noqa: E402
from golden_util import load_small  # noqa: E402
from oracle import Corpus, OracleState  # noqa: E402


def hot_diff(e, st):
    t = torch.zeros(pkg.TABLE_BINS, dtype=torch.int64, device='cuda')
    e.export_counts(t.data_ptr())
    t = t.cpu().numpy()
    pa, pb, pc, _ = st.count_pairs()
    want = np.zeros(65536, np.int64)
    for a, b, c in zip(pa.tolist(), pb.tolist(), pc.tolist()):
        if a < 256 and b < 256:
            want[(b << 8) | a] += c   # hot bin b*256 + a (the LDS counter order)
    d = np.nonzero(t[:65536] != want)[0]
    return [(int(i & 255), int(i >> 8), int(t[i]), int(want[i])) for i in d[:10]]


def main():
    n_bad = 0
    for case in load_small():
        c = Corpus()
        for s in case['samples']:
            c.add(s)
        e = pkg.Engine(0)
        for i, l in enumerate(c.len16):
            e.set_token_len16(i, l)
        for s in c.samples:
            e.add_sample(s)
        off = np.concatenate([[0], np.cumsum([len(s) for s in c.samples])]).astype(np.int64)
        ids = np.concatenate(c.samples).astype(np.int32) if c.samples else np.zeros(0, np.int32)
        st = OracleState(ids, off, c.len16, len(c.len16))
        opts = case['opts']
        ml, mw = opts.get('max_length') or 0, opts.get('min_weight') or 0
        nt = len(c.len16)
        for it in range(10000):
            before = e.samples()
            if before != st.samples():
                print('CORPUS DIFF', case['name'], 'iter', it)
                print(' engine', before)
                print(' oracle', st.samples())
                n_bad += 1
                break
            m = e.find_next_merge(ml, mw)
            w = st.find_next_merge(opts.get('max_length'), opts.get('min_weight'))
            if m != (tuple(w) if w else None):
                print('FIND DIFF', case['name'], 'iter', it, 'engine', m, 'oracle', w)
                print(' corpus', before)
                print(' hot diff (a, b, engine, oracle)', hot_diff(e, st))
                n_bad += 1
                break
            if m is None:
                break
            rep = e.apply_merge(m[0], m[1], nt)
            st.apply_merge(m[0], m[1], nt)
            if rep != m[2]:
                print('APPLY COUNT', case['name'], 'iter', it, m, 'replaced', rep)
                print(' before', before)
                print(' engine', e.samples())
                print(' oracle', st.samples())
                n_bad += 1
                break
            nt += 1
        e.close()
        if n_bad >= 3:
            break
    print('bad cases:', n_bad)


if __name__ == '__main__':
    main()
