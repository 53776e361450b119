"""Shared helpers for the golden-vector tests (test infrastructure)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def load_small():
    with open(os.path.join(GOLDEN, 'small_cases.json')) as f:
        return json.load(f)['cases']


def load_config2():
    p = os.path.join(GOLDEN, 'config2.json')
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def token_table_after(chars, char_weights, merges):
    """Host-side token table bookkeeping of the reference: addToCorpus weights (core.ts:201-202),
    new token c (core.ts:315-323), applyMerge weight update (core.ts:345-346)."""
    table = [[c, w, w] for c, w in zip(chars, char_weights)]
    for a, b, w in merges:
        table.append([table[a][0] + table[b][0], w, w])
        table[a][1] -= w
        table[b][1] -= w
    return table


def compact_index(table):
    """compactVectorIndex (core.ts:222-241)."""
    to_vec = {}
    v = 0
    for i, t in enumerate(table):
        if t[1] > 0:
            to_vec[i] = v
            v += 1
    return to_vec


def to_vector(ids, table):
    """encodeToVector's final mapping (core.ts:434-444)."""
    to_vec = compact_index(table)
    out = []
    for i in ids:
        if i not in to_vec:
            return 'error: unknown token index: %d' % i
        out.append(to_vec[i])
    return out


def char_weights(samples_ids, n_chars):
    w = np.zeros(n_chars, dtype=np.int64)
    for s in samples_ids:
        if len(s):
            w += np.bincount(np.asarray(s), minlength=n_chars)[:n_chars]
    return w.tolist()


def load_config3_prefix():
    """The reference's first merges on BASELINE config 3 (oracle/gen_golden.py --config3-prefix)."""
    p = os.path.join(GOLDEN, 'config3_prefix.json')
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)
