"""Pins the multi-threaded CPU restatement (oracle/bpe_cpu_mt.cc — the larger parity cases'
checker and bench.py's multi-core CPU baseline) to the reference's own outputs and to the literal
restatement oracle/bpe_oracle.c."""
import random

import numpy as np
import pytest

from golden_util import load_small
from oracle import Corpus, CpuMT, OracleState

CASES = load_small()


@pytest.mark.parametrize('threads', [1, 3])
def test_mt_matches_reference_golden(threads):
    """Every reference-generated case (tests/golden/small_cases.json): merges and final corpus."""
    bad = []
    for case in CASES:
        c = Corpus()
        for s in case['samples']:
            c.add(s)
        ids, off = c.flat()
        st = CpuMT(ids, off, c.len16, len(c.chars), threads=threads)
        o = case['opts']
        merges = st.merge_until(o.get('max_length'), o.get('min_weight'), o.get('max_iterations'))
        if [list(m) for m in merges] != case['merges'] or st.samples() != case['final_ids']:
            bad.append(case['name'])
        st.close()
    assert not bad, bad[:10]


def random_samples(rng, n_samples, alphabet, run_bias, per):
    out = []
    for _ in range(n_samples):
        L = rng.randint(0, 2 * per)
        toks = []
        while len(toks) < L:
            t = rng.randrange(alphabet)
            k = 1 if rng.random() > run_bias else rng.randint(2, 40)
            toks += [t] * k
        out.append(np.asarray(toks[:L], np.int32))
    return out


@pytest.mark.parametrize('seed', range(8))
def test_mt_matches_literal_oracle(seed):
    """Random multi-sample corpora (runs, cold ids >= 256, max_length / min_weight): the
    threaded restatement's merges and corpus equal the literal scan-order one's."""
    rng = random.Random(1000 + seed)
    alphabet = rng.choice([2, 5, 40, 256, 300, 700])
    samples = random_samples(rng, rng.choice([1, 5, 40]), alphabet, rng.choice([0.0, 0.2, 0.6]),
                             rng.choice([50, 2000]))
    len16 = [rng.choice([1, 1, 2]) for _ in range(alphabet)]
    ids = np.concatenate(samples) if samples else np.zeros(0, np.int32)
    off = np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64)
    opts = (rng.choice([0, 0, 3, 5]), rng.choice([0, 2, 3, -1]), rng.choice([30, 80]))
    want = OracleState(ids, off, len16, alphabet).merge_until(*opts)
    ref = OracleState(ids, off, len16, alphabet)
    ref.merge_until(*opts)
    st = CpuMT(ids, off, len16, alphabet, threads=rng.choice([2, 4, 7]))
    assert st.merge_until(*opts) == want
    assert st.samples() == ref.samples()


@pytest.mark.slow
def test_config3_prefix_fixture():
    """BASELINE config 3 (1 GiB, 256-char alphabet, 1 MiB samples): the threaded restatement's
    first merges and live token count equal the reference's own run
    (tests/golden/config3_prefix.json, oracle/gen_golden.py --config3-prefix)."""
    from golden_util import load_config3_prefix
    from oracle import xorshift_corpus
    g = load_config3_prefix()
    if g is None:
        pytest.skip('config3 prefix fixture not generated')
    n = g['total']
    data = xorshift_corpus(g['seed'], g['A'], g['base'], n)
    lut = np.full(256, -1, np.int32)
    uniq, idx = np.unique(data[:1 << 20], return_index=True)
    for k, u in enumerate(uniq[np.argsort(idx)]):
        lut[u] = k
    assert (lut >= 0).sum() == g['char_count']
    ids = lut[data]
    del data
    off = np.arange(0, n + 1, g['sample'], dtype=np.int64)
    st = CpuMT(ids, off, [1] * g['char_count'], g['char_count'])
    del ids
    got = st.merge_until(0, g['min_weight'], g['max_iterations'])
    assert [list(m) for m in got] == g['merges']
    assert st.live() == g['live_tokens_after']
