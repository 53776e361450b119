"""The incremental mode (bpe_set_mode BPE_MODE_INCREMENTAL, csrc/bpe_pix.hip.h): mergeUntil on a
position index, O(W) work per merge.  The same merges and corpus as the reference's full recount
are required: against the oracle, against the streaming mode on corpora the oracle cannot finish,
and across the hand-offs between the index and the stream.  (The randomized, golden, tie, run and
compaction tests of test_gpu_parity.py run in this mode too: MODES includes 'pix'.)"""
import random

import numpy as np
import pytest

from bpe_amd import make_engine, pkg
from oracle import CpuMT, OracleState
from test_gpu_parity import check_sample_index, random_corpus

pytestmark = pytest.mark.gpu


def _flat(samples):
    ids = np.concatenate(samples).astype(np.int32) if samples else np.zeros(0, np.int32)
    return ids, np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64)


@pytest.mark.parametrize('seed', range(6))
def test_mixed_calls_and_option_changes(seed):
    """mergeUntil on the index, single findNextMerge/applyMerge calls on the stream between, and
    max_length changing from call to call (each call builds its index): the oracle's merges."""
    rng = random.Random(900 + seed)
    alphabet = rng.choice([3, 30, 256, 280])
    samples = random_corpus(rng, rng.choice([30000, 400000]), alphabet, rng.choice([0.0, 0.3]),
                            rng.choice([1, 9, 100]))
    len16 = [rng.choice([1, 1, 2]) for _ in range(alphabet)]
    ids, off = _flat(samples)
    st = OracleState(ids, off, len16, alphabet)
    e = make_engine(samples, len16)
    e.set_mode('incremental')
    e.stats_enable(True)
    n_tok = alphabet
    for step in range(6):
        ml = rng.choice([0, 0, 4, 6])
        if step % 2 == 0:
            want = st.merge_until(ml, 2, 15)
            got = e.merge_until(ml, 2, 15)
            assert got == want, (step, got[:3], want[:3])
            n_tok += len(got)
        else:
            w = st.merge_until(ml, 2, 1)
            m = e.find_next_merge(ml, 2)
            assert (m is None and not w) or [m] == w
            if m is not None:
                assert e.apply_merge(m[0], m[1], n_tok) == m[2]
                n_tok += 1
    assert e.samples() == st.samples()
    check_sample_index(e, st.samples(), rng)
    assert e.stats()['pix_merges'] > 0


@pytest.mark.parametrize('n', [5, 9, 10, 1023, 70000, 300001])
def test_runs_in_the_index(n):
    """'x' * n between other tokens: runs walked by one thread up to PIX_WALK, longer ones handed
    to the stream; x x merges, their (c, c) runs, trailing x's."""
    sample = np.array([1] + [0] * n + [2, 0, 0, 0, 1], np.int32)
    st = OracleState(sample, np.array([0, len(sample)], np.int64), [1, 1, 1], 3)
    want = st.merge_until(0, 2, 0)
    e = make_engine([sample], [1, 1, 1])
    e.set_mode('incremental')
    e.stats_enable(True)
    assert e.merge_until(0, 2, 0) == want
    assert e.samples() == st.samples()
    s = e.stats()
    assert s['pix_merges'] > 0
    if n > 1 << 16:   # runs past the walk bound: the stream takes them (heavy-merge prefix or hand-off)
        assert s['pix_host'] >= 1 or s['iterations'] > s['pix_merges'], s


def test_uniform_c3_slice_matches_the_stream():
    """A 32 MiB slice of BASELINE config 3, 2500 merges: the incremental mode against the
    streaming mode and the multi-threaded CPU restatement (first 300 merges)."""
    data = pkg.synth_latin1(32 << 20, seed=12345, A=256, base=0)
    a = pkg.Engine(0)
    a.add_latin1(data, sample_bytes=1 << 20)
    b = pkg.Engine(0)
    cmap, nt, _ = b.add_latin1(data, sample_bytes=1 << 20)
    b.set_mode('incremental')
    b.stats_enable(True)
    want = a.merge_until(0, 2, 2500)
    got = b.merge_until(0, 2, 2500)
    assert got == want
    s = b.stats()
    assert s['pix_merges'] == 2500 and s['pix_host'] == 0, s
    ia, oa = a.read_corpus()
    ib, ob = b.read_corpus()
    assert np.array_equal(ia, ib) and np.array_equal(oa, ob)
    ids = cmap[data]
    off = np.arange(0, len(data) + 1, 1 << 20, dtype=np.int64)
    cpu = CpuMT(ids, off, [1] * nt, nt, threads=8)
    assert cpu.merge_until(0, 2, 300) == got[:300]
    cpu.close()


def test_zipf_words_match_the_stream():
    """Skewed corpus (Zipf words): long merged tokens, cold pairs, runs of merged tokens."""
    data = pkg.synth_zipf(8 << 20, seed=3)
    a = pkg.Engine(0)
    a.add_latin1(data, sample_bytes=1 << 20)
    b = pkg.Engine(0)
    b.add_latin1(data, sample_bytes=1 << 20)
    b.set_mode('incremental')
    want = a.merge_until(0, 2, 1500)
    got = b.merge_until(0, 2, 1500)
    assert got == want
    assert np.array_equal(a.read_corpus()[0], b.read_corpus()[0])


@pytest.mark.parametrize('ml', [3, 5])
def test_max_length_new_pairs_stay_on_the_index(ml):
    """Under max_length the new token's length is known before its pairs are ranked (pix_commit
    writes it; k_pix_alloc lifts the block maxima from it): a new pair too long to merge must not
    raise its block's max, which would leave k_pix_select without a candidate (a hand-off to the
    stream and a rebuilt index).  'ab' repeats make (c, c) the most frequent new pair."""
    rng = np.random.default_rng(5 + ml)
    samples = []
    for _ in range(60):
        n = int(rng.integers(500, 3000))
        s = np.resize(np.array([0, 1], np.int32), n)
        noise = rng.random(n) < 0.15
        s[noise] = rng.integers(2, 20, int(noise.sum()))
        samples.append(s)
    len16 = [1] * 20
    ids, off = _flat(samples)
    st = OracleState(ids, off, len16, 20)
    e = make_engine(samples, len16)
    e.set_mode('incremental')
    e.stats_enable(True)
    want = st.merge_until(ml, 2, 40)
    got = e.merge_until(ml, 2, 40)
    assert got == want, (got[:4], want[:4])
    assert e.samples() == st.samples()
    s = e.stats()
    assert s['pix_merges'] == len(got) and s['pix_host'] == 0, s


def test_index_build_count_sweeps():
    """Per-workgroup counts far past the index build's 16-bit LDS counters (k_pix_hot_count: the
    block-end sweeps into the slab): 24 MiB of 'ab' repeats, runs of 'z' of every parity and
    random bytes, against the streaming mode."""
    rng = np.random.default_rng(77)
    parts = []
    for kind, n in zip(rng.choice(3, 60000, p=[0.55, 0.3, 0.15]), rng.integers(40, 1200, 60000)):
        if kind == 0:
            parts.append(np.resize(np.frombuffer(b'ab', np.uint8), n))
        elif kind == 1:
            parts.append(np.full(n, ord('z'), np.uint8))
        else:
            parts.append(rng.integers(0, 256, n, dtype=np.uint8))
    data = np.concatenate(parts)[:24 << 20]
    a = pkg.Engine(0)
    a.add_latin1(data, sample_bytes=1 << 20)
    b = pkg.Engine(0)
    b.add_latin1(data, sample_bytes=1 << 20)
    b.set_mode('incremental')
    b.stats_enable(True)
    want = a.merge_until(0, 2, 40)
    got = b.merge_until(0, 2, 40)
    assert got == want
    assert b.stats()['pix_merges'] > 0
    assert np.array_equal(a.read_corpus()[0], b.read_corpus()[0])


@pytest.mark.parametrize('fill', ['two_level', 'pairs'])
@pytest.mark.parametrize('seed', range(3))
def test_index_build_fill_forms(fill, seed, monkeypatch):
    """The index build's two fill forms (csrc/bpe_pix.hip.h: the two-level scatter by first then
    second token, and the per-pair cursors it falls back to when one first token dominates,
    forced here with BPE_PIX_FILL_PAIRS): the oracle's merges either way, with skewed first tokens
    in one of the corpora."""
    if fill == 'pairs':
        monkeypatch.setenv('BPE_PIX_FILL_PAIRS', '1')
    rng = random.Random(1300 + seed)
    alphabet = [256, 40, 256][seed]
    samples = random_corpus(rng, 300000, alphabet, [0.0, 0.2, 0.6][seed], rng.choice([9, 100]))
    if seed == 2:   # (one first token in most hot positions)
        samples = [np.where(np.arange(len(s)) % 2 == 0, 7, s).astype(np.int32) for s in samples]
    len16 = [1] * alphabet
    ids, off = _flat(samples)
    st = OracleState(ids, off, len16, alphabet)
    e = make_engine(samples, len16)
    e.set_mode('incremental')
    e.stats_enable(True)
    want = st.merge_until(0, 2, 60)
    got = e.merge_until(0, 2, 60)
    assert got == want, (got[:3], want[:3])
    assert e.samples() == st.samples()
    assert e.stats()['pix_merges'] > 0
