"""GPU parity: the HIP engine (through the C ABI) against the reference's golden vectors and the
oracle.  Bit-exact merge sequences and corpora are required everywhere."""
import hashlib
import random

import numpy as np
import pytest

from bpe_amd import pkg, run_engine
from golden_util import load_config2, load_small
from oracle import Corpus, OracleState

pytestmark = pytest.mark.gpu


def engine_case(case):
    c = Corpus()
    for s in case['samples']:
        c.add(s)
    e, merges = run_engine(c.samples, c.len16, case['opts'])
    return c, e, merges


def test_small_golden_cases():
    """All reference-generated small cases (spec inputs + 1500 seeded random corpora)."""
    bad = []
    for case in load_small():
        c, e, merges = engine_case(case)
        got = [list(m) for m in merges]
        if got != case['merges'] or e.samples() != case['final_ids']:
            bad.append((case['name'], got[:5], case['merges'][:5]))
        e.close()
        if len(bad) > 5:
            break
    assert not bad, bad


def test_config1_drop_in_numbers():
    """BASELINE config 1: 'aaabdaaabac', mergeUntil({min_weight:2})."""
    c = Corpus()
    c.add('aaabdaaabac')
    e, merges = run_engine(c.samples, c.len16, {'min_weight': 2})
    assert merges == [(0, 0, 2), (0, 1, 2), (4, 5, 2)]
    assert e.samples() == [[6, 2, 6, 0, 3]]


def random_corpus(rng, n_tokens, alphabet, run_bias, n_samples):
    """Seeded corpus with controllable run structure (runs exercise the X X skip rule)."""
    out = []
    per = max(1, n_tokens // n_samples)
    for _ in range(n_samples):
        L = rng.randint(0, 2 * per)
        toks = np.empty(L, np.int32)
        i = 0
        while i < L:
            t = rng.randrange(alphabet)
            k = 1 if rng.random() > run_bias else rng.randint(2, 12 if rng.random() < 0.9 else 900)
            toks[i:i + k] = t
            i += k
        out.append(toks[:L])
    return out


@pytest.mark.parametrize('seed', range(12))
def test_random_vs_oracle(seed):
    rng = random.Random(seed)
    n_tokens = rng.choice([3000, 40000, 300000, 1500000])
    alphabet = rng.choice([2, 3, 5, 20, 95, 256, 300])
    samples = random_corpus(rng, n_tokens, alphabet, rng.choice([0.0, 0.05, 0.3, 0.7]),
                            rng.choice([1, 3, 17, 200]))
    len16 = [rng.choice([1, 1, 1, 2]) for _ in range(alphabet)]
    opts = {'max_iterations': rng.choice([20, 60]),
            'max_length': rng.choice([0, 0, 3, 4, 6]),
            'min_weight': rng.choice([0, 2, 3])}
    st = OracleState(np.concatenate(samples) if samples else np.zeros(0, np.int32),
                     np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64),
                     len16, alphabet)
    want = st.merge_until(opts['max_length'], opts['min_weight'], opts['max_iterations'])
    e, got = run_engine(samples, len16, opts)
    assert got == want
    assert e.samples() == st.samples()


@pytest.mark.parametrize('n', [9, 10, 1023, 1024, 65536 * 3 + 7, 3_000_001])
def test_long_runs_cross_chunks_and_regions(n):
    """'x' * n (+ a breaker) — runs far longer than a chunk and than a region."""
    samples = [np.zeros(n, np.int32), np.array([0, 0, 1, 0, 0, 0], np.int32),
               np.concatenate([np.zeros(n // 3, np.int32), [1], np.zeros(n // 2, np.int32)]).astype(np.int32)]
    st = OracleState(np.concatenate(samples), np.array([0, n, n + 6, n + 6 + len(samples[2])],
                                                       np.int64), [1, 1], 2)
    want = st.merge_until(0, 0, 0)
    e, got = run_engine(samples, [1, 1], {})
    assert got == want
    assert e.samples() == st.samples()


def test_ties_need_r3():
    """Many pairs with equal W and equal a+b: the earliest W-th occurrence must win (R3)."""
    rng = random.Random(5)
    for trial in range(20):
        V = rng.choice([12, 40, 300])
        B = V - 1                              # breaker token, keeps pairs apart
        s = rng.randint(V // 3, V - 2)         # common a+b
        pairs = [(i, s - i) for i in range(0, s + 1) if s - i < B and i < B]
        rng.shuffle(pairs)
        pairs = pairs[:rng.randint(2, len(pairs))]
        r = rng.randint(1, 5)
        seq = []
        events = [p for p in pairs for _ in range(r)]
        rng.shuffle(events)
        for a, b in events:
            seq += [a, b, B]
        samples = [np.array(seq, np.int32)]
        len16 = [1] * V
        st = OracleState(samples[0], np.array([0, len(seq)], np.int64), len16, V)
        want = st.merge_until(0, -1, 30)
        e, got = run_engine(samples, len16, {'min_weight': -1, 'max_iterations': 30})
        assert got == want, trial
        assert e.samples() == st.samples()


def test_latin1_ingest_matches_host_mapping():
    data = pkg.synth_latin1(3 << 20, seed=99, A=200, base=40)
    e = pkg.Engine(0)
    cmap, nt, hist = e.add_latin1(data, sample_bytes=1 << 20)
    first = {}
    for b in data.tolist():
        if b not in first:
            first[b] = len(first)
    assert nt == len(first)
    for b, i in first.items():
        assert cmap[b] == i
    assert hist.sum() == data.size
    ids, off = e.read_corpus()
    assert off.tolist() == [0, 1 << 20, 2 << 20, 3 << 20]
    assert np.array_equal(ids, cmap[data])


def test_config2_golden():
    """BASELINE config 2: 10 MiB ASCII, 1000 merges — merge list and final-corpus SHA-256 equal
    the reference's own run (tests/golden/config2.json)."""
    g = load_config2()
    if g is None:
        pytest.skip('config2 fixture not generated')
    data = pkg.synth_latin1(g['total'], seed=g['seed'], A=g['A'], base=g['base'])
    e = pkg.Engine(0)
    cmap, nt, hist = e.add_latin1(data, sample_bytes=g['sample'])
    assert nt == g['char_count']
    merges = e.merge_until(0, g['min_weight'], g['max_iterations'])
    assert [list(m) for m in merges] == g['merges']
    ids, off = e.read_corpus()
    h = hashlib.sha256()
    for i in range(len(off) - 1):
        h.update(np.append(ids[off[i]:off[i + 1]], -1).astype('<i4').tobytes())
    assert h.hexdigest() == g['final_ids_sha256']


@pytest.mark.slow
def test_config3_prefix_vs_oracle():
    """1 GiB, 256-char corpus (BASELINE config 3): first merges equal the C restatement; apply
    removes exactly W tokens each time."""
    n = 1 << 30
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    e = pkg.Engine(0)
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    ids = cmap[data]
    del data
    off = np.arange(0, n + 1, 1 << 20, dtype=np.int64)
    st = OracleState(ids, off, [1] * nt, nt, extra=64)
    del ids
    for _ in range(3):
        want = st.find_next_merge(0, 2)
        got = e.find_next_merge(0, 2)
        assert got == want
        c = st.n_tokens
        st.apply_merge(want[0], want[1])
        assert e.apply_merge(got[0], got[1], c) == got[2]
    assert e.corpus_size()[1] == st.off[-1]


def test_restore_style_apply_and_append_after_merges():
    """applyMerge without findNextMerge (restoreMerge, core.ts:477-494), then addToCorpus on a
    merged corpus (forces a compaction), then more merges — all against the oracle."""
    rng = random.Random(11)
    V = 40
    samples = [np.array([rng.randrange(V) for _ in range(rng.randint(0, 3000))], np.int32)
               for _ in range(9)]
    len16 = [1] * V
    st = OracleState(np.concatenate(samples), np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64), len16, V)
    e = pkg.Engine(0)
    for i in range(V):
        e.set_token_len16(i, 1)
    for s in samples:
        e.add_sample(s)
    # replay a merge log without counting (restoreMerge)
    log = st.merge_until(0, 2, 8)
    for k, (a, b, w) in enumerate(log):
        assert e.apply_merge(a, b, V + k) == w
    assert e.samples() == st.samples()
    # append a new sample to the merged corpus, then keep merging from both sides
    extra = np.array([rng.randrange(V) for _ in range(5000)], np.int32)
    e.add_sample(extra)
    flat, off = st.ids.copy(), st.off.copy()
    st2 = OracleState(np.concatenate([flat, extra]), np.append(off, off[-1] + len(extra)),
                      list(st.len16[:st.n_tokens]), st.n_tokens)
    want = st2.merge_until(0, 2, 25)
    got = []
    n_tokens = st.n_tokens
    for _ in range(25):
        m = e.find_next_merge(0, 2)
        if m is None:
            break
        assert e.apply_merge(m[0], m[1], n_tokens) == m[2]
        n_tokens += 1
        got.append(m)
    assert got == want
    assert e.samples() == st2.samples()


def test_compaction_under_heavy_merging():
    """'ab' * 1.5M: the first merge halves the corpus, which triggers the dead-slot compaction."""
    n = 3_000_000
    sample = np.tile(np.array([0, 1], np.int32), n // 2)
    st = OracleState(sample, np.array([0, n], np.int64), [1, 1], 2, extra=64)
    want = st.merge_until(0, 2, 0)
    e, got = run_engine([sample], [1, 1], {})
    assert got == want
    assert e.samples() == st.samples()


@pytest.mark.parametrize('early', [1, 2, 3])
def test_ties_resolved_from_the_corpus_tail(early):
    """R3 ties in a corpus larger than the device loop's tail window (8192 chunks): `early` of the
    tied pairs occur only in the first quarter.  One such pair wins from the window alone; two or
    more need the full pass (the loop hands the iteration to the host path)."""
    rng = np.random.default_rng(early)
    n, V = 4_000_000, 3000
    seq = rng.integers(0, V, n, dtype=np.int32)      # filler: every filler pair is rare
    S = 2 * V + 90                                  # common a + b of the tied pairs
    pairs = [(V + i, S - V - i) for i in range(6)]   # ids in [V, V + 90]
    W = 40
    for k, (a, b) in enumerate(pairs):
        hi = n // 4 if k < early else n - 200      # (the window is the last ~2.1M slots)
        pos = rng.choice(np.arange(4, hi, 7), W, replace=False)
        if k >= early:
            pos[0] = n - 14 - 7 * k                 # one occurrence in the last chunks
        for p in pos:
            seq[p - 1], seq[p], seq[p + 1], seq[p + 2] = V + 95, a, b, V + 96
    # (the breakers V+95 / V+96 keep the inserted pairs apart; their own pairs stay below W)
    n_tok = V + 97
    len16 = [1] * n_tok
    st = OracleState(seq, np.array([0, n], np.int64), len16, n_tok)
    want = st.merge_until(0, 2, 8)
    e, got = run_engine([seq], len16, {'min_weight': 2, 'max_iterations': 8})
    assert got == want
    assert e.samples() == st.samples()


def _flat(samples):
    ids = np.concatenate(samples).astype(np.int32) if samples else np.zeros(0, np.int32)
    return ids, np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64)


@pytest.mark.parametrize('seed', range(6))
def test_apply_merges_replays_a_merge_log(seed):
    """restoreMerge replay (core.ts:477-494) through bpe_apply_merges: the apply-only passes rewrite
    the corpus exactly as the oracle's sequential applyMerge, with replacement counts == W; with
    count_after, the merging that follows continues exactly as the oracle's."""
    rng = random.Random(100 + seed)
    alphabet = rng.choice([2, 3, 20, 256, 300])
    samples = random_corpus(rng, rng.choice([5000, 200000, 2500000]), alphabet,
                            rng.choice([0.0, 0.3, 0.7]), rng.choice([1, 5, 60]))
    len16 = [rng.choice([1, 2]) for _ in range(alphabet)]
    ids, off = _flat(samples)
    st = OracleState(ids, off, len16, alphabet)
    log = st.merge_until(0, 2, 40)
    more = st.merge_until(0, 2, 10)
    abc = [(a, b, alphabet + i) for i, (a, b, _) in enumerate(log)]
    e = pkg.Engine(0)
    for i, l in enumerate(len16):
        e.set_token_len16(i, l)
    for s in samples:
        e.add_sample(s)
    count_after = seed % 2 == 0
    rep = e.apply_merges(abc, count_after=count_after)
    assert rep == [w for _, _, w in log]
    st2 = OracleState(ids, off, len16, alphabet)
    for a, b, _ in log:
        st2.apply_merge(a, b)
    assert e.samples() == st2.samples()
    n_tokens = alphabet + len(log)
    got = []
    for _ in range(10):
        m = e.find_next_merge(0, 2)
        if m is None:
            break
        assert e.apply_merge(m[0], m[1], n_tokens) == m[2]
        n_tokens += 1
        got.append(m)
    assert got == more
    e.close()


def test_encode_samples_with_a_trained_merge_list():
    """Batch encodeToCode (core.ts:392-409) of unseen texts with the merges trained on another
    corpus: equal to applying the merges in order with the oracle."""
    rng = random.Random(7)
    alphabet = 40
    train = random_corpus(rng, 300000, alphabet, 0.3, 20)
    len16 = [1] * alphabet
    ids, off = _flat(train)
    log = OracleState(ids, off, len16, alphabet).merge_until(0, 2, 120)
    abc = [(a, b, alphabet + i) for i, (a, b, _) in enumerate(log)]
    texts = random_corpus(random.Random(8), 2_000_000, alphabet, 0.3, 300) + [np.zeros(0, np.int32)]
    got = pkg.encode_samples(texts, abc, len16)
    tid, toff = _flat(texts)
    st = OracleState(tid, toff, len16, alphabet)
    for a, b, _ in log:
        st.apply_merge(a, b)
    assert got == st.samples()


def test_runs_across_region_boundaries_from_a_fast_chunk():
    """x x | x y at every region boundary (two chunks per region): the trailing run of each
    region has even length, which only the exact path of the region's last chunk works out
    (RegionSum.trail_odd -> k_runs).  A wrong parity counts one (x, x) too many per boundary."""
    n = 1_500_000                                   # 5860 chunks: two per region
    rng = np.random.default_rng(3)
    seq = rng.integers(0, 3000, n, dtype=np.int32)
    x, y = 3000, 3001
    for r in range(1, (n + 1) // 512):
        p = 512 * r
        seq[p - 3:p + 2] = [3002, x, x, x, y]
    st = OracleState(seq, np.array([0, n], np.int64), [1] * 3003, 3003)
    want = st.merge_until(0, 2, 3)
    e, got = run_engine([seq], [1] * 3003, {'min_weight': 2, 'max_iterations': 3})
    assert got == want
    assert e.samples() == st.samples()


@pytest.mark.parametrize('mib,n,max_length', [(4, 600, 0), (3, 400, 5), (8, 1500, 0)])
def test_zipf_words_vs_oracle(mib, n, max_length):
    """Skewed corpus (bpe_synth_zipf): a 28-symbol alphabet whose merges soon
    build whole words, so most winning pairs are pairs of merged tokens (ids >= 256: the cold
    sketch, heavy buckets) and long equal-pair runs are rare.  After two exact passes in a row the
    engine keeps an exact table of every cold pair, refreshed merge by merge for the pairs touching
    the merged tokens.  mergeUntil against the C restatement: merges and final corpus bit-exact,
    and the exact passes stay few (the maintained table answers the rest)."""
    data = pkg.synth_zipf(mib << 20, seed=2024)
    e = pkg.Engine(0)
    e.stats_enable(True)
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    ids = cmap[data]
    off = np.arange(0, (mib << 20) + 1, 1 << 20, dtype=np.int64)
    st = OracleState(ids, off, [1] * nt, nt, extra=n + 8)
    want = st.merge_until(max_length, 2, n)
    got = e.merge_until(max_length, 2, n)
    assert got == [tuple(m) for m in want]
    flat, eoff = e.read_corpus()
    assert eoff.tolist() == st.off.tolist()
    assert np.array_equal(flat, st.ids[:st.off[-1]])
    assert e.stats()['exact_passes'] <= 10
