"""GPU parity: the HIP engine (through the C ABI) against the reference's golden vectors and the
oracle.  Bit-exact merge sequences and corpora are required everywhere."""
import hashlib
import random

import numpy as np
import pytest

from bpe_amd import MODES, pkg, run_engine
from golden_util import load_config2, load_config3_prefix, load_small
from oracle import Corpus, CpuMT, OracleState

pytestmark = pytest.mark.gpu


def engine_case(case, mode='host'):
    c = Corpus()
    for s in case['samples']:
        c.add(s)
    e, merges = run_engine(c.samples, c.len16, case['opts'], mode=mode)
    return c, e, merges


@pytest.mark.parametrize('mode', MODES)
def test_small_golden_cases(mode):
    """All reference-generated small cases (spec inputs + 1500 seeded random corpora), through
    findNextMerge/applyMerge and through mergeUntil's device-resident loop."""
    bad = []
    for case in load_small():
        c, e, merges = engine_case(case, mode)
        got = [list(m) for m in merges]
        if got != case['merges'] or e.samples() != case['final_ids']:
            bad.append((case['name'], got[:5], case['merges'][:5]))
        e.close()
        if len(bad) > 5:
            break
    assert not bad, bad


@pytest.mark.parametrize('mode', MODES)
def test_config1_drop_in_numbers(mode):
    """BASELINE config 1: 'aaabdaaabac', mergeUntil({min_weight:2})."""
    c = Corpus()
    c.add('aaabdaaabac')
    e, merges = run_engine(c.samples, c.len16, {'min_weight': 2}, mode=mode)
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


@pytest.mark.parametrize('mode', MODES)
@pytest.mark.parametrize('seed', range(12))
def test_random_vs_oracle(seed, mode):
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
    e, got = run_engine(samples, len16, opts, mode=mode)
    assert got == want
    assert e.samples() == st.samples()
    check_sample_index(e, st.samples(), rng)


def check_sample_index(e, want, rng):
    """bpe_sample_lengths / bpe_read_samples (the db twin's row write-back) against the expected
    samples: every length, and a random selection read back in a random order."""
    assert e.sample_lengths().tolist() == [len(s) for s in want]
    idx = [rng.randrange(len(want)) for _ in range(min(50, 2 * len(want)))] if want else []
    ids, off = e.read_samples(idx)
    assert [ids[off[k]:off[k + 1]].tolist() for k in range(len(idx))] == [list(want[i]) for i in idx]


@pytest.mark.parametrize('mode', MODES)
@pytest.mark.parametrize('seed', range(3))
def test_only_cold_pairs(seed, mode):
    """A corpus of ids >= 256 only: no hot pair exists, so the best hot key is empty and every
    candidate hides in the cold sketch.  The device loop must hand such iterations to the exact
    counts instead of stopping (core.ts:312 returns null only when no pair exists at all)."""
    rng = random.Random(300 + seed)
    V = 256 + rng.choice([3, 20, 60])
    samples = [np.array([rng.randrange(256, V) for _ in range(rng.randint(0, 4000))], np.int32)
               for _ in range(rng.choice([1, 7]))]
    len16 = [1] * V
    ids, off = np.concatenate(samples), np.concatenate([[0], np.cumsum([len(s) for s in samples])])
    st = OracleState(ids, off.astype(np.int64), len16, V)
    want = st.merge_until(0, 2, 12)
    e, got = run_engine(samples, len16, {'max_iterations': 12}, mode=mode)
    assert got == want
    assert e.samples() == st.samples()


@pytest.mark.parametrize('mode', MODES)
@pytest.mark.parametrize('n', [9, 10, 1023, 1024, 65536 * 3 + 7, 3_000_001])
def test_long_runs_cross_chunks_and_regions(n, mode):
    """'x' * n (+ a breaker) — runs far longer than a chunk and than a region."""
    samples = [np.zeros(n, np.int32), np.array([0, 0, 1, 0, 0, 0], np.int32),
               np.concatenate([np.zeros(n // 3, np.int32), [1], np.zeros(n // 2, np.int32)]).astype(np.int32)]
    st = OracleState(np.concatenate(samples), np.array([0, n, n + 6, n + 6 + len(samples[2])],
                                                       np.int64), [1, 1], 2)
    want = st.merge_until(0, 0, 0)
    e, got = run_engine(samples, [1, 1], {}, mode=mode)
    assert got == want
    assert e.samples() == st.samples()


@pytest.mark.parametrize('mode', MODES)
def test_ties_need_r3(mode):
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
        e, got = run_engine(samples, len16, {'min_weight': -1, 'max_iterations': 30}, mode=mode)
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
    # encodeToVector of every sample (core.ts:424-445) on the device encoder: the 10 raw samples
    # replayed through the merge list by apply-only passes (encode_samples), then compactVectorIndex
    # from the reference's weight bookkeeping; hashed as the reference's own run was
    from test_oracle_golden import config2_vectors
    raw = cmap[data].astype(np.int32)
    samples = [raw[o:o + g['sample']] for o in range(0, g['total'], g['sample'])]
    abc = [(a, b, nt + i) for i, (a, b, _) in enumerate(merges)]
    enc = pkg.encode_samples(samples, abc, [1] * nt)
    vec, n_vec = config2_vectors(enc, np.bincount(raw, minlength=nt), merges)
    assert n_vec == g['vectors_len']
    assert vec == g['vectors_sha256']


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
    g = load_config3_prefix()
    if g is not None:   # the reference's own first merges (tests/golden/config3_prefix.json)
        assert nt == g['char_count']
    for _ in range(3):
        want = st.find_next_merge(0, 2)
        got = e.find_next_merge(0, 2)
        assert got == want
        c = st.n_tokens
        st.apply_merge(want[0], want[1])
        assert e.apply_merge(got[0], got[1], c) == got[2]
        if g is not None:
            assert list(got) == g['merges'][_]
    assert e.corpus_size()[1] == st.off[-1]
    if g is not None:
        assert e.corpus_size()[1] == g['live_tokens_after']


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


@pytest.mark.parametrize('mode', MODES)
def test_lds_counters_past_16_bits(mode):
    """Pairs so frequent that every workgroup's 16-bit LDS counters pass 0x4000 many times in one
    pass (each workgroup sees ~30 K of each pair here): a hot pair on the fast path, a cold pair in
    its sketch bucket, a hot/cold mix, and one long run counted by the exact path.  The round-end
    overflow screen and the sweep to the global spill (lds_sweep) must keep every count exact."""
    n = 8 << 20
    samples = [np.tile(np.array([0, 1], np.int32), n // 2),
               np.tile(np.array([300, 301], np.int32), n // 2),
               np.tile(np.array([2, 300], np.int32), n // 2),
               np.full(n, 3, np.int32)]
    ids, off = _flat(samples)
    len16 = [1] * 302
    st = OracleState(ids, off, len16, 302, extra=64)
    want = st.merge_until(0, 2, 6)
    e, got = run_engine(samples, len16, {'max_iterations': 6}, mode=mode)
    assert got == want
    assert [m[2] for m in got[:2]] == [n // 2, n // 2]
    assert e.samples() == st.samples()


@pytest.mark.parametrize('mode', MODES)
def test_unscreened_passes_from_the_counts_bound(mode):
    """The device loop's passes without the LDS overflow screen (LoopCtl::unscreened: adds that
    return nothing), taken only while (largest table bin) + 2 W < 2^16.  'ab' x 2^19 makes a chain
    of X X merges whose W halves from 2^19 (screened passes: a workgroup's counters pass 16 bits),
    then a random text's merges (counts ~2 K: unscreened), so one batch switches mid-way; a long
    run of one token (the exact path's adds) rides along.  100 base ids, so the merged tokens stay
    hot (a cold X X chain would send the loop to the maintained state).  Merges and corpus equal
    the oracle's."""
    rng = np.random.default_rng(7)
    samples = [np.tile(np.array([0, 1], np.int32), 1 << 19),
               rng.integers(2, 42, size=3 << 20).astype(np.int32),
               np.full(70000, 42, np.int32)]
    ids, off = _flat(samples)
    len16 = [1] * 100
    st = OracleState(ids, off, len16, 100, extra=256)
    want = st.merge_until(0, 2, 90)
    e, got = run_engine(samples, len16, {'max_iterations': 90}, mode=mode, stats=True)
    assert got == want
    assert [m[2] for m in got[:3]] == [1 << 19, 1 << 18, 1 << 17]
    assert e.samples() == st.samples()
    if mode == 'loop':
        s = e.stats()
        # (the chain's first passes screened: W + 2 W passes 2^16 until W = 2^14)
        assert 0 < s['unscreened_passes'] <= 90 - 4, s
    e.close()


@pytest.mark.parametrize('mode', MODES)
def test_compaction_under_heavy_merging(mode):
    """'ab' * 1.5M: the first merge halves the corpus, which triggers the dead-slot compaction."""
    n = 3_000_000
    sample = np.tile(np.array([0, 1], np.int32), n // 2)
    st = OracleState(sample, np.array([0, n], np.int64), [1, 1], 2, extra=64)
    want = st.merge_until(0, 2, 0)
    e, got = run_engine([sample], [1, 1], {}, mode=mode, stats=True)
    assert got == want
    assert e.samples() == st.samples()
    if mode == 'pix':       # runs of 1.5M: the first merges walk too far and go to the stream
        s = e.stats()
        assert s['pix_host'] >= 1 or s['iterations'] > s['pix_merges'], s


@pytest.mark.parametrize('mode', MODES)
@pytest.mark.parametrize('early', [1, 2, 3])
def test_ties_of_cold_pairs_in_a_large_corpus(early, mode):
    """R3 ties of cold pairs (ids >= 256) in a corpus larger than the device loop's tail window:
    `early` of the tied pairs occur only in the first quarter.  Their sketch buckets are heavy, so
    the device loop hands these iterations to the host path (exact pass + full tie pass)."""
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
    e, got = run_engine([seq], len16, {'min_weight': 2, 'max_iterations': 8}, mode=mode)
    assert got == want
    assert e.samples() == st.samples()


def tail_tie_corpus(early, n=4_000_000, W=200, seed=0):
    """Six hot pairs (a, b) with a + b = 11 and count W each (R3 ties: equal W, equal c_index),
    in a filler of hot ids 12..239 whose pairs stay far below W.  The first `early` tied pairs
    occur only in the first quarter of the corpus, before the device loop's tail window (the last
    ~2M slots); the others occur all over, once in the last chunks.  Breakers drawn from 240..255
    around every inserted pair keep the pairs of merged tokens (cold ids) rare, so no sketch
    bucket turns heavy and the device loop decides every tie itself."""
    rng = np.random.default_rng(seed + early)
    seq = rng.integers(12, 240, n, dtype=np.int32)
    pairs = [(k, 11 - k) for k in range(6)]
    grid = np.arange(4, n - 200, 7)
    perm = rng.permutation(len(grid))
    early_grid = perm[grid[perm] < n // 4]
    late_grid = perm[grid[perm] >= n // 4]
    used_e = used_l = 0
    for k, (a, b) in enumerate(pairs):
        if k < early:
            pos = grid[early_grid[used_e:used_e + W]]
            used_e += W
        else:
            pos = grid[late_grid[used_l:used_l + W]]
            used_l += W
            pos[0] = n - 14 - 7 * k                    # one occurrence in the last chunks
        for p in pos:
            seq[p - 1] = 240 + rng.integers(0, 16)
            seq[p], seq[p + 1] = a, b
            seq[p + 2] = 240 + rng.integers(0, 16)
    return seq


@pytest.mark.parametrize('mode', MODES)
@pytest.mark.parametrize('early', [0, 1, 2, 3])
def test_ties_resolved_from_the_corpus_tail(early, mode):
    """The device loop's R3 tail window (k_tie tail mode + k_decide phase 1,
    csrc/bpe_kernels.hip.h) against the oracle, with each of its branches asserted through the
    engine's counters: every tied pair in the window (decided there), the lone pair missing from
    it (it wins: its last occurrence is earlier than every window occurrence), and two or more
    missing (the iteration goes to the host path's full tie pass).  Reference: core.ts:294-305."""
    seq = tail_tie_corpus(early)
    n = len(seq)
    len16 = [1] * 256
    st = OracleState(seq, np.array([0, n], np.int64), len16, 256)
    want = st.merge_until(0, 2, 8)
    e, got = run_engine([seq], len16, {'min_weight': 2, 'max_iterations': 8}, mode=mode,
                        stats=True)
    assert got == want
    assert [m[2] for m in got[:6]] == [200] * 6 and sorted(m[0] + m[1] for m in got[:6]) == [11] * 6
    assert e.samples() == st.samples()
    s = e.stats()
    if mode == 'pix':       # every merge on the index, R3 from the candidates' lists
        assert s['pix_merges'] == len(got) and s['pix_host'] == 0, s
    if mode == 'loop':
        assert s['exact_passes'] == 0, s
        if early == 0:      # every tie decided from the window
            assert s['tie_tail'] >= 5 and s['tie_lone'] == 0 and s['loop_host'] == 0, s
        elif early == 1:    # the lone missing pair wins, then the window decides the rest
            assert s['tie_lone'] == 1 and s['tie_tail'] >= 5 and s['loop_host'] == 0, s
        else:               # two or more missing: handed to the host path's full pass
            assert s['loop_host'] >= 1, s


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


@pytest.mark.parametrize('mode', MODES)
def test_runs_across_region_boundaries_from_a_fast_chunk(mode):
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
    e, got = run_engine([seq], [1] * 3003, {'min_weight': 2, 'max_iterations': 3}, mode=mode)
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


@pytest.mark.slow
def test_zipf_maintained_rows_past_16_bits():
    """256 MiB of Zipf words (a workgroup holds 1 MiB of it), so that in the maintained state the
    merge pass's LDS rows (MODE_INCR: the pairs (a, y), (b, y), (x, a), (x, b) of the merge
    (a, b)) of frequent tokens pass 0x4000 in a workgroup: the round's overflow screen and the
    rows' sweep must keep every count exact.  mergeUntil against the multi-threaded CPU
    restatement: every merge and the final corpus."""
    mib, n = 256, 300
    data = pkg.synth_zipf(mib << 20, seed=77)
    e = pkg.Engine(0)
    e.stats_enable(True)
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    ids = cmap[data]
    del data
    off = np.arange(0, (mib << 20) + 1, 1 << 20, dtype=np.int64)
    cpu = CpuMT(ids, off, [1] * nt, nt, threads=16, extra=n + 8)
    del ids
    want = cpu.merge_until(0, 2, n)
    got = e.merge_until(0, 2, n)
    assert got == want
    flat, eoff = e.read_corpus()
    cflat, coff = cpu.read()
    assert np.array_equal(eoff, coff) and np.array_equal(flat, cflat)
    assert e.stats()['fused_passes'] > 0, e.stats()


def test_cold_table_rebuilt_from_itself(monkeypatch):
    """The maintained cold table, when too full or mostly dead claims, is rebuilt from its own live
    claims (round 5, cold_rebuild) instead of by an exact pass over the corpus and table-state
    passes until the maintained state is entered again (BPE_COLD_REBUILD=0, the earlier path):
    the same merges and final corpus, fewer exact passes, more merges in the maintained state."""
    data = pkg.synth_zipf(256 << 20, seed=31)
    runs = {}
    for flag in ('0', '1'):
        monkeypatch.setenv('BPE_COLD_REBUILD', flag)
        e = pkg.Engine(0)
        e.stats_enable(True)
        e.add_latin1(data, sample_bytes=1 << 20)
        got = e.merge_until(0, 2, 3000)
        flat, off = e.read_corpus()
        runs[flag] = (got, flat, off, e.stats())
        e.close()
    assert runs['1'][0] == runs['0'][0]
    assert np.array_equal(runs['1'][1], runs['0'][1]) and np.array_equal(runs['1'][2], runs['0'][2])
    st1, st0 = runs['1'][3], runs['0'][3]
    assert st1['cold_rebuilds'] >= 1 and st0['cold_rebuilds'] == 0, (st1, st0)
    assert st1['exact_passes'] < st0['exact_passes'], (st1, st0)
    assert st1['fused_passes'] > st0['fused_passes'], (st1, st0)


@pytest.mark.slow
def test_cold_pair_count_beyond_2_32():
    """A cold pair whose count exceeds 2^32 (the reference's Map counts are JS numbers, exact to
    2^53, core.ts:280-292): 'x' * (2^33 + 2) ingested as token id 300, so (300, 300) occurs
    2^32 + 1 times (leftmost non-overlapping, core.ts:285-290).  Its sketch bucket is heavy, so
    the exact cold-pair table counts it (64-bit counts), and the run crosses every region (k_runs
    adds the pairs the waves could not see).  mergeUntil must give W = 2^32 + 1, 2^31, 2^30, 2^29."""
    n = (1 << 33) + 2
    data = np.full(n, ord('x'), np.uint8)
    e = pkg.Engine(0)
    for i in range(301):
        e.set_token_len16(i, 1)
    cmap = np.full(256, -1, np.int32)
    cmap[ord('x')] = 300
    _, nt, hist = e.add_latin1(data, sample_bytes=0, char_to_id=cmap, n_tokens=301)
    del data
    assert nt == 301 and hist[ord('x')] == n
    got = e.merge_until(0, 2, 4)
    assert got == [(300, 300, (1 << 32) + 1), (301, 301, 1 << 31), (302, 302, 1 << 30),
                   (303, 303, 1 << 29)]
    assert e.corpus_size() == (1, n - sum(m[2] for m in got))
    e.close()


@pytest.mark.slow
def test_c3_dynamics_through_the_device_loop():
    """The bench's timed path (bpe_merge_until: k_step_loop, k_select_multi, k_decide, the
    tail-window tie pass, the dead-slot compaction) over the dynamics of BASELINE config 3, scaled
    down: a 32 MiB uniform 256-char corpus (xorshift32 seed 12345, 1 MiB samples), 3000 merges.
    Each merge removes ~W/N = 1/65536 of the stream, so the run crosses the 1 % compaction, and
    about one iteration in ten is an R3 tie.  Checked against the multi-threaded CPU restatement
    (itself pinned to the reference's fixtures): every merge and the final corpus."""
    n = 32 << 20
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    e = pkg.Engine(0)
    e.stats_enable(True)
    cmap, nt, _ = e.add_latin1(data, sample_bytes=1 << 20)
    ids = cmap[data]
    del data
    off = np.arange(0, n + 1, 1 << 20, dtype=np.int64)
    cpu = CpuMT(ids, off, [1] * nt, nt, threads=16, extra=4096)
    del ids
    want = cpu.merge_until(0, 2, 3000)
    got = e.merge_until(0, 2, 3000)
    s = e.stats()
    assert got == want
    flat, eoff = e.read_corpus()
    cflat, coff = cpu.read()
    assert np.array_equal(eoff, coff) and np.array_equal(flat, cflat)
    assert s['compactions'] >= 1, s
    assert s['tie_tail'] >= 10, s
    assert s['tie_passes'] >= s['tie_tail'], s
