"""The device encoder (bpe_encoder_* / bpe_encode_batch, csrc/bpe_encode.hip): encodeToCode
(core.ts:392-409) for batches of texts, checked against

  - the reference's own encodeToVector outputs (tests/golden/small_cases.json `vectors`, made by
    running core.ts itself: oracle/gen_golden.py), and
  - the C restatement of the replay (oracle_encode: every merge in order, core.ts:404-406) on
    seeded random merge lists and texts, at every launch shape (k_encode<64/256/1024>) and on the
    apply-pass route (texts over ENCODE_LDS_TOKENS tokens, merge lists the greedy cannot take).

The CPU-only test at the bottom checks the merge-rank greedy itself (the kernel's algorithm,
restated in Python) against the replay, without a device.
"""
import numpy as np
import pytest

import oracle
from bpe_amd import pkg
from golden_util import char_weights, load_small, to_vector, token_table_after
from oracle import Corpus, OracleState

CASES = load_small()


def trained_merges(rng, alphabet, n_samples, sample_len, max_iterations=0, min_weight=2):
    """(a, b, c) merges of a reference-style training run (the oracle's mergeUntil)."""
    samples = [rng.integers(0, alphabet, size=rng.integers(0, sample_len + 1)).astype(np.int32)
               for _ in range(n_samples)]
    c = Corpus()
    for s in samples:
        c.add_ids(s)
    c.chars = list(range(alphabet))
    c.len16 = [1] * alphabet
    st = OracleState.from_corpus(c)
    merges = st.merge_until(None, min_weight, max_iterations)
    return [(a, b, alphabet + k) for k, (a, b, _w) in enumerate(merges)]


def random_texts(rng, alphabet, lengths):
    return [rng.integers(0, alphabet, size=l).astype(np.int32) for l in lengths]


def skewed_texts(rng, alphabet, lengths):
    """Texts with long runs and repeats (x == y pairs, chains across thread segments)."""
    out = []
    for l in lengths:
        t = np.empty(l, np.int32)
        i = 0
        while i < l:
            run = int(rng.integers(1, 40))
            t[i:i + run] = rng.integers(0, max(1, alphabet // 4))
            i += run
        out.append(t)
    return out


def check(enc, texts, merges):
    got = enc.encode(texts)
    want = oracle.encode(texts, merges)
    for k, (g, w) in enumerate(zip(got, want)):
        assert g.tolist() == w.tolist(), 'text %d (len %d)' % (k, len(texts[k]))


@pytest.mark.gpu
def test_reference_vectors_of_every_small_case():
    """encodeToVector of every training sample of the 1509 golden cases, through the device
    encoder, equals the vector the reference itself produced (core.ts:424-445)."""
    enc = pkg.Encoder(0)
    n_checked = 0
    try:
        for case in CASES:
            c = Corpus()
            for s in case['samples']:
                c.add(s)
            merges = [tuple(m) for m in case['merges']]
            table = token_table_after(c.chars, char_weights(c.samples, len(c.chars)), merges)
            if not table:
                continue
            enc.clear()
            abc = [(a, b, len(c.chars) + k) for k, (a, b, _w) in enumerate(merges)]
            if abc:
                enc.add_merges(abc)
            texts = [np.asarray([c.char_to_index[ch] for ch in s], np.int32) for s in case['samples']]
            got = enc.encode(texts)
            for g, expect in zip(got, case['vectors']):
                assert to_vector(g.tolist(), table) == expect, case['name']
                n_checked += 1
    finally:
        enc.close()
    assert n_checked > 1500


@pytest.mark.gpu
@pytest.mark.parametrize('seed', [1, 2, 3])
def test_random_texts_every_launch_shape(seed):
    rng = np.random.default_rng(seed)
    alphabet = [3, 12, 40][seed - 1]
    merges = trained_merges(rng, alphabet, 40, 300)
    assert len(merges) > 20
    cap = pkg.ENCODE_LDS_TOKENS
    lengths = [0, 1, 2, 3, 63, 64, 65, 200, 511, 512, 513, 1000, 4095, 4096, 4097, 9000,
               cap - 1, cap, cap + 1, 20000]
    texts = random_texts(rng, alphabet, lengths) + skewed_texts(rng, alphabet, lengths[:16])
    enc = pkg.Encoder(0, merges)
    enc.reset_stats()
    check(enc, texts, merges)
    st = enc.stats()
    long = sum(1 for t in texts if len(t) > cap)
    assert st['texts_replay'] == long
    assert st['texts_rank'] == sum(1 for t in texts if len(t) <= cap)
    assert st['steps'] > 0
    enc.close()


@pytest.mark.gpu
def test_many_short_texts_one_batch():
    """A batch of 5000 ragged short texts (the serving shape): one launch per shape."""
    rng = np.random.default_rng(7)
    merges = trained_merges(rng, 30, 200, 400)
    lengths = rng.integers(0, 700, size=5000)
    texts = random_texts(rng, 30, lengths)
    enc = pkg.Encoder(0, merges)
    check(enc, texts, merges)
    enc.close()


@pytest.mark.gpu
def test_runs_of_one_token():
    """x == y chains over whole texts (every thread walks back across earlier segments), with
    merges x x -> y, y y -> z, ... (core.spec.ts:91-140 shape: 'x' * 9 -> [xxxx, xxxx, x])."""
    merges = [(0, 0, 1), (1, 1, 2), (2, 2, 3), (3, 3, 4), (0, 1, 5), (4, 4, 6)]
    texts = [np.zeros(l, np.int32) for l in (2, 3, 9, 64, 65, 127, 511, 1023, 4096, 4097, 16384)]
    texts += [np.asarray(([0] * 5 + [1]) * 50, np.int32)]
    enc = pkg.Encoder(0, merges)
    check(enc, texts, merges)
    enc.close()


@pytest.mark.gpu
def test_merges_added_in_batches_and_cleared():
    rng = np.random.default_rng(11)
    merges = trained_merges(rng, 20, 60, 300)
    texts = random_texts(rng, 20, [50, 700, 3000, 12000])
    enc = pkg.Encoder(0)
    for i in range(0, len(merges), 7):   # restoreMerge-style growth, encoding in between
        enc.add_merges(merges[i:i + 7])
        assert enc.num_merges() == min(len(merges), i + 7)
        check(enc, texts, merges[:i + 7])
    enc.clear()
    assert enc.num_merges() == 0
    assert [t.tolist() for t in enc.encode(texts)] == [t.tolist() for t in texts]
    enc.close()


@pytest.mark.gpu
@pytest.mark.parametrize('m', [3000, 20000])
def test_synthetic_merge_lists_few_and_many_texts(m):
    """Random valid merge lists (c = a fresh id, inputs any earlier id): 3000 merges keep the
    table in LDS for a call of few texts, 20000 do not (the HBM table then); the same texts in a
    call of many (the HBM table)."""
    rng = np.random.default_rng(m)
    A = 60
    merges = [(int(rng.integers(0, A + k)), int(rng.integers(0, A + k)), A + k) for k in range(m)]
    # texts built from merged tokens' expansions, so that deep merges fire
    exp = [[i] for i in range(A)]
    for a, b, _c in merges:
        exp.append(exp[a] + exp[b] if len(exp[a]) + len(exp[b]) < 64 else exp[a])
    texts = []
    for l in [5, 50, 300, 600, 3000, 9000]:
        t = []
        while len(t) < l:
            t += exp[int(rng.integers(0, len(exp)))]
        texts.append(np.asarray(t[:l], np.int32))
    enc = pkg.Encoder(0, merges)
    check(enc, texts, merges)
    check(enc, texts * 60, merges)   # 360 texts: past the few-texts form
    enc.close()


@pytest.mark.gpu
def test_list_the_greedy_cannot_take_is_replayed():
    """A hand-made list where a merge's new token is an earlier merge's input (fromJSON of a
    non-reference file): the encoder replays it in order, as replaceAll does."""
    merges = [(0, 1, 2), (2, 0, 3), (1, 1, 0), (0, 2, 4)]   # c = 0 is an input of merge 0
    rng = np.random.default_rng(3)
    texts = random_texts(rng, 3, [10, 100, 1000]) + [np.asarray([1, 1, 0, 1, 1, 1, 0, 1], np.int32)]
    enc = pkg.Encoder(0, merges)
    enc.reset_stats()
    check(enc, texts, merges)
    assert enc.stats()['texts_rank'] == 0
    enc.close()


@pytest.mark.gpu
def test_large_call_in_groups(monkeypatch):
    """A call of more than 2 x 2^23 input tokens goes through the pipelined groups
    (encode_groups): the same ids and offsets as the one-group form, the reference replay on texts
    around every group boundary, and a bad id in a late group refused."""
    rng = np.random.default_rng(21)
    merges = trained_merges(rng, 30, 200, 400)
    lengths = rng.integers(0, 1500, size=24000)
    lengths[100] = pkg.ENCODE_LDS_TOKENS                      # (every launch shape)
    flat = np.concatenate([np.full(5, 7, np.int32),           # (off[0] > 0)
                           rng.integers(0, 30, size=int(lengths.sum())).astype(np.int32)])
    off = np.concatenate([[0], np.cumsum(lengths)]).astype(np.int64) + 5
    assert off[-1] - off[0] >= 2 * (1 << 23)
    enc = pkg.Encoder(0, merges)
    got, got_off = enc.encode_flat(flat, off)
    monkeypatch.setenv('BPE_ENCODE_ONE_GROUP', '1')
    one, one_off = enc.encode_flat(flat, off)
    monkeypatch.delenv('BPE_ENCODE_ONE_GROUP')
    assert np.array_equal(got_off, one_off) and np.array_equal(got, one)
    # texts around each group's first text (three groups by default; BPE_ENCODE_GROUPS) and a
    # spread of others
    T = int(off[-1] - off[0])
    starts = np.searchsorted(off - off[0], [T // 3, 2 * T // 3, T // 2, 1 << 23, 1 << 24])
    pick = sorted({int(k) for s in starts for k in range(max(0, s - 3), min(len(lengths), s + 3))} |
                  set(range(0, 24000, 997)) | {100, 23999})
    texts = [flat[off[k]:off[k + 1]] for k in pick]
    want = oracle.encode(texts, merges)
    for k, w in zip(pick, want):
        assert got[got_off[k]:got_off[k + 1]].tolist() == w.tolist(), k
    bad = flat.copy()
    bad[off[23000] + 1] = -3
    with pytest.raises(pkg.BpeError, match='out of range'):
        enc.encode_flat(bad, off)
    again, again_off = enc.encode_flat(flat, off)
    assert np.array_equal(again_off, got_off) and np.array_equal(again, got)
    enc.close()


@pytest.mark.gpu
def test_bad_ids_are_refused():
    enc = pkg.Encoder(0, [(0, 1, 2)])
    with pytest.raises(pkg.BpeError, match='out of range'):
        enc.encode([np.asarray([0, pkg.MAX_VOCAB], np.int32)])
    with pytest.raises(pkg.BpeError, match='out of range'):   # (checked on the device)
        enc.encode([np.asarray([0, 1, 0], np.int32), np.asarray([3, -1, 2, 0], np.int32)])
    with pytest.raises(pkg.BpeError, match='out of range'):   # (the replay route: on the host)
        enc.encode([np.asarray([0, 1] * 9000 + [-5], np.int32)])
    # the encoder is still usable after a refused call
    assert [t.tolist() for t in enc.encode([np.asarray([0, 1, 0, 1], np.int32)])] == [[2, 2]]
    with pytest.raises(pkg.BpeError, match='out of range'):
        enc.add_merges([(0, -1, 3)])
    enc.close()


# ---- CPU: the merge-rank greedy (the kernel's algorithm) against the replay --------------------

def greedy_encode(text, merges):
    """Python restatement of k_encode: take the lowest rank present, flag its counted occurrences
    segment by segment (walk back for the chain parity), delete each counted i + 1."""
    rank = {}
    for r, (a, b, _c) in enumerate(merges):
        rank.setdefault((a, b), r)
    tok = list(text)
    INF = 1 << 30
    while True:
        rk = [rank.get((tok[i], tok[i + 1]), INF) for i in range(len(tok) - 1)] + [INF]
        r = min(rk) if tok else INF
        if r == INF:
            return tok
        c = merges[r][2]
        n = len(tok)
        seg = max(1, (n + 6) // 7)           # 7 "threads"
        fl = [False] * n
        for s in range(0, n, seg):
            d = 0
            j = s - 1
            while j >= 0 and rk[j] == r:
                d += 1
                j -= 1
            for i in range(s, min(n, s + seg)):
                m = rk[i] == r
                fl[i] = m and d % 2 == 0
                d = d + 1 if m else 0
        tok = [c if fl[i] else tok[i] for i in range(n) if not (i > 0 and fl[i - 1])]


@pytest.mark.parametrize('seed', range(6))
def test_greedy_equals_replay_cpu(seed):
    rng = np.random.default_rng(100 + seed)
    alphabet = [2, 3, 5, 8, 16, 30][seed]
    merges = trained_merges(rng, alphabet, 20, 120)
    texts = random_texts(rng, alphabet, rng.integers(0, 200, size=30)) + \
        skewed_texts(rng, alphabet, [50, 150, 300])
    want = oracle.encode(texts, merges)
    for t, w in zip(texts, want):
        assert greedy_encode(t.tolist(), merges) == w.tolist()


@pytest.mark.parametrize('seed', range(6))
def test_cpu_rank_greedy_equals_replay(seed):
    """The device encoder's CPU baseline (oracle/bpe_cpu_encode.cc: rank-greedy with a heap of
    (rank, position), OpenMP over texts) against the replay, on several thread counts."""
    rng = np.random.default_rng(300 + seed)
    alphabet = [2, 3, 5, 8, 16, 30][seed]
    merges = trained_merges(rng, alphabet, 20, 150)
    texts = random_texts(rng, alphabet, rng.integers(0, 300, size=200)) + \
        skewed_texts(rng, alphabet, [1, 2, 50, 150, 700])
    want = oracle.encode(texts, merges)
    off = np.zeros(len(texts) + 1, np.int64)
    np.cumsum([len(t) for t in texts], out=off[1:])
    ids = np.concatenate(texts).astype(np.int32)
    for threads in (1, 3):
        got, oo, used = oracle.cpu_encode_flat(ids, off, merges, threads=threads)
        assert used == threads
        for k, w in enumerate(want):
            assert got[oo[k]:oo[k + 1]].tolist() == w.tolist(), (threads, k)
