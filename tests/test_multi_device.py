"""One corpus sharded over several shards behind ONE context (bpe_create_multi, include/bpe.h):
the drop-in's BPE_NUM_GPUS path.  On the one-GPU test box the shards share device 0 and exchange
their tables through a device kernel (BPE_REDUCE_HOST: bpe_sum_shards, ordered by events), or a
1-rank RCCL communicator; the RCCL exchange over several devices runs only where they exist.
Every result must equal the oracle's on the whole corpus."""
import os
import random

import numpy as np
import pytest

from bpe_amd import pkg
from golden_util import load_small
from oracle import Corpus, OracleState
from test_gpu_parity import check_sample_index, random_corpus

pytestmark = pytest.mark.gpu

# (RCCL's warnings, if a communicator fails to come up, land in the failing test's captured output)
os.environ.setdefault('NCCL_DEBUG', 'WARN')


def multi_engine(samples, len16, n_shards, mode_devices=None):
    e = pkg.Engine(devices=mode_devices or [0] * n_shards, reduce='host')
    for i, l in enumerate(len16):
        e.set_token_len16(i, l)
    for s in samples:
        e.add_sample(s)
    return e


def run(e, opts, mode, n_tokens):
    if mode == 'pix':
        e.set_mode('incremental')
    if mode in ('loop', 'pix'):
        return e.merge_until(opts.get('max_length') or 0, opts.get('min_weight') or 0,
                             opts.get('max_iterations') or 0)
    out = []
    it = 1
    while not opts.get('max_iterations') or it <= opts['max_iterations']:
        m = e.find_next_merge(opts.get('max_length') or 0, opts.get('min_weight') or 0)
        if m is None:
            break
        assert e.apply_merge(m[0], m[1], n_tokens) == m[2]
        n_tokens += 1
        out.append(m)
        it += 1
    return out


@pytest.mark.parametrize('mode', ['host', 'loop', 'pix'])
@pytest.mark.parametrize('seed', range(8))
def test_sharded_context_vs_oracle(seed, mode):
    """Random corpora (runs, cold ids >= 256, ties, max_length / min_weight) over 2-4 shards:
    merges and final corpus equal the oracle's on the unsharded corpus."""
    rng = random.Random(500 + seed)
    alphabet = rng.choice([3, 20, 256, 300])
    samples = random_corpus(rng, rng.choice([20000, 400000]), alphabet, rng.choice([0.0, 0.3]),
                            rng.choice([5, 17, 60]))
    len16 = [rng.choice([1, 1, 2]) for _ in range(alphabet)]
    opts = {'max_iterations': rng.choice([25, 60]), 'max_length': rng.choice([0, 0, 4]),
            'min_weight': rng.choice([0, 2, 3])}
    ids = np.concatenate(samples)
    off = np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64)
    st = OracleState(ids, off, len16, alphabet)
    want = st.merge_until(opts['max_length'], opts['min_weight'], opts['max_iterations'])
    e = multi_engine(samples, len16, rng.choice([2, 3, 4]))
    got = run(e, opts, mode, alphabet)
    assert got == want
    assert e.samples() == st.samples()
    check_sample_index(e, st.samples(), rng)
    e.close()


@pytest.mark.parametrize('mode', ['loop', 'pix'])
def test_golden_cases_over_two_shards(mode):
    """The reference-generated golden cases (tests/golden/small_cases.json) through a 2-shard
    context, in the streaming and the incremental mode: merges and final corpus."""
    bad = []
    for case in load_small()[::3]:
        c = Corpus()
        for s in case['samples']:
            c.add(s)
        e = multi_engine(c.samples, c.len16, 2)
        o = case['opts']
        got = run(e, o, mode, len(c.chars))
        if [list(m) for m in got] != case['merges'] or e.samples() != case['final_ids']:
            bad.append(case['name'])
        e.close()
    assert not bad, bad[:10]


def test_latin1_ingest_is_split_in_corpus_order():
    """Bulk ingest over 3 shards: whole samples in order, corpus-wide first-appearance ids, the
    same merges as one context."""
    data = pkg.synth_latin1(6 << 20, seed=7, A=200, base=40)
    one = pkg.Engine(0)
    cm1, nt1, h1 = one.add_latin1(data, sample_bytes=1 << 20)
    multi = pkg.Engine(devices=[0, 0, 0], reduce='host')
    assert multi.shard_count() == 3
    cm3, nt3, h3 = multi.add_latin1(data, sample_bytes=1 << 20)
    assert nt1 == nt3 and np.array_equal(cm1, cm3) and np.array_equal(h1, h3)
    assert multi.corpus_size() == one.corpus_size()
    a, oa = one.read_corpus()
    b, ob = multi.read_corpus()
    assert np.array_equal(a, b) and np.array_equal(oa, ob)
    assert multi.merge_until(0, 2, 150) == one.merge_until(0, 2, 150)
    a, _ = one.read_corpus()
    b, _ = multi.read_corpus()
    assert np.array_equal(a, b)


def test_samples_added_after_merging_go_to_the_last_shard():
    rng = random.Random(9)
    V = 30
    first = [np.array([rng.randrange(V) for _ in range(rng.randint(0, 4000))], np.int32)
             for _ in range(7)]
    later = [np.array([rng.randrange(V) for _ in range(3000)], np.int32) for _ in range(2)]
    e = multi_engine(first, [1] * V, 3)
    m1 = e.merge_until(0, 2, 10)
    for s in later:
        e.add_sample(s)
    m2 = e.merge_until(0, 2, 10)
    st = OracleState(np.concatenate(first), np.concatenate([[0], np.cumsum([len(s) for s in first])]),
                     [1] * V, V)
    assert m1 == st.merge_until(0, 2, 10)
    ids = np.concatenate([st.ids] + later)
    off = np.concatenate([st.off, st.off[-1] + np.cumsum([len(s) for s in later])])
    st2 = OracleState(ids, off, list(st.len16[:st.n_tokens]), st.n_tokens)
    assert m2 == st2.merge_until(0, 2, 10)
    assert e.samples() == st2.samples()


def test_sample_with_new_ids_after_merging_grows_every_shard():
    """A later sample brings ids the shards never saw (the C-ABI caller registers nothing): every
    shard's vocabulary grows alike, so the next merges number their tokens alike and match the
    oracle on the whole corpus."""
    rng = random.Random(21)
    V = 12
    first = [np.array([rng.randrange(V) for _ in range(3000)], np.int32) for _ in range(6)]
    e = multi_engine(first, [1] * V, 3)
    m1 = e.merge_until(0, 2, 8)
    nt = e.num_tokens()
    assert nt == V + 8
    # ids nt .. nt+4 are brand new (never registered); the sample mixes them with old ones
    later = np.array([rng.choice([nt, nt + 1, nt + 4, 0, 1]) for _ in range(5000)], np.int32)
    e.add_sample(later)
    assert e.num_tokens() == nt + 5
    m2 = e.merge_until(0, 2, 12)
    st = OracleState(np.concatenate(first), np.concatenate([[0], np.cumsum([len(s) for s in first])]),
                     [1] * V, V)
    assert m1 == st.merge_until(0, 2, 8)
    ids = np.concatenate([st.ids, later])
    off = np.concatenate([st.off, [st.off[-1] + len(later)]])
    l16 = list(st.len16[:st.n_tokens]) + [1] * 5
    st2 = OracleState(ids, off, l16, nt + 5)
    assert m2 == st2.merge_until(0, 2, 12)
    assert e.samples() == st2.samples()
    e.close()


def test_per_shard_entry_points_refuse_a_multi_context():
    e = pkg.Engine(devices=[0, 0], reduce='host')
    with pytest.raises(pkg.BpeError, match='multi-device'):
        e.recount()


@pytest.mark.skipif(pkg.device_count() < 2, reason='RCCL exchange needs two devices')
def test_rccl_exchange_over_two_devices():
    data = pkg.synth_latin1(8 << 20, seed=12345, A=256)
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    two = pkg.Engine(devices=[0, 1], reduce='rccl')
    two.add_latin1(data, sample_bytes=1 << 20)
    assert two.merge_until(0, 2, 300) == one.merge_until(0, 2, 300)


def test_rccl_context_when_libbpe_loads_before_torch():
    """libbpe loaded (system HIP runtime) before `import torch` (torch's bundled HIP runtime and
    RCCL, same sonames): the RCCL context must still come up, on the RCCL next to libbpe's own HIP
    runtime (bpe_multi.cpp load_rccl).  Before the fix ncclCommInitAll picked torch's RCCL and
    failed with 'unhandled cuda error' (this is the order pytest's collection produces)."""
    import subprocess
    import sys
    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools',
                          'debug', 'rccl_after_torch.py')
    out = subprocess.run([sys.executable, script, 'bpefirst', 'torch', 'work'], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0 and '\nok' in out.stdout, out.stdout[-2000:] + out.stderr[-2000:]


@pytest.mark.parametrize('corpus', ['uniform', 'zipf'])
def test_rccl_one_device_context(corpus):
    """bpe_create_multi with RCCL on one device (ncclCommInitAll over [0]): the rank loop's
    all-reduces are real RCCL calls on the shard's stream.  A 64 MiB C3 slice (table state) and a
    zipf slice (maintained state: delta rows all-reduced every merge) give the single context's
    merges and corpus."""
    if corpus == 'zipf':
        data, n = pkg.synth_zipf(16 << 20, seed=12345), 700
    else:
        data, n = pkg.synth_latin1(64 << 20, seed=12345, A=256), 400
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    want = one.merge_until(0, 2, n)
    ids1, off1 = one.read_corpus()
    one.close()
    r = pkg.Engine(devices=[0], reduce='rccl')
    assert r.shard_count() == 1
    r.add_latin1(data, sample_bytes=1 << 20)
    r.stats_enable(True)
    got = r.merge_until(0, 2, n)
    st = r.stats()
    assert got == want
    ids, off = r.read_corpus()
    assert np.array_equal(ids, ids1) and np.array_equal(off, off1)
    if corpus == 'zipf':
        assert st['fused_passes'] > n // 2, st
    r.close()


@pytest.mark.parametrize('shards', [3, 1])
def test_samples_added_in_the_maintained_state(shards):
    """merge (zipf: the shards reach the maintained state), add samples, merge on: a sample added
    to the last shard makes every shard leave the global tables, so the exchange sizes stay equal;
    the merges and corpus equal one context's."""
    data = pkg.synth_zipf(6 << 20, seed=12345)
    extra = pkg.synth_zipf(2 << 20, seed=777)
    one = pkg.Engine(0)
    cm, _, _ = one.add_latin1(data, sample_bytes=1 << 20)
    w1 = one.merge_until(0, 2, 500)
    one.add_latin1(extra, sample_bytes=1 << 20, char_to_id=cm)
    w2 = one.merge_until(0, 2, 300)
    ids1, off1 = one.read_corpus()
    one.close()
    multi = pkg.Engine(devices=[0] * shards, reduce='host')
    cm3, _, _ = multi.add_latin1(data, sample_bytes=1 << 20)
    assert np.array_equal(cm, cm3)
    multi.stats_enable(True)
    assert multi.merge_until(0, 2, 500) == w1
    assert multi.stats()['fused_passes'] > 0
    multi.add_latin1(extra, sample_bytes=1 << 20, char_to_id=cm)
    assert multi.merge_until(0, 2, 300) == w2
    ids, off = multi.read_corpus()
    assert np.array_equal(ids, ids1) and np.array_equal(off, off1)
    multi.close()


@pytest.mark.parametrize('shards,mib,n,max_length', [(3, 6, 900, 0), (4, 4, 600, 5), (2, 8, 700, 0)])
def test_maintained_state_over_shards_on_zipf_words(shards, mib, n, max_length):
    """A skewed corpus over several shards: the cold pairs outgrow the sketch, the shards move to
    the maintained state (global tables on every shard, delta rows exchanged per merge) and stay
    in the device loop.  Same merges and corpus as one context."""
    data = pkg.synth_zipf(mib << 20, seed=12345)
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    want = one.merge_until(max_length, 2, n)
    ids1, off1 = one.read_corpus()
    one.close()
    multi = pkg.Engine(devices=[0] * shards, reduce='host')
    multi.add_latin1(data, sample_bytes=1 << 20)
    multi.stats_enable(True)
    got = multi.merge_until(max_length, 2, n)
    st = multi.stats()
    assert got == want
    ids, off = multi.read_corpus()
    assert np.array_equal(ids, ids1) and np.array_equal(off, off1)
    assert st['fused_passes'] > n // 2, st      # (summed over the shards)
    assert st['loop_host'] <= 12, st
    multi.close()


@pytest.mark.parametrize('shards,corpus,n,max_length', [(3, 'zipf', 900, 0), (4, 'uniform', 700, 0),
                                                       (2, 'zipf', 500, 6)])
def test_incremental_mode_over_shards(shards, corpus, n, max_length):
    """The incremental mode over shards: every shard's position index holds its own lists and
    the global counts, each merge's count changes exchanged as signed delta rows (the rank loop's
    all-reduce), ties decided from every shard's last counted occurrences.  Same merges and corpus
    as one context; every merge on the indexes."""
    data = (pkg.synth_zipf(6 << 20, seed=12345) if corpus == 'zipf' else
            pkg.synth_latin1(8 << 20, seed=4242, A=64, base=32))
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    want = one.merge_until(max_length, 2, n)
    ids1, off1 = one.read_corpus()
    one.close()
    multi = pkg.Engine(devices=[0] * shards, reduce='host')
    multi.add_latin1(data, sample_bytes=1 << 20)
    multi.set_mode('incremental')
    multi.stats_enable(True)
    got = multi.merge_until(max_length, 2, n)
    st = multi.stats()
    assert got == want
    ids, off = multi.read_corpus()
    assert np.array_equal(ids, ids1) and np.array_equal(off, off1)
    assert st['pix_merges'] >= shards * (n - 8 * (st['pix_host'] + 1)), st
    multi.close()


def test_incremental_exchange_lanes_vs_dense_rows(monkeypatch):
    """The sharded incremental mode's exchange in its lane layout (round 5: per merge, one count
    per token id and side, the sites with that neighbour, in lanes as wide as the last merge's
    count needs) against the dense delta rows (6 u64 per token id, BPE_XCHG_DENSE=1), and with
    lanes of at most 4 bits (BPE_XCHG_LANE_BITS=4: every count outgrows them, the batch pauses
    before the merge and the next one, in full words, makes it; the layouts alternate, so a
    batch's first iteration decodes the last batch's pending merge in that batch's layout): the
    same merges and corpus as one context, and far fewer bytes per merge."""
    data = pkg.synth_latin1(16 << 20, seed=4242, A=96, base=32)
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    want = one.merge_until(0, 2, 1500)
    ids1, _ = one.read_corpus()
    one.close()
    per_merge = {}
    for layout in ('dense', 'lanes', 'lanes4'):
        monkeypatch.delenv('BPE_XCHG_DENSE', raising=False)
        monkeypatch.delenv('BPE_XCHG_LANE_BITS', raising=False)
        if layout == 'dense':
            monkeypatch.setenv('BPE_XCHG_DENSE', '1')
        elif layout == 'lanes4':
            monkeypatch.setenv('BPE_XCHG_LANE_BITS', '4')
        multi = pkg.Engine(devices=[0] * 4, reduce='host')
        multi.add_latin1(data, sample_bytes=1 << 20)
        multi.set_mode('incremental')
        multi.stats_enable(True)
        got = multi.merge_until(0, 2, 1500)
        st = multi.stats()
        assert got == want, layout
        ids, _ = multi.read_corpus()
        assert np.array_equal(ids, ids1), layout
        assert st['pix_merges'] >= 4 * 1400 and st['xchg_iters'] >= 1400, st
        assert st['pix_host'] == 0, (layout, st)
        # (xchg_bytes is summed over the 4 shards)
        per_merge[layout] = st['xchg_bytes'] / 4 / st['xchg_iters']
        multi.close()
    print('exchange bytes per merge', per_merge)
    assert per_merge['lanes'] * 8 < per_merge['dense'], per_merge


def test_incremental_exchange_lanes_across_max_length_changes():
    """The lane layout bounds each count by the last merge's W, which holds while the selection's
    filter stays: a call with max_length set, then one without (pairs the filter held back, with
    counts above the last W, become selectable: the layout must go back to full words), then one
    with it again.  4 shards against one context, the same calls."""
    data = pkg.synth_zipf(16 << 20, seed=404)
    calls = [(4, 300), (0, 300), (6, 300)]
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    want = [one.merge_until(ml, 2, k) for ml, k in calls]
    ids1, _ = one.read_corpus()
    one.close()
    multi = pkg.Engine(devices=[0] * 4, reduce='host')
    multi.add_latin1(data, sample_bytes=1 << 20)
    multi.set_mode('incremental')
    multi.stats_enable(True)
    got = [multi.merge_until(ml, 2, k) for ml, k in calls]
    st = multi.stats()
    ids, _ = multi.read_corpus()
    multi.close()
    assert got == want
    assert np.array_equal(ids, ids1)
    # (a few iterations go to the host protocol here, as in one context: ties of many candidates)
    assert st['pix_merges'] >= 4 * 800 and st['pix_host'] <= 6, st


def test_automatic_switch_to_the_incremental_mode_and_its_fallback(monkeypatch):
    """The streaming mode's switch to the incremental mode past a vocabulary size (18432 ids;
    BPE_AUTO_PIX_VOCAB=600 here), and its fall-back to the stream when the shards' indexes do not
    fit (BPE_PIX_FORCE_OOM=1: every index build fails as out of device memory): the same merges
    and corpus as one context either way.  A mode the caller set (set_mode('stream')) is kept:
    no switch."""
    data = pkg.synth_latin1(16 << 20, seed=4243, A=96, base=32)
    one = pkg.Engine(0)
    one.add_latin1(data, sample_bytes=1 << 20)
    want = one.merge_until(0, 2, 1200)
    ids1, _ = one.read_corpus()
    one.close()
    monkeypatch.setenv('BPE_AUTO_PIX_VOCAB', '600')
    for leg in ('auto', 'oom', 'explicit'):
        if leg == 'oom':
            monkeypatch.setenv('BPE_PIX_FORCE_OOM', '1')
        multi = pkg.Engine(devices=[0] * 4, reduce='host')
        multi.add_latin1(data, sample_bytes=1 << 20)
        if leg == 'explicit':
            multi.set_mode('stream')
        multi.stats_enable(True)
        got = multi.merge_until(0, 2, 1200)
        st = multi.stats()
        assert got == want, leg
        ids, _ = multi.read_corpus()
        assert np.array_equal(ids, ids1), leg
        if leg == 'oom':
            assert st['pix_fallbacks'] >= 1 and st['pix_merges'] == 0, st
        elif leg == 'explicit':
            assert st['pix_fallbacks'] == 0 and st['pix_merges'] == 0, st
        else:
            assert st['pix_fallbacks'] == 0 and st['pix_merges'] >= 4 * 500, st
        multi.close()


@pytest.mark.slow
@pytest.mark.parametrize('mode', ['stream', 'pix'])
def test_eight_shards_to_the_32k_vocabulary(mode):
    """8 shards of the C5 stream on one device (exchanged by a device kernel, the same rank loop
    as RCCL over 8 GPUs; one enqueue thread per shard) taken to the 32k-token vocabulary: past the
    sketch's reach the shards keep the global tables themselves (maintained state; past 18432 ids
    the streaming mode goes on in the incremental mode), so the iterations stay in the device loop
    (few host hand-offs); merges and final corpus equal one context's."""
    n = 512 << 20
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    one = pkg.Engine(0)
    _, nt, _ = one.add_latin1(data, sample_bytes=1 << 20)
    want = one.merge_until(0, 2, 32768 - nt)
    ids1, _ = one.read_corpus()
    one.close()
    multi = pkg.Engine(devices=[0] * 8, reduce='host')
    multi.add_latin1(data, sample_bytes=1 << 20)
    del data
    if mode == 'pix':
        multi.set_mode('incremental')
    multi.stats_enable(True)
    got = multi.merge_until(0, 2, 32768 - nt)
    st = multi.stats()
    assert len(got) == len(want) == 32768 - nt
    assert got == want
    ids, _ = multi.read_corpus()
    assert np.array_equal(ids, ids1)
    assert st['loop_host'] <= 24, st
    if mode == 'pix':   # (summed over the 8 shards)
        assert st['pix_merges'] > 8 * 30000, st
        # the compact exchange: bytes per merge over the run (was 6 dense rows per token id:
        # 1.57 MB per merge at the 32k vocabulary)
        print('exchange bytes per merge: %.0f' % (st['xchg_bytes'] / 8 / max(1, st['xchg_iters'])))
    else:
        # the streaming mode's maintained state up to AUTO_PIX_VOCAB (18432) token ids, then the
        # incremental mode (bpe_multi.cpp: the maintained state outgrows its LDS rows there)
        assert st['fused_passes'] > 8 * 9000 and st['pix_merges'] > 8 * 14000, st
    multi.close()
