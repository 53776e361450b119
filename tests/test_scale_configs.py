"""BASELINE configs 3, 4 and 5 at their full sizes on one MI355X (core.ts:365-383, mergeUntil).

  C3 — 1 GiB, the device loop (and the incremental mode) for 1000 merges, and for the whole run of
       8000, against the threaded CPU restatement's run (tests/golden/config3_cpu_mt_1000.json,
       config3_cpu_mt_8000.json: merges, live tokens and the SHA-256 of the final corpus); the
       skewed variant (Zipf words) for 2000 merges (zipf_cpu_mt_2000.json).  The restatement is
       pinned to the reference's own first C3 merges (config3_prefix.json) and to every golden
       case (tests/test_oracle_mt.py).
  C4 — 4 GiB sharded 4 ways behind one context (bpe_create_multi): on the one-GPU box the four
       shards share device 0 and exchange through a device kernel (bpe_sum_shards), the same rank
       loop and protocol as the RCCL exchange over 4 GPUs.  200 merges against config4_cpu_mt_200.json and against
       one context over the whole corpus.
  C5 — 16 GiB sharded 8 ways the same way (64 GiB of int32 slots per corpus copy), 200 merges
       against one context and the restatement's first merges on the host; and one GPU's C5
       shard (2 GiB) taken to the 32k-token vocabulary, its final state recounted from scratch on
       the host.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from bpe_amd import pkg
from golden_util import GOLDEN
from oracle import CpuMT

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

SAMPLE = 1 << 20


def fixture(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def host_threads():
    # (the box's CPU share is 16 threads; the affinity mask may show the whole machine)
    return max(1, min(16, len(os.sched_getaffinity(0))))


def engine(data, devices=None):
    e = pkg.Engine(0) if devices is None else pkg.Engine(devices=devices, reduce='host')
    cmap, nt, _ = e.add_latin1(data, sample_bytes=SAMPLE)
    e.stats_enable(True)
    return e, cmap, nt


@pytest.mark.parametrize('mode', ['loop', 'pix'])
def test_config3_1000_merges_vs_cpu_restatement(mode):
    g = fixture('config3_cpu_mt_1000.json')
    data = pkg.synth_latin1(g['bytes'], seed=g['seed'], A=g['alphabet'], base=0)
    e, _, nt = engine(data)
    del data
    assert nt == g['char_count']
    if mode == 'pix':
        e.set_mode('incremental')
    got = e.merge_until(0, g['min_weight'], len(g['merges']))
    assert [list(m) for m in got] == g['merges']
    assert e.corpus_size()[1] == g['live_tokens_after']
    st = e.stats()
    if mode == 'loop':
        assert st['loop_host'] <= 2, st
        ids, off = e.read_corpus()
        assert hashlib.sha256(np.ascontiguousarray(ids, '<i4').tobytes()).hexdigest() == g['sha256_ids_after']
        assert hashlib.sha256(np.ascontiguousarray(off, '<i8').tobytes()).hexdigest() == g['sha256_offsets_after']
    else:
        assert st['pix_merges'] == len(g['merges']), st
    e.close()


def run_against_fixture(g, data, mode):
    """mergeUntil({min_weight}) for the fixture's merges on one context, in the device loop or the
    incremental mode: the merge list, the live tokens and the final corpus's SHA-256 must equal
    the threaded CPU restatement's run."""
    e, _, nt = engine(data)
    del data
    assert nt == g['char_count']
    if mode == 'pix':
        e.set_mode('incremental')
    got = e.merge_until(0, g['min_weight'], len(g['merges']))
    assert [list(m) for m in got] == g['merges']
    assert hashlib.sha256(np.asarray(got, dtype=np.int64).tobytes()).hexdigest() == g['merges_sha256']
    assert e.corpus_size()[1] == g['live_tokens_after']
    ids, off = e.read_corpus()
    assert hashlib.sha256(np.ascontiguousarray(ids, '<i4').tobytes()).hexdigest() == g['sha256_ids_after']
    assert hashlib.sha256(np.ascontiguousarray(off, '<i8').tobytes()).hexdigest() == g['sha256_offsets_after']
    st = e.stats()
    e.close()
    return st


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, 'config3_cpu_mt_8000.json')),
                    reason='fixture not generated (oracle/gen_cpu_mt_fixtures.py c3_8000)')
@pytest.mark.parametrize('mode', ['loop', 'pix'])
def test_config3_all_8000_merges_vs_cpu_restatement(mode):
    """The whole headline run (BASELINE config 3: 1 GiB, 8000 merges, the bench's workload) against
    the threaded CPU restatement's: every merge, including the ~370 R3 tie decisions and the 12
    compactions of the streaming mode, and the final corpus."""
    g = fixture('config3_cpu_mt_8000.json')
    st = run_against_fixture(g, pkg.synth_latin1(g['bytes'], seed=g['seed'], A=g['alphabet'], base=0),
                             mode)
    if mode == 'loop':
        assert st['loop_host'] <= 4 and st['compactions'] >= 10 and st['tie_passes'] >= 100, st
    else:
        assert st['pix_merges'] == len(g['merges']), st


@pytest.mark.skipif(not os.path.exists(os.path.join(GOLDEN, 'zipf_cpu_mt_2000.json')),
                    reason='fixture not generated (oracle/gen_cpu_mt_fixtures.py zipf_2000)')
@pytest.mark.parametrize('mode', ['loop', 'pix'])
def test_zipf_2000_merges_vs_cpu_restatement(mode):
    """The skewed variant of config 3 (1 GiB of Zipf(1.1) words, bench.py --corpus zipf) for 2000
    merges against the CPU restatement: the streaming mode's maintained state (hot and cold tables
    kept merge by merge, MODE_INCR passes, the cold table rebuilt from itself when it fills) and
    the incremental mode with its heavy-merge prefix."""
    g = fixture('zipf_cpu_mt_2000.json')
    st = run_against_fixture(g, pkg.synth_zipf(g['bytes'], seed=g['seed']), mode)
    if mode == 'loop':
        assert st['fused_passes'] > 1000 and st['cold_rebuilds'] >= 1, st
    else:
        assert st['pix_merges'] > 0, st


def test_config4_four_shards_vs_one_context_and_cpu_restatement():
    g = fixture('config4_cpu_mt_200.json')
    data = pkg.synth_latin1(g['bytes'], seed=g['seed'], A=g['alphabet'], base=0)
    multi, _, nt = engine(data, devices=[0] * 4)
    assert multi.shard_count() == 4 and nt == g['char_count']
    got = multi.merge_until(0, g['min_weight'], len(g['merges']))
    st = multi.stats()
    live = multi.corpus_size()[1]
    multi.close()
    assert [list(m) for m in got] == g['merges']
    assert live == g['live_tokens_after']
    assert st['loop_host'] <= 2, st
    one, _, _ = engine(data)
    del data
    assert one.merge_until(0, g['min_weight'], len(g['merges'])) == got
    assert one.corpus_size()[1] == live
    one.close()


def test_config5_eight_shards_vs_one_context_and_cpu_restatement():
    n = 16 << 30
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    multi, cmap, nt = engine(data, devices=[0] * 8)
    assert multi.shard_count() == 8
    got = multi.merge_until(0, 2, 200)
    st = multi.stats()
    live = multi.corpus_size()[1]
    multi.close()
    assert len(got) == 200 and st['loop_host'] <= 2, st
    assert live == n - sum(m[2] for m in got)
    one, cmap1, _ = engine(data)
    assert np.array_equal(cmap, cmap1)
    assert one.merge_until(0, 2, 200) == got
    one.close()
    # the first merges of the whole 16 GiB on the host (the restatement, 64 GiB of host ids)
    cpu = CpuMT.from_latin1(data, SAMPLE, cmap, nt, threads=host_threads(), extra=64)
    del data
    want = cpu.merge_until(0, 2, 3)
    cpu.close()
    assert got[:3] == want


def test_config5_shard_to_the_32k_vocabulary_stream_and_incremental():
    """One GPU's C5 shard (2 GiB, the first 2 GiB of the C5 stream; 2^31 + 2048 slots) to the
    32k-token vocabulary (32512 merges).  The streaming mode (most merges in the maintained state,
    MODE_INCR): the first merges against the restatement, the final state's next merge against a
    recount from scratch of the corpus read back from HBM, tokens conserved.  Then the incremental
    mode on a second copy (positions past 2^31): every merge on the position index, the same merges
    and corpus as the streaming mode's (one streaming run serves both checks)."""
    n = 2 << 30
    data = pkg.synth_latin1(n, seed=12345, A=256, base=0)
    e, cmap, nt = engine(data)
    e2, _, _ = engine(data)
    cpu = CpuMT.from_latin1(data, SAMPLE, cmap, nt, threads=host_threads(), extra=64)
    del data
    want = cpu.merge_until(0, 2, 3)
    cpu.close()
    got = e.merge_until(0, 2, 32768 - nt)
    assert len(got) == 32768 - nt
    assert got[:3] == want
    st = e.stats()
    assert st['loop_host'] <= 16 and st['fused_passes'] > 10000, st
    assert e.corpus_size()[1] == n - sum(m[2] for m in got)
    ids, off = e.read_corpus()
    cpu = CpuMT(ids, off, [1] * 32768, 32768, threads=host_threads())
    nxt = cpu.find_next_merge(0, 2)
    cpu.close()
    assert e.find_next_merge(0, 2) == nxt
    e.close()
    e2.set_mode('incremental')
    got2 = e2.merge_until(0, 2, 32768 - nt)
    st2 = e2.stats()
    assert got2 == got
    assert st2['pix_merges'] >= len(got) - 64 * (st2['pix_host'] + 1), st2
    ids2, off2 = e2.read_corpus()
    assert np.array_equal(ids2, ids) and np.array_equal(off2, off)
    e2.close()
