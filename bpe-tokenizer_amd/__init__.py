"""bpe-tokenizer_amd — MI355X-native engine for the BPE merge-training hot path of
beenotung/bpe-tokenizer (reference: core.ts findNextMerge/applyMerge/mergeUntil).

This module is the Python (ctypes) binding of libbpe.so (C ABI: include/bpe.h).  The drop-in
replacement of the reference's `BPETokenizer` class lives in js/core.js (Node N-API addon over the
same C ABI); this binding serves the bench, the tests and multi-process (one rank per GPU) runs.

There is no CPU fallback: importing works anywhere (so the C ABI can be inspected), but creating
an `Engine` requires libbpe.so and a HIP device and raises otherwise.

Import with ``importlib.import_module('bpe-tokenizer_amd')`` (the directory name has a hyphen).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BPE_LIB selects an experimental build of the same C ABI (tools/ kernel experiments)
LIB_PATH = os.environ.get('BPE_LIB') or os.path.join(HERE, 'libbpe.so')

BPE_OK = 0
BPE_NO_MERGE = 1
MAX_VOCAB = 55296

# Every symbol include/bpe.h and include/bpe_tools.h declare (checked by tests/test_capi.py).
C_API = [
    'bpe_version', 'bpe_last_error', 'bpe_device_count', 'bpe_create', 'bpe_destroy',
    'bpe_create_multi', 'bpe_shard_count', 'bpe_set_mode',
    'bpe_set_token_len16', 'bpe_num_tokens', 'bpe_add_sample', 'bpe_add_latin1',
    'bpe_clear_corpus', 'bpe_corpus_size', 'bpe_read_corpus', 'bpe_sample_lengths',
    'bpe_read_samples', 'bpe_find_next_merge',
    'bpe_apply_merge', 'bpe_apply_merges', 'bpe_merge_until', 'bpe_stats_enable', 'bpe_get_stats', 'bpe_reset_stats',
    'bpe_get_stream', 'bpe_synth_latin1', 'bpe_synth_zipf', 'bpe_recount', 'bpe_export_counts',
    'bpe_heavy_counts', 'bpe_select_counts', 'bpe_tie_positions', 'bpe_rank_loop_begin',
    'bpe_rank_loop_select', 'bpe_rank_loop_decide', 'bpe_rank_loop_count', 'bpe_rank_loop_end',
    'bpe_cold_counts', 'bpe_set_global_counts',
    'bpe_encoder_create', 'bpe_encoder_destroy', 'bpe_encoder_add_merges', 'bpe_encoder_clear',
    'bpe_encoder_num_merges', 'bpe_encode_batch', 'bpe_encoder_get_stats', 'bpe_encoder_reset_stats',
    'bpe_rccl_unique_id', 'bpe_rank_rccl_init', 'bpe_rank_loop_rccl', 'bpe_rank_rccl_destroy',
]
HOT_BINS = 65536
TABLE_BINS = 81920
MAX_CAND = 16       # BPE_MAX_CAND
REDUCE_RCCL = 0     # BPE_REDUCE_RCCL
REDUCE_HOST = 1     # BPE_REDUCE_HOST
MODE_STREAM = 0     # BPE_MODE_STREAM
MODE_INCREMENTAL = 1   # BPE_MODE_INCREMENTAL
LOOP_BATCH = 64     # BPE_LOOP_BATCH
XCHG_HDR = 8        # BPE_XCHG_HDR
DELTA_ROWS = 6      # BPE_DELTA_ROWS
XCHG_WORDS = XCHG_HDR + DELTA_ROWS * MAX_VOCAB   # BPE_XCHG_WORDS
TIE_WORDS = 32      # BPE_TIE_WORDS
ENCODE_LDS_TOKENS = 16384   # BPE_ENCODE_LDS_TOKENS: longer texts are replayed by apply passes


ERR_ARG, ERR_HIP, ERR_OOM, ERR_STATE, ERR_VOCAB = -1, -2, -3, -4, -5
ERR_NOFIT = -6      # BPE_ERR_NOFIT: the position index does not fit beside the shard's corpus


class BpeError(RuntimeError):
    """A libbpe call failed; `code` is its status (BPE_ERR_*, include/bpe.h)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [
        ('step_ms', ctypes.c_double), ('step_launches', ctypes.c_int64),
        ('step_slots', ctypes.c_int64), ('step_live', ctypes.c_int64),
        ('select_ms', ctypes.c_double), ('tie_passes', ctypes.c_int64),
        ('iterations', ctypes.c_int64), ('live_tokens', ctypes.c_int64),
        ('compactions', ctypes.c_int64), ('exact_passes', ctypes.c_int64),
        ('step_timed', ctypes.c_int64), ('tie_tail', ctypes.c_int64),
        ('tie_lone', ctypes.c_int64), ('loop_host', ctypes.c_int64),
        ('fused_passes', ctypes.c_int64), ('pix_builds', ctypes.c_int64),
        ('pix_merges', ctypes.c_int64), ('pix_host', ctypes.c_int64),
        ('pix_build_ms', ctypes.c_double), ('cold_used', ctypes.c_int64),
        ('sel_blocks', ctypes.c_int64), ('xchg_bytes', ctypes.c_int64),
        ('xchg_iters', ctypes.c_int64), ('pix_fallbacks', ctypes.c_int64),
        ('cold_rebuilds', ctypes.c_int64), ('incr_ms', ctypes.c_double),
        ('incr_timed', ctypes.c_int64), ('incr_launches', ctypes.c_int64),
        ('incr_live', ctypes.c_int64), ('unscreened_passes', ctypes.c_int64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def rccl_unique_id():
    """ncclGetUniqueId of the RCCL beside libbpe's HIP runtime: 128 bytes (bpe_rccl_unique_id)."""
    buf = ctypes.create_string_buffer(128)
    _check(lib().bpe_rccl_unique_id(buf, 128), 'bpe_rccl_unique_id')
    return buf.raw


class EncoderStats(ctypes.Structure):
    """bpe_encoder_stats (include/bpe.h)."""
    _fields_ = [('kernel_ms', ctypes.c_double), ('calls', ctypes.c_int64),
                ('texts_rank', ctypes.c_int64), ('texts_replay', ctypes.c_int64),
                ('tokens_in', ctypes.c_int64), ('tokens_out', ctypes.c_int64),
                ('steps', ctypes.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


def build(force=False):
    """Compiles libbpe.so for gfx950 (hipcc cross-compiles; no GPU needed)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(['make', '-s', '-C', HERE] + (['-B'] if force else []))
    return LIB_PATH


_lib = None


def lib():
    """Loads libbpe.so (raises if it was not built — no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BpeError('libbpe.so is missing: run make -C bpe-tokenizer_amd (HIP engine required)')
    L = ctypes.CDLL(LIB_PATH)
    i32p, i64p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)
    vp = ctypes.c_void_p
    sig = {
        'bpe_version': ([], ctypes.c_int),
        'bpe_last_error': ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_int),
        'bpe_device_count': ([ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        'bpe_create': ([ctypes.POINTER(vp), ctypes.c_int], ctypes.c_int),
        'bpe_destroy': ([vp], ctypes.c_int),
        'bpe_create_multi': ([ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                              ctypes.c_int], ctypes.c_int),
        'bpe_shard_count': ([vp, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
        'bpe_set_mode': ([vp, ctypes.c_int], ctypes.c_int),
        'bpe_set_token_len16': ([vp, ctypes.c_int32, ctypes.c_int32], ctypes.c_int),
        'bpe_num_tokens': ([vp, i32p], ctypes.c_int),
        'bpe_add_sample': ([vp, i32p, ctypes.c_int64], ctypes.c_int),
        'bpe_add_latin1': ([vp, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, i32p, i32p, i64p],
                           ctypes.c_int),
        'bpe_clear_corpus': ([vp], ctypes.c_int),
        'bpe_corpus_size': ([vp, i64p, i64p], ctypes.c_int),
        'bpe_read_corpus': ([vp, i32p, ctypes.c_int64, i64p, ctypes.c_int64], ctypes.c_int),
        'bpe_sample_lengths': ([vp, i64p, ctypes.c_int64], ctypes.c_int),
        'bpe_read_samples': ([vp, i64p, ctypes.c_int64, i32p, ctypes.c_int64, i64p], ctypes.c_int),
        'bpe_find_next_merge': ([vp, ctypes.c_int64, ctypes.c_int64, i32p, i32p, i64p],
                                ctypes.c_int),
        'bpe_apply_merge': ([vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, i64p],
                            ctypes.c_int),
        'bpe_apply_merges': ([vp, i32p, ctypes.c_int64, i64p, ctypes.c_int], ctypes.c_int),
        'bpe_merge_until': ([vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, i64p,
                             ctypes.c_int64, i64p], ctypes.c_int),
        'bpe_stats_enable': ([vp, ctypes.c_int], ctypes.c_int),
        'bpe_get_stats': ([vp, ctypes.POINTER(Stats)], ctypes.c_int),
        'bpe_reset_stats': ([vp], ctypes.c_int),
        'bpe_get_stream': ([vp, ctypes.POINTER(vp)], ctypes.c_int),
        'bpe_recount': ([vp], ctypes.c_int),
        'bpe_export_counts': ([vp, vp], ctypes.c_int),
        'bpe_heavy_counts': ([vp, vp, ctypes.c_int64, vp, vp, ctypes.c_int64, i64p], ctypes.c_int),
        'bpe_select_counts': ([vp, vp, vp, vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                               i32p, ctypes.c_int64, i64p, i64p], ctypes.c_int),
        'bpe_tie_positions': ([vp, i32p, ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64)],
                              ctypes.c_int),
        'bpe_rank_loop_begin': ([vp, ctypes.c_int64, ctypes.c_int64, vp, vp, ctypes.c_int,
                                 ctypes.c_int, i64p], ctypes.c_int),
        'bpe_cold_counts': ([vp, vp, vp, ctypes.c_int64, i64p], ctypes.c_int),
        'bpe_set_global_counts': ([vp, vp, vp, vp, ctypes.c_int64], ctypes.c_int),
        'bpe_rank_loop_select': ([vp], ctypes.c_int),
        'bpe_rank_loop_decide': ([vp], ctypes.c_int),
        'bpe_rank_loop_count': ([vp], ctypes.c_int),
        'bpe_rank_loop_end': ([vp, i64p, ctypes.c_int64, i64p, ctypes.POINTER(ctypes.c_int)],
                              ctypes.c_int),
        'bpe_rccl_unique_id': ([vp, ctypes.c_size_t], ctypes.c_int),
        'bpe_rank_rccl_init': ([vp, vp, ctypes.c_int, ctypes.c_int], ctypes.c_int),
        'bpe_rank_loop_rccl': ([vp, vp, ctypes.c_int64, vp, ctypes.c_int], ctypes.c_int),
        'bpe_rank_rccl_destroy': ([vp], ctypes.c_int),
        'bpe_encoder_create': ([ctypes.POINTER(vp), ctypes.c_int], ctypes.c_int),
        'bpe_encoder_destroy': ([vp], ctypes.c_int),
        'bpe_encoder_add_merges': ([vp, i32p, ctypes.c_int64], ctypes.c_int),
        'bpe_encoder_clear': ([vp], ctypes.c_int),
        'bpe_encoder_num_merges': ([vp, i64p], ctypes.c_int),
        'bpe_encode_batch': ([vp, i32p, i64p, ctypes.c_int64, i32p, i64p], ctypes.c_int),
        'bpe_encoder_get_stats': ([vp, ctypes.POINTER(EncoderStats)], ctypes.c_int),
        'bpe_encoder_reset_stats': ([vp], ctypes.c_int),
        'bpe_synth_zipf': ([ctypes.c_uint32, ctypes.c_double, ctypes.c_uint32, ctypes.c_uint64,
                            ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64], ctypes.c_int),
        'bpe_synth_latin1': ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64,
                              ctypes.c_void_p, ctypes.c_int64], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        if not hasattr(L, name):   # (an older experimental build: BPE_LIB)
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def last_error():
    buf = ctypes.create_string_buffer(1024)
    lib().bpe_last_error(buf, 1024)
    return buf.value.decode(errors='replace')


def _check(rc, what):
    if rc < 0:
        raise BpeError('%s failed (%d): %s' % (what, rc, last_error()), rc)
    return rc


def device_count():
    n = ctypes.c_int(0)
    _check(lib().bpe_device_count(ctypes.byref(n)), 'bpe_device_count')
    return n.value


def synth_latin1(n, seed=12345, A=256, base=0, skip=0):
    """SURVEY.md §8(d) synthetic corpus: xorshift32 bytes (jump-ahead `skip` outputs)."""
    out = np.empty(n, dtype=np.uint8)
    _check(lib().bpe_synth_latin1(seed, A, base, skip, out.ctypes.data, n), 'bpe_synth_latin1')
    return out


def synth_zipf(n, seed=12345, s=1.1, n_words=32768, sample_bytes=1 << 20, first_sample=0):
    """Skewed synthetic corpus (include/bpe_tools.h bpe_synth_zipf): Zipf(s) words from a fixed
    word list, samples of sample_bytes starting at sample `first_sample`."""
    out = np.empty(n, dtype=np.uint8)
    _check(lib().bpe_synth_zipf(seed, s, n_words, first_sample, sample_bytes, out.ctypes.data, n),
           'bpe_synth_zipf')
    return out


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


class Engine:
    """One corpus shard on one HIP device (a `bpe_ctx`); with `devices`, one corpus sharded over
    several (bpe_create_multi: RCCL all-reduces, or host copies when reduce='host')."""

    def __init__(self, device=0, devices=None, reduce='rccl'):
        self._ctx = ctypes.c_void_p()
        if devices is None:
            _check(lib().bpe_create(ctypes.byref(self._ctx), device), 'bpe_create')
        else:
            dv = (ctypes.c_int * len(devices))(*devices)
            _check(lib().bpe_create_multi(ctypes.byref(self._ctx), len(devices), dv,
                                          REDUCE_HOST if reduce == 'host' else REDUCE_RCCL),
                   'bpe_create_multi')

    def set_mode(self, mode):
        """'stream' (every merge one pass over the corpus) or 'incremental' (mergeUntil on the
        position index: O(W) work per merge; bpe_set_mode)."""
        m = {'stream': MODE_STREAM, 'incremental': MODE_INCREMENTAL}[mode]
        _check(lib().bpe_set_mode(self._ctx, m), 'bpe_set_mode')

    def shard_count(self):
        n = ctypes.c_int()
        _check(lib().bpe_shard_count(self._ctx, ctypes.byref(n)), 'bpe_shard_count')
        return n.value

    def close(self):
        if self._ctx:
            lib().bpe_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # vocabulary -------------------------------------------------------------------------------
    def set_token_len16(self, token_id, len16):
        _check(lib().bpe_set_token_len16(self._ctx, token_id, len16), 'bpe_set_token_len16')

    def num_tokens(self):
        n = ctypes.c_int32()
        _check(lib().bpe_num_tokens(self._ctx, ctypes.byref(n)), 'bpe_num_tokens')
        return n.value

    # corpus ------------------------------------------------------------------------------------
    def add_sample(self, ids):
        a = _i32(ids)
        p = a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)) if a.size else None
        _check(lib().bpe_add_sample(self._ctx, p, a.size), 'bpe_add_sample')

    def add_latin1(self, data, sample_bytes=0, char_to_id=None, n_tokens=None):
        """Bulk ingest; returns (char_to_id[256], n_tokens, char_hist[256])."""
        data = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else data, dtype=np.uint8)
        cmap = np.full(256, -1, np.int32) if char_to_id is None else _i32(char_to_id).copy()
        nt = ctypes.c_int32(self.num_tokens() if n_tokens is None else n_tokens)
        hist = np.zeros(256, np.int64)
        _check(lib().bpe_add_latin1(self._ctx, data.ctypes.data, data.size, sample_bytes,
                                    cmap.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                    ctypes.byref(nt),
                                    hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))),
               'bpe_add_latin1')
        return cmap, nt.value, hist

    def clear_corpus(self):
        _check(lib().bpe_clear_corpus(self._ctx), 'bpe_clear_corpus')

    def corpus_size(self):
        s, t = ctypes.c_int64(), ctypes.c_int64()
        _check(lib().bpe_corpus_size(self._ctx, ctypes.byref(s), ctypes.byref(t)), 'bpe_corpus_size')
        return s.value, t.value

    def read_corpus(self):
        """Returns (flat ids int32, sample offsets int64)."""
        ns, nt = self.corpus_size()
        ids = np.zeros(max(nt, 1), np.int32)
        off = np.zeros(ns + 1, np.int64)
        _check(lib().bpe_read_corpus(self._ctx, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                     ids.size, off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                     off.size), 'bpe_read_corpus')
        return ids[:nt], off

    def sample_lengths(self):
        """Live tokens per sample (int64), from the device-side sample index."""
        ns, _ = self.corpus_size()
        lens = np.zeros(max(ns, 1), np.int64)
        _check(lib().bpe_sample_lengths(self._ctx, lens.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                        lens.size), 'bpe_sample_lengths')
        return lens[:ns]

    def read_samples(self, idx):
        """The listed samples' ids: (flat ids int32, offsets int64), in the order of idx."""
        idx = np.ascontiguousarray(idx, np.int64)
        lens = self.sample_lengths()
        need = int(lens[idx].sum()) if idx.size else 0
        ids = np.zeros(max(need, 1), np.int32)
        off = np.zeros(idx.size + 1, np.int64)
        _check(lib().bpe_read_samples(self._ctx, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                      idx.size, ids.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      ids.size, off.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))),
               'bpe_read_samples')
        return ids[:need], off

    def samples(self):
        ids, off = self.read_corpus()
        return [ids[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]

    # hot path ----------------------------------------------------------------------------------
    def find_next_merge(self, max_length=0, min_weight=0):
        a, b, w = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        rc = _check(lib().bpe_find_next_merge(self._ctx, int(max_length or 0), int(min_weight or 0),
                                              ctypes.byref(a), ctypes.byref(b), ctypes.byref(w)),
                    'bpe_find_next_merge')
        return None if rc == BPE_NO_MERGE else (a.value, b.value, w.value)

    def apply_merge(self, a, b, c, sync=True):
        """applyMerge's corpus rewrite.  With sync=False the replacement count stays on the device
        (settled at the next engine call; no host round trip) and None is returned."""
        if not sync:
            _check(lib().bpe_apply_merge(self._ctx, a, b, c, None), 'bpe_apply_merge')
            return None
        r = ctypes.c_int64()
        _check(lib().bpe_apply_merge(self._ctx, a, b, c, ctypes.byref(r)), 'bpe_apply_merge')
        return r.value

    def apply_merges(self, merges, count_after=True):
        """restoreMerge replay / batch encoding (bpe_apply_merges): applies the (a, b, c) triples
        in order without counting pairs; returns the replacement counts."""
        abc = np.ascontiguousarray(np.asarray(merges, np.int32).reshape(-1, 3))
        rep = np.zeros(len(abc), np.int64)
        _check(lib().bpe_apply_merges(self._ctx, abc.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      len(abc), rep.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                      1 if count_after else 0), 'bpe_apply_merges')
        return rep.tolist()

    def merge_until(self, max_length=0, min_weight=0, max_iterations=0, cap=1 << 16):
        out = np.zeros(3 * cap, np.int64)
        n = ctypes.c_int64()
        _check(lib().bpe_merge_until(self._ctx, int(max_length or 0), int(min_weight or 0),
                                     int(max_iterations or 0),
                                     out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), cap,
                                     ctypes.byref(n)), 'bpe_merge_until')
        k = min(n.value, cap)
        return [tuple(int(v) for v in out[3 * i:3 * i + 3]) for i in range(k)]

    # measurement -------------------------------------------------------------------------------
    def stats_enable(self, on=True):
        _check(lib().bpe_stats_enable(self._ctx, 1 if on else 0), 'bpe_stats_enable')

    def stats(self):
        s = Stats()
        _check(lib().bpe_get_stats(self._ctx, ctypes.byref(s)), 'bpe_get_stats')
        return s.as_dict()

    # sharded corpus (device pointers, e.g. torch tensors' data_ptr()) ------------------------------
    def export_counts(self, table_ptr):
        """Copies this shard's [TABLE_BINS] u64 table (hot bins + cold sketch) to device memory."""
        _check(lib().bpe_export_counts(self._ctx, table_ptr), 'bpe_export_counts')

    def heavy_counts(self, table_ptr, keys_ptr, counts_ptr, cap, max_length=0):
        """Exact shard counts of the cold pairs whose GLOBAL sketch bucket could still win.
        Returns the entry count (> cap means nothing was written: grow and retry; -1 means no
        bucket qualified, which every rank decides alike)."""
        n = ctypes.c_int64()
        rc = lib().bpe_heavy_counts(self._ctx, table_ptr, int(max_length or 0), keys_ptr,
                                    counts_ptr, cap, ctypes.byref(n))
        if rc < 0 and n.value <= cap:
            _check(rc, 'bpe_heavy_counts')
        return n.value

    def select_counts(self, table_ptr, keys_ptr, counts_ptr, n_cold, max_length=0, min_weight=0,
                      cap=4096):
        """Selection over global tables: None, or (W, [(a, b), ...] candidates sorted)."""
        cand = np.zeros(2 * cap, np.int32)
        n, w = ctypes.c_int64(), ctypes.c_int64()
        rc = _check(lib().bpe_select_counts(self._ctx, table_ptr, keys_ptr, counts_ptr, n_cold,
                                            int(max_length or 0), int(min_weight or 0),
                                            cand.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                            cap, ctypes.byref(n), ctypes.byref(w)),
                    'bpe_select_counts')
        if rc == BPE_NO_MERGE:
            return None
        if n.value > cap:
            raise BpeError('more than %d tied candidates' % cap)
        return w.value, [(int(cand[2 * i]), int(cand[2 * i + 1])) for i in range(n.value)]

    def tie_positions(self, cands):
        """Shard-local last counted occurrence (+1, 0 = none) of each (a, b) candidate (R3)."""
        c = np.ascontiguousarray(np.asarray(cands, np.int32).reshape(-1))
        last = np.zeros(len(cands), np.uint64)
        _check(lib().bpe_tie_positions(self._ctx, c.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                       len(cands), last.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))),
               'bpe_tie_positions')
        return last

    # device-resident loop on one rank (bpe.h: bpe_rank_loop_*); the caller all-reduces `table`
    # and `tie` in order on stream() between the calls
    def stream(self):
        st = ctypes.c_void_p()
        _check(lib().bpe_get_stream(self._ctx, ctypes.byref(st)), 'bpe_get_stream')
        return st.value or 0

    def rank_loop_begin(self, max_length, min_weight, xchg_ptr, tie_ptr, rank, world):
        """Returns the number of exchange words to all-reduce per iteration of this batch."""
        nw = ctypes.c_int64()
        _check(lib().bpe_rank_loop_begin(self._ctx, int(max_length or 0), int(min_weight or 0),
                                         xchg_ptr, tie_ptr, rank, world, ctypes.byref(nw)),
               'bpe_rank_loop_begin')
        return nw.value

    def rank_loop_select(self):
        _check(lib().bpe_rank_loop_select(self._ctx), 'bpe_rank_loop_select')

    def rank_loop_decide(self):
        _check(lib().bpe_rank_loop_decide(self._ctx), 'bpe_rank_loop_decide')

    def rank_loop_count(self):
        _check(lib().bpe_rank_loop_count(self._ctx), 'bpe_rank_loop_count')

    def rank_loop_end(self):
        """Syncs; returns ([(a, b, W)] merged in this batch, [this shard's replacement count of
        each], status) with status 0 = run on, 1 = no pair qualifies, 2 = the next iteration needs
        the host protocol."""
        out = np.zeros(4 * LOOP_BATCH, np.int64)
        n, st = ctypes.c_int64(), ctypes.c_int()
        _check(lib().bpe_rank_loop_end(self._ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                       LOOP_BATCH, ctypes.byref(n), ctypes.byref(st)),
               'bpe_rank_loop_end')
        k = n.value
        return ([tuple(int(v) for v in out[4 * i:4 * i + 3]) for i in range(k)],
                [int(out[4 * i + 3]) for i in range(k)], st.value)

    def rccl_init(self, unique_id, rank, world):
        """This context's RCCL communicator (bpe_rank_rccl_init); unique_id: 128 bytes made by
        rccl_unique_id() on rank 0 and broadcast."""
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        _check(lib().bpe_rank_rccl_init(self._ctx, buf, int(rank), int(world)), 'bpe_rank_rccl_init')

    def rank_loop_rccl(self, xchg_ptr, xchg_words, tie_ptr, iterations):
        """`iterations` rank-loop iterations with their all-reduces from C++ (bpe_rank_loop_rccl)."""
        _check(lib().bpe_rank_loop_rccl(self._ctx, xchg_ptr, int(xchg_words), tie_ptr, int(iterations)),
               'bpe_rank_loop_rccl')

    def cold_counts(self, keys_ptr, counts_ptr, cap):
        """This shard's exact count of every cold pair (one pass, kept for a second call): the
        entry count (> cap: nothing written, call again with room)."""
        n = ctypes.c_int64()
        _check(lib().bpe_cold_counts(self._ctx, keys_ptr, counts_ptr, cap, ctypes.byref(n)),
               'bpe_cold_counts')
        return n.value

    def set_global_counts(self, table_ptr, keys_ptr, counts_ptr, n):
        """The maintained state of a sharded corpus: the global table and every shard's cold
        lists (device pointers, duplicates summed) become this rank's global tables."""
        _check(lib().bpe_set_global_counts(self._ctx, table_ptr, keys_ptr, counts_ptr, n),
               'bpe_set_global_counts')

    def recount(self):
        """One plain streaming count pass (K1 alone; measurement helper)."""
        _check(lib().bpe_recount(self._ctx), 'bpe_recount')

    def reset_stats(self):
        _check(lib().bpe_reset_stats(self._ctx), 'bpe_reset_stats')


class Encoder:
    """encodeToCode (core.ts:392-409) for batches of texts with a trained merge list, apart from
    any corpus (bpe_encoder_*, include/bpe.h): the merge list lives on the device as a rank table;
    texts up to ENCODE_LDS_TOKENS tokens are encoded by the merge-rank kernel (csrc/bpe_encode.hip), longer
    ones by apply-only replay passes.  No CPU fallback."""

    def __init__(self, device=0, merges=None):
        p = ctypes.c_void_p()
        _check(lib().bpe_encoder_create(ctypes.byref(p), int(device)), 'bpe_encoder_create')
        self._enc = p
        if merges is not None and len(merges):
            self.add_merges(merges)

    def close(self):
        if self._enc:
            lib().bpe_encoder_destroy(self._enc)
            self._enc = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def add_merges(self, merges):
        """Appends (a, b, c) triples in list order (merge_codes, core.ts:91,352)."""
        abc = _i32(np.asarray(merges, dtype=np.int32).reshape(-1))
        _check(lib().bpe_encoder_add_merges(self._enc, abc.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                            len(abc) // 3), 'bpe_encoder_add_merges')

    def clear(self):
        _check(lib().bpe_encoder_clear(self._enc), 'bpe_encoder_clear')

    def num_merges(self):
        n = ctypes.c_int64()
        _check(lib().bpe_encoder_num_merges(self._enc, ctypes.byref(n)), 'bpe_encoder_num_merges')
        return n.value

    def encode_flat(self, ids, off):
        """Flat form: texts ids[off[k]:off[k+1]] -> (ids_out, out_off) numpy arrays."""
        ids = _i32(ids)
        off = np.ascontiguousarray(off, dtype=np.int64)
        n = len(off) - 1
        total = int(off[-1] - off[0]) if n > 0 else 0
        out = np.zeros(max(total, 1), dtype=np.int32)
        out_off = np.zeros(max(n + 1, 1), dtype=np.int64)
        src = ids if ids.size else np.zeros(1, np.int32)
        i32p, i64p = ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64)
        _check(lib().bpe_encode_batch(self._enc, src.ctypes.data_as(i32p), off.ctypes.data_as(i64p),
                                      n, out.ctypes.data_as(i32p), out_off.ctypes.data_as(i64p)),
               'bpe_encode_batch')
        return out[:out_off[n] if n > 0 else 0], out_off

    def encode(self, texts):
        """texts: a list of id sequences -> list of encoded int32 arrays."""
        lens = [len(t) for t in texts]
        off = np.zeros(len(texts) + 1, dtype=np.int64)
        np.cumsum(lens, out=off[1:])
        ids = np.concatenate([np.asarray(t, dtype=np.int32) for t in texts]) if texts and off[-1] \
            else np.zeros(0, np.int32)
        out, oo = self.encode_flat(ids, off)
        return [out[oo[k]:oo[k + 1]].copy() for k in range(len(texts))]

    def stats(self):
        s = EncoderStats()
        _check(lib().bpe_encoder_get_stats(self._enc, ctypes.byref(s)), 'bpe_encoder_get_stats')
        return s.as_dict()

    def reset_stats(self):
        _check(lib().bpe_encoder_reset_stats(self._enc), 'bpe_encoder_reset_stats')


def encode_samples(samples, merges, len16=None, device=0):
    """Batch encoding with a trained merge list (encodeToCode, core.ts:392-409, for many texts at
    once): the device encoder (bpe_encode_batch) — the merge-rank kernel for samples up to
    ENCODE_LDS_TOKENS tokens, apply-only replay passes for longer ones.  merges: (a, b, c) triples
    in list order.  (len16 is accepted for the older signature; encoding never reads it.)"""
    enc = Encoder(device, merges)
    try:
        return [x.tolist() for x in enc.encode([np.asarray(s, dtype=np.int32) for s in samples])]
    finally:
        enc.close()
