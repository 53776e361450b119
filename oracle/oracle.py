"""ctypes wrapper over liboracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.  The
product path (libbpe.so + bpe-tokenizer_amd host code) never does.

`Corpus` mirrors the host-side bookkeeping of the reference's `addToCorpus` (core.ts:182-207):
code point -> token index in first-appearance order across calls, UTF-16 length per token
(`chars.length`, used by the max_length filter core.ts:270-273).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ORACLE_LIB') or os.path.join(HERE, 'liboracle.so')
_lib = None


def build():
    subprocess.check_call(['make', '-s', '-C', HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.oracle_find_next_merge.argtypes = [i32p, i64p, ctypes.c_int64, i32p, ctypes.c_int32,
                                             ctypes.c_int64, ctypes.c_int64, i32p, i32p, i64p]
        L.oracle_find_next_merge.restype = ctypes.c_int
        L.oracle_apply_merge.argtypes = [i32p, i64p, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_int32]
        L.oracle_apply_merge.restype = ctypes.c_int64
        L.oracle_merge_until.argtypes = [i32p, i64p, ctypes.c_int64, i32p, ctypes.c_int32,
                                         ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, i64p,
                                         ctypes.c_int64]
        L.oracle_merge_until.restype = ctypes.c_int64
        L.oracle_count_pairs.argtypes = [i32p, i64p, ctypes.c_int64, i32p, ctypes.c_int32,
                                         ctypes.c_int64, i32p, i32p, i64p, i64p, ctypes.c_int64]
        L.oracle_count_pairs.restype = ctypes.c_int64
        L.oracle_xorshift_corpus.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             ctypes.c_void_p, ctypes.c_int64]
        L.oracle_xorshift_corpus.restype = None
        L.oracle_encode.argtypes = [i32p, i64p, ctypes.c_int64, i32p, ctypes.c_int64]
        L.oracle_encode.restype = None
        _lib = L
    return _lib


def _p(arr, ct):
    return arr.ctypes.data_as(ctypes.POINTER(ct))


def js_truthy_int(v):
    """JS `x || 0` for the numeric options the tests use (None/0 -> 0)."""
    return 0 if v is None else int(v)


class Corpus:
    """Token ids + sample offsets, with the reference's char->index bookkeeping."""

    def __init__(self):
        self.char_to_index = {}
        self.chars = []          # token.chars per index (chars only for base tokens)
        self.len16 = []
        self.samples = []        # list of int32 arrays

    def add(self, content):
        ids = []
        for ch in content:                                   # core.ts:185 (code points)
            idx = self.char_to_index.get(ch)
            if idx is None:
                idx = len(self.chars)
                self.char_to_index[ch] = idx
                self.chars.append(ch)
                self.len16.append(2 if ord(ch) > 0xFFFF else 1)
            ids.append(idx)
        self.samples.append(np.asarray(ids, dtype=np.int32))

    def add_ids(self, ids):
        self.samples.append(np.asarray(ids, dtype=np.int32))

    def flat(self):
        off = np.zeros(len(self.samples) + 1, dtype=np.int64)
        for i, s in enumerate(self.samples):
            off[i + 1] = off[i] + len(s)
        ids = np.concatenate(self.samples) if self.samples else np.zeros(0, np.int32)
        return np.ascontiguousarray(ids, dtype=np.int32), off


class OracleState:
    """Flat corpus state driven through the C restatement."""

    def __init__(self, ids, off, len16, n_tokens, extra=1 << 16):
        self.ids = np.array(ids, dtype=np.int32, copy=True)
        if self.ids.size == 0:
            self.ids = np.zeros(1, np.int32)[:0].copy()
        self.off = np.array(off, dtype=np.int64, copy=True)
        self.len16 = np.zeros(n_tokens + extra, dtype=np.int32)
        self.len16[:len(len16)] = len16
        self.n_tokens = n_tokens

    @classmethod
    def from_corpus(cls, c, extra=1 << 16):
        ids, off = c.flat()
        return cls(ids, off, c.len16, len(c.chars), extra)

    def find_next_merge(self, max_length=None, min_weight=None):
        a = ctypes.c_int32()
        b = ctypes.c_int32()
        w = ctypes.c_int64()
        buf = self.ids if self.ids.size else np.zeros(1, np.int32)
        rc = lib().oracle_find_next_merge(_p(buf, ctypes.c_int32), _p(self.off, ctypes.c_int64),
                                          len(self.off) - 1, _p(self.len16, ctypes.c_int32),
                                          self.n_tokens, js_truthy_int(max_length),
                                          js_truthy_int(min_weight), ctypes.byref(a),
                                          ctypes.byref(b), ctypes.byref(w))
        if rc < 0:
            raise MemoryError('oracle allocation failed')
        return None if rc == 1 else (a.value, b.value, w.value)

    def apply_merge(self, a, b, c=None):
        if c is None:
            c = self.n_tokens
        if c >= self.n_tokens:
            self.len16[c] = self.len16[a] + self.len16[b]
            self.n_tokens = c + 1
        buf = self.ids if self.ids.size else np.zeros(1, np.int32)
        w = lib().oracle_apply_merge(_p(buf, ctypes.c_int32), _p(self.off, ctypes.c_int64),
                                     len(self.off) - 1, a, b, c)
        self.ids = self.ids[:self.off[-1]]
        return w

    def merge_until(self, max_length=None, min_weight=None, max_iterations=None):
        merges = []
        it = 1
        while not max_iterations or it <= max_iterations:
            m = self.find_next_merge(max_length, min_weight)
            if m is None:
                break
            self.apply_merge(m[0], m[1])
            merges.append(m)
            it += 1
        return merges

    def samples(self):
        return [self.ids[self.off[i]:self.off[i + 1]].tolist() for i in range(len(self.off) - 1)]

    def count_pairs(self, max_length=None):
        cap = max(16, self.n_tokens * self.n_tokens)
        pa = np.zeros(cap, np.int32)
        pb = np.zeros(cap, np.int32)
        pc = np.zeros(cap, np.int64)
        pl = np.zeros(cap, np.int64)
        buf = self.ids if self.ids.size else np.zeros(1, np.int32)
        n = lib().oracle_count_pairs(_p(buf, ctypes.c_int32), _p(self.off, ctypes.c_int64),
                                     len(self.off) - 1, _p(self.len16, ctypes.c_int32),
                                     self.n_tokens, js_truthy_int(max_length),
                                     _p(pa, ctypes.c_int32), _p(pb, ctypes.c_int32),
                                     _p(pc, ctypes.c_int64), _p(pl, ctypes.c_int64), cap)
        if n < 0:
            raise RuntimeError('oracle_count_pairs failed %d' % n)
        return pa[:n], pb[:n], pc[:n], pl[:n]


def encode(texts, merges):
    """encodeToCode's replay (core.ts:404-406) of the (a, b, c) merges over each text, in list
    order: the checker of the device encoder (bpe_encode_batch)."""
    off = np.zeros(len(texts) + 1, dtype=np.int64)
    np.cumsum([len(t) for t in texts], out=off[1:])
    ids = np.zeros(max(int(off[-1]), 1), dtype=np.int32)
    if off[-1]:
        ids[:off[-1]] = np.concatenate([np.asarray(t, dtype=np.int32) for t in texts])
    abc = np.ascontiguousarray(np.asarray(merges, dtype=np.int32).reshape(-1))
    if abc.size == 0:
        abc = np.zeros(3, np.int32)
        n = 0
    else:
        n = abc.size // 3
    lib().oracle_encode(_p(ids, ctypes.c_int32), _p(off, ctypes.c_int64), len(texts),
                        _p(abc, ctypes.c_int32), n)
    return [ids[off[k]:off[k + 1]].copy() for k in range(len(texts))]


def xorshift_corpus(seed, A, base, n):
    out = np.empty(n, dtype=np.uint8)
    lib().oracle_xorshift_corpus(seed, A, base, out.ctypes.data, n)
    return out


# ---- the multi-threaded restatement (oracle/bpe_cpu_mt.cc): larger parity cases + CPU baseline --
LIB_MT_PATH = os.environ.get('ORACLE_MT_LIB') or os.path.join(HERE, 'liboracle_mt.so')
_lib_mt = None


def lib_mt():
    global _lib_mt
    if _lib_mt is None:
        if not os.path.exists(LIB_MT_PATH):
            build()
        L = ctypes.CDLL(LIB_MT_PATH)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        vp = ctypes.c_void_p
        L.cpu_create.argtypes = [i32p, i64p, ctypes.c_int64, i32p, ctypes.c_int32, ctypes.c_int64,
                                 ctypes.c_int]
        L.cpu_create.restype = vp
        L.cpu_create_latin1.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, i32p, ctypes.c_int32,
                                        ctypes.c_int64, ctypes.c_int]
        L.cpu_create_latin1.restype = vp
        L.cpu_destroy.argtypes = [vp]
        L.cpu_destroy.restype = None
        L.cpu_live.argtypes = [vp]
        L.cpu_live.restype = ctypes.c_int64
        L.cpu_threads.argtypes = [vp]
        L.cpu_threads.restype = ctypes.c_int
        L.cpu_find_next_merge.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, i32p, i32p, i64p]
        L.cpu_find_next_merge.restype = ctypes.c_int
        L.cpu_apply_merge.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]
        L.cpu_apply_merge.restype = ctypes.c_int64
        L.cpu_merge_until.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, i64p,
                                      ctypes.c_int64, i64p]
        L.cpu_merge_until.restype = ctypes.c_int64
        L.cpu_read.argtypes = [vp, i32p, i64p]
        L.cpu_read.restype = None
        _lib_mt = L
    return _lib_mt


class CpuMT:
    """The corpus held by the multi-threaded restatement (threads <= 0: all host cores)."""

    def __init__(self, ids, off, len16, n_tokens, threads=0, extra=1 << 16):
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        if ids.size == 0:
            ids = np.zeros(1, np.int32)
        off = np.ascontiguousarray(off, dtype=np.int64)
        l16 = np.ascontiguousarray(np.asarray(len16, dtype=np.int32)[:n_tokens])
        if l16.size == 0:
            l16 = np.zeros(1, np.int32)
        self.n_samples = len(off) - 1
        self.n_tokens = n_tokens
        self._h = lib_mt().cpu_create(_p(ids, ctypes.c_int32), _p(off, ctypes.c_int64),
                                      self.n_samples, _p(l16, ctypes.c_int32), n_tokens, extra,
                                      threads)

    @classmethod
    def from_latin1(cls, data, sample_bytes, char_to_id, n_tokens, threads=0, extra=1 << 16):
        """The corpus from latin1 bytes (byte b -> char_to_id[b]) in samples of sample_bytes,
        mapped natively (no host int32 copy: bpe_cpu_mt.cc cpu_create_latin1)."""
        self = cls.__new__(cls)
        data = np.ascontiguousarray(data, dtype=np.uint8)
        cmap = np.ascontiguousarray(char_to_id, dtype=np.int32)
        self.n_samples = (len(data) + sample_bytes - 1) // sample_bytes if len(data) else 1
        self.n_tokens = n_tokens
        self._h = lib_mt().cpu_create_latin1(data.ctypes.data, len(data), sample_bytes,
                                             _p(cmap, ctypes.c_int32), n_tokens, extra, threads)
        return self

    def close(self):
        if self._h:
            lib_mt().cpu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def threads(self):
        return lib_mt().cpu_threads(self._h)

    def live(self):
        return lib_mt().cpu_live(self._h)

    def find_next_merge(self, max_length=None, min_weight=None):
        a, b, w = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int64()
        rc = lib_mt().cpu_find_next_merge(self._h, js_truthy_int(max_length),
                                          js_truthy_int(min_weight), ctypes.byref(a),
                                          ctypes.byref(b), ctypes.byref(w))
        return None if rc else (a.value, b.value, w.value)

    def apply_merge(self, a, b, c=None):
        if c is None:
            c = self.n_tokens
        self.n_tokens = max(self.n_tokens, c + 1)
        return lib_mt().cpu_apply_merge(self._h, a, b, c)

    def merge_until(self, max_length=None, min_weight=None, max_iterations=None, cap=1 << 16):
        out = np.zeros(3 * cap, np.int64)
        scans = ctypes.c_int64()
        n = lib_mt().cpu_merge_until(self._h, js_truthy_int(max_length), js_truthy_int(min_weight),
                                     js_truthy_int(max_iterations), _p(out, ctypes.c_int64), cap,
                                     ctypes.byref(scans))
        self.n_tokens += n
        self.last_scans = scans.value
        return [tuple(int(v) for v in out[3 * i:3 * i + 3]) for i in range(min(n, cap))]

    def read(self):
        ids = np.zeros(max(1, self.live()), np.int32)
        off = np.zeros(self.n_samples + 1, np.int64)
        lib_mt().cpu_read(self._h, _p(ids, ctypes.c_int32), _p(off, ctypes.c_int64))
        return ids[:self.live()], off

    def samples(self):
        ids, off = self.read()
        return [ids[off[i]:off[i + 1]].tolist() for i in range(len(off) - 1)]


# ---- the rank-greedy batch encoder on the host's cores (oracle/bpe_cpu_encode.cc): the device
# encoder's CPU baseline, checked against encode() (the in-order replay) by the tests ----------
LIB_ENC_PATH = os.environ.get('ORACLE_ENC_LIB') or os.path.join(HERE, 'liboracle_enc.so')
_lib_enc = None


def lib_enc():
    global _lib_enc
    if _lib_enc is None:
        if not os.path.exists(LIB_ENC_PATH):
            build()
        L = ctypes.CDLL(LIB_ENC_PATH)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        L.cpu_encode_batch.argtypes = [i32p, i64p, ctypes.c_int64, i32p, ctypes.c_int64, i32p, i64p,
                                       ctypes.c_int]
        L.cpu_encode_batch.restype = ctypes.c_int
        _lib_enc = L
    return _lib_enc


def cpu_encode_flat(ids, off, abc, threads=0):
    """encodeToCode of the texts ids[off[k]:off[k+1]] through the (a, b, c) merges, rank-greedy on
    `threads` host threads (0: all).  Returns (packed ids, offsets, threads used)."""
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    off = np.ascontiguousarray(off, dtype=np.int64)
    abc = np.ascontiguousarray(np.asarray(abc, dtype=np.int32).reshape(-1))
    n = len(off) - 1
    out = np.zeros(max(1, int(off[-1] - off[0])), np.int32)
    oo = np.zeros(n + 1, np.int64)
    buf = ids if ids.size else np.zeros(1, np.int32)
    m = abc.size // 3
    if abc.size == 0:
        abc = np.zeros(3, np.int32)
    used = lib_enc().cpu_encode_batch(_p(buf, ctypes.c_int32), _p(off, ctypes.c_int64), n,
                                      _p(abc, ctypes.c_int32), m, _p(out, ctypes.c_int32),
                                      _p(oo, ctypes.c_int64), threads)
    return out[:oo[-1]], oo, used
