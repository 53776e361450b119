"""CPU-side checks of the C ABI: the library builds, loads and exports every declared symbol."""
import os
import re
import subprocess

import pytest

from bpe_amd import ROOT, pkg


def declared_symbols():
    names = []
    for h in ('bpe.h', 'bpe_tools.h'):
        src = open(os.path.join(ROOT, 'include', h)).read()
        names += re.findall(r'^int (bpe_\w+)\(', src, re.M)
    return names


def test_library_exports_every_declared_symbol():
    pkg.build()
    out = subprocess.check_output(['nm', '-D', '--defined-only', pkg.LIB_PATH]).decode()
    exported = set(re.findall(r' T (bpe_\w+)', out))
    decl = declared_symbols()
    assert decl, 'no declarations parsed'
    missing = [d for d in decl if d not in exported]
    assert not missing, missing
    assert sorted(decl) == sorted(pkg.C_API)


def test_library_loads_and_reports_no_device_without_gpu():
    L = pkg.lib()
    assert L.bpe_version() >= 100
    n = pkg.device_count()
    if n == 0:
        with pytest.raises(pkg.BpeError, match='no HIP device'):
            pkg.Engine(0)


def test_code_object_is_gfx950():
    """Every device code object in the offload bundles is gfx950 (host-side library code may
    name other targets in strings, so the bundle headers are parsed)."""
    import struct
    data = open(pkg.LIB_PATH, 'rb').read()
    magic = b'__CLANG_OFFLOAD_BUNDLE__'
    ids = []
    i = data.find(magic)
    while i >= 0:
        n = struct.unpack_from('<Q', data, i + len(magic))[0]
        q = i + len(magic) + 8
        for _ in range(n):
            _off, _size, idlen = struct.unpack_from('<QQQ', data, q)
            ids.append(data[q + 24:q + 24 + idlen].decode())
            q += 24 + idlen
        i = data.find(magic, q)
    dev = [x for x in ids if not x.startswith('host')]
    assert dev and all(x.endswith('gfx950') for x in dev), ids


def test_synthetic_generator_matches_oracle_and_jumps():
    import numpy as np
    from oracle import xorshift_corpus
    a = pkg.synth_latin1(1 << 16, seed=12345, A=95, base=0x20)
    assert a.tolist() == xorshift_corpus(12345, 95, 0x20, 1 << 16).tolist()
    b = pkg.synth_latin1(1000, seed=12345, A=256, base=0, skip=5000)
    full = pkg.synth_latin1(6000, seed=12345, A=256, base=0)
    assert np.array_equal(b, full[5000:])
    big = pkg.synth_latin1(1 << 23, seed=7, A=256)           # multithreaded path
    assert np.array_equal(big[-100:], pkg.synth_latin1(100, seed=7, A=256, skip=(1 << 23) - 100))


def test_synth_zipf_is_deterministic_and_shardable():
    from bpe_amd import pkg
    import numpy as np
    a = pkg.synth_zipf(6 << 16, seed=7, sample_bytes=1 << 16)
    assert np.array_equal(a, pkg.synth_zipf(6 << 16, seed=7, sample_bytes=1 << 16))
    b = pkg.synth_zipf(2 << 16, seed=7, sample_bytes=1 << 16, first_sample=4)
    assert np.array_equal(a[4 << 16:], b)
    letters = set(range(ord('a'), ord('z') + 1)) | {ord(' '), ord('\n')}
    assert set(np.unique(a).tolist()) <= letters
    # Zipf: the most frequent word dominates
    words = bytes(a[:1 << 16]).split()
    top = max(set(words), key=words.count)
    assert words.count(top) > len(words) // 20
