"""AddressSanitizer + UndefinedBehaviorSanitizer over both CPU restatements (race /
memory checks on the host side; GPU sanitizers are not available on this pool).  The
instrumented builds (make -C oracle asan) run golden cases and random corpora in a subprocess with
libasan preloaded; any report fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, 'oracle')

SCRIPT = r'''
import sys, random
sys.path.insert(0, %(oracle)r); sys.path.insert(0, %(tests)r)
import numpy as np
from golden_util import load_small
from oracle import Corpus, CpuMT, OracleState
for case in load_small()[:400]:
    c = Corpus()
    for s in case['samples']:
        c.add(s)
    ids, off = c.flat()
    o = case['opts']
    opts = (o.get('max_length'), o.get('min_weight'), o.get('max_iterations'))
    a = OracleState(ids, off, c.len16, len(c.chars)).merge_until(*opts)
    st = CpuMT(ids, off, c.len16, len(c.chars), threads=3)
    b = st.merge_until(*opts)
    assert [list(m) for m in a] == case['merges'] == [list(m) for m in b], case['name']
    assert st.samples() == case['final_ids']
rng = random.Random(5)
for _ in range(20):
    V = rng.choice([3, 300])
    samples = [np.array([rng.randrange(V) for _ in range(rng.randint(0, 3000))], np.int32) for _ in range(6)]
    ids = np.concatenate(samples); off = np.concatenate([[0], np.cumsum([len(s) for s in samples])]).astype(np.int64)
    a = OracleState(ids, off, [1] * V, V).merge_until(0, 2, 40)
    b = CpuMT(ids, off, [1] * V, V, threads=4).merge_until(0, 2, 40)
    assert a == b
print('asan-clean')
'''


def test_restatements_under_asan():
    try:
        subprocess.check_call(['make', '-s', '-C', ORACLE, 'asan'])
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip('no sanitizer toolchain: %s' % e)
    libasan = subprocess.check_output(['gcc', '-print-file-name=libasan.so']).decode().strip()
    env = dict(os.environ)
    env.update({'LD_PRELOAD': libasan, 'ASAN_OPTIONS': 'detect_leaks=0:abort_on_error=0',
                'UBSAN_OPTIONS': 'halt_on_error=1:print_stacktrace=1',
                'ORACLE_LIB': os.path.join(ORACLE, '_asan', 'liboracle.so'),
                'ORACLE_MT_LIB': os.path.join(ORACLE, '_asan', 'liboracle_mt.so')})
    r = subprocess.run([sys.executable, '-c', SCRIPT % {'oracle': ORACLE,
                                                       'tests': os.path.join(ROOT, 'tests')}],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and 'asan-clean' in r.stdout, r.stderr[-4000:]
    assert 'runtime error' not in r.stderr and 'AddressSanitizer' not in r.stderr, r.stderr[-4000:]
