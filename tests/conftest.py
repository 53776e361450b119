import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device)')
    config.addinivalue_line('markers', 'slow: long-running (large corpora)')


# BPE_TRACK_MEM=<file>: free device memory after every GPU test, one line per test (leak hunting)
if os.environ.get('BPE_TRACK_MEM'):
    import ctypes

    def pytest_runtest_teardown(item, nextitem):
        if item.get_closest_marker('gpu') is None:
            return
        try:
            hip = ctypes.CDLL('libamdhip64.so')
            free, total = ctypes.c_size_t(), ctypes.c_size_t()
            hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total))
            with open(os.environ['BPE_TRACK_MEM'], 'a') as f:
                f.write('%s %.3f %.3f\n' % (item.nodeid, free.value / 2**30, total.value / 2**30))
        except OSError:
            pass
