"""Does bpe_create_multi(reduce=RCCL) come up next to PyTorch?  torch's wheel bundles libamdhip64.so.7
and librccl.so.1 under the same sonames as /opt/rocm/lib.  Arguments: bpefirst (load libbpe before
torch), torch (import it), work / enc (an ordinary engine / encoder first).  Prints 'ok' or 'FAIL ...'.
Used by tests/test_multi_device.py::test_rccl_context_when_libbpe_loads_before_torch."""
import importlib, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
pkg = importlib.import_module('bpe-tokenizer_amd')
if 'bpefirst' in sys.argv:   # libbpe (the system HIP runtime) loaded before torch, as pytest's
    pkg.device_count()       # collection does (a skipif calling device_count())
if 'torch' in sys.argv:
    import torch  # noqa: F401
maps = open('/proc/self/maps').read()
print('hip libs:', sorted({l.split()[-1] for l in maps.splitlines() if 'amdhip64' in l or 'rccl' in l}))
if 'work' in sys.argv:   # an ordinary engine first (HIP initialised by libbpe before RCCL)
    w = pkg.Engine(0)
    w.add_latin1(pkg.synth_latin1(1 << 20))
    w.merge_until(0, 2, 5)
    w.close()
if 'enc' in sys.argv:
    en = pkg.Encoder(0, [(0, 1, 300)])
    en.encode([[0, 1, 0, 1]])
    en.close()
try:
    e = pkg.Engine(devices=[0], reduce='rccl')
    e.add_latin1(pkg.synth_latin1(1 << 20))
    print('merges', e.merge_until(0, 2, 5))
    e.close()
    print('ok')
except Exception as ex:
    print('FAIL', ex)
    e = None
    maps = open('/proc/self/maps').read()
    print('hip libs after:', sorted({l.split()[-1] for l in maps.splitlines() if 'amdhip64' in l or 'rccl' in l}))
