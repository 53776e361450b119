"""The Node drop-in (bpe-tokenizer_amd/js/core.js over the N-API addon): host logic on CPU, the
reference's spec + golden cases through the full JS surface on the GPU."""
import os
import shutil
import subprocess

import pytest

from bpe_amd import ROOT

NODE = shutil.which('node')
ADDON_DIR = os.path.join(ROOT, 'bpe-tokenizer_amd', 'addon')

pytestmark = pytest.mark.skipif(NODE is None, reason='node not installed')


def build_addon():
    subprocess.check_call(['make', '-s', '-C', ADDON_DIR])


def run_node(script, *flags, timeout=600, env=None, args=()):
    out = subprocess.run([NODE, *flags, os.path.join(ROOT, 'tests', 'js', script), *args],
                         capture_output=True, text=True, timeout=timeout,
                         env=dict(os.environ, **(env or {})))
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    return out.stdout


def test_addon_builds_and_exports():
    build_addon()
    out = subprocess.check_output([NODE, '-e', "const a=require(process.argv[1]);"
                                   "console.log(Object.keys(a).sort().join(','))",
                                   os.path.join(ADDON_DIR, 'bpe_napi.node')], text=True)
    assert out.strip() == ('addLatin1,addSample,applyMerge,applyMerges,clearCorpus,corpusSize,createEncoder,'
                           'createEngine,destroyEngine,deviceCount,encodeBatch,encoderAddMerges,'
                           'encoderClear,findNextMerge,mergeUntil,readCorpus,'
                           'readSamples,sampleLengths,setTokenLen16')


# (the default routing: with no device here, every encodeToCode the cost model sends to the
# device encoder falls back to the reference's JS replay; the GPU tests run the same golden vectors
# through the device encoder)
DEFAULT_ROUTING = {'BPE_ENCODE_DEVICE': ''}


def test_host_logic_against_golden():
    build_addon()
    assert 'host_only ok' in run_node('host_only.js', env=DEFAULT_ROUTING)


def test_encode_routing_falls_back_without_a_device():
    """encodeToCode with a 2000-merge list on short texts (the cost model picks the device) and with
    a list past the device encoder's ids (>= 55296): no HIP device here, so each call replays as the
    reference does, and the owner remembers that the encoder cannot be made."""
    build_addon()
    assert 'encode_routing ok host' in run_node('encode_routing.js', env=DEFAULT_ROUTING, args=['host'])


@pytest.mark.gpu
def test_encode_routing_on_the_device():
    """The same lists with a device: the 2000-merge list encodes on the device encoder, the list
    with ids >= 55296 falls back to the replay (remembered for that list, not for the owner)."""
    build_addon()
    assert 'encode_routing ok gpu' in run_node('encode_routing.js', env=DEFAULT_ROUTING, args=['gpu'])


def test_db_twin_host_logic_over_sqlite():
    """BPETokenizerDB (js/db.js) over a real sqlite database (Python's sqlite3 behind
    tests/js/sqlite_bridge.js): schema, JSON round trips and golden encode/decode vectors, token
    rows and weights, the proxy views, error messages.  No device needed."""
    build_addon()
    assert 'db_host_only ok' in run_node('db_host_only.js', env=DEFAULT_ROUTING)


@pytest.mark.gpu
def test_db_twin_spec_golden_and_lockstep():
    """BPETokenizerDB on the GPU: the reference's db spec, golden cases in both loop modes,
    row-by-row lockstep with core.js, resume from the database, rows added out of id order."""
    build_addon()
    out = run_node('spec_db_gpu.js', '--expose-gc')
    assert 'spec_db_gpu ok' in out


@pytest.mark.gpu
def test_reference_spec_and_golden_through_js():
    build_addon()
    out = run_node('spec_gpu.js', '--expose-gc')
    assert 'spec_gpu ok' in out


@pytest.mark.gpu
def test_reference_spec_and_golden_through_js_device_encoder():
    """The same run with every encodeToCode that has a merge sent to the device encoder
    (BPE_ENCODE_DEVICE=1): the golden vectors of all 1509 cases through bpe_encode_batch."""
    build_addon()
    out = run_node('spec_gpu.js', '--expose-gc', env={'BPE_ENCODE_DEVICE': '1'})
    assert 'spec_gpu ok' in out


@pytest.mark.gpu
def test_reference_spec_and_golden_through_js_on_two_shards():
    """The same spec + golden run with the corpus sharded over two shards (BPE_DEVICES=0,0 on the
    one-GPU box, pair counts exchanged through host copies): the class surface and every result
    are unchanged."""
    build_addon()
    out = run_node('spec_gpu.js', '--expose-gc', env={'BPE_DEVICES': '0,0', 'BPE_REDUCE': 'host'})
    assert 'spec_gpu ok' in out


@pytest.mark.gpu
def test_config2_vectors_through_js():
    """BASELINE config 2 through the drop-in: 10 x 1 MiB samples, mergeUntil({min_weight: 2,
    max_iterations: 1000}), encodeToVector of every sample on the device encoder; merges, weights,
    final corpus and vectors hashed as the reference's own run (tests/golden/config2.json)."""
    build_addon()
    out = run_node('config2_gpu.js', timeout=900)
    assert 'config2_gpu ok' in out
