#!/usr/bin/env python3
"""Golden-vector generator (TEST INFRASTRUCTURE — never shipped, never on the product path).

Runs the *reference itself* (`/root/reference/core.ts`, beenotung/bpe-tokenizer v2.2.0) under the
container's Node v12 and records its outputs as JSON fixtures under `tests/golden/`.

How the reference is run: `core.ts` is type-erased at run time into
`/tmp/bpe_ref/core.js` (TS annotations stripped, `?.` desugared, a `replaceAll` shim added because
Node 12 lacks it).  The erased file lives only in /tmp: no reference source enters the repository.
The fixtures hold only inputs and the reference's outputs (merge lists, token tables, final ids,
vectors).

Fixture sets:
  * ``small_cases.json``  — seeded random small corpora (runs, ties, astral chars, empty samples,
    max_length / min_weight / max_iterations variants): merges [a_index, b_index, W], final corpus
    ids per sample, token table, encodeToVector per sample.
  * ``config2.json``      — BASELINE config 2: 10 MiB synthetic ASCII corpus (xorshift32 seed 12345,
    95-char alphabet, 1 MiB samples), ``mergeUntil({min_weight:2, max_iterations:1000})``; full merge
    list + SHA-256 of final ids and of encodeToVector output.  Slow (~20 min of Node): ``--config2``.

Usage:  python3 oracle/gen_golden.py [--small] [--config2]
"""
import argparse
import json
import os
import random
import re
import subprocess
import sys

REF = '/root/reference/core.ts'
WORK = '/tmp/bpe_ref'
HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(os.path.dirname(HERE), 'tests', 'golden')


def erase_reference():
    """Type-erase core.ts into /tmp/bpe_ref/core.js (SURVEY.md Appendix B recipe)."""
    src = open(REF).read()
    src = re.sub(r'(?ms)^(export )?type \w+ = \{.*?^\}\n', '', src)
    src = re.sub(r'(?m)^(export )?type \w+ = \[.*?\]\n', '', src)
    src = re.sub(r'(?s)(\w+)\?: \{[^{}]*\}\)', r'\1)', src)
    src = re.sub(r'\)\: [^{=;]+? \{', ') {', src)
    src = re.sub(r'\((\w+): [\w\[\]| ]+\)', r'(\1)', src)
    src = re.sub(r'(?m)^(\s*(?:let )?\(?)(\w+): [^=\n]+? = ', r'\1\2 = ', src)
    src = re.sub(r'(?m)^(\s*)(\w+): [^=\n]+? = ', r'\1\2 = ', src)
    src = src.replace('new Map<Token, Map<Token, number>>()', 'new Map()')
    src = re.sub(r'(\w|\))!(?=[.\s),\]])', r'\1', src)
    src = src.replace('protected ', '')
    src = re.sub(r'(\w+)\?\.(\w+)', r'(\1 && \1.\2)', src)
    src = re.sub(r'let (\w+): number\[\] = ', r'let \1 = ', src)
    names = re.findall(r'(?m)^export (?:let|function|class) (\w+)', src)
    src = re.sub(r'(?m)^export ', '', src)
    shim = ("if (!String.prototype.replaceAll) String.prototype.replaceAll = function (p, r) {\n"
            "  if (typeof p !== 'string' || typeof r !== 'string') throw new Error('shim');\n"
            "  return this.split(p).join(r) }\n")
    os.makedirs(WORK, exist_ok=True)
    with open(os.path.join(WORK, 'core.js'), 'w') as f:
        f.write(shim + src + '\nmodule.exports = {' + ', '.join(names) + '}\n')
    subprocess.check_call(['node', '--check', os.path.join(WORK, 'core.js')])


# Node harness: runs one batch of cases through the erased reference.  Written to /tmp only.
HARNESS = r"""
const { BPETokenizer } = require('./core.js')
const fs = require('fs')
const crypto = require('crypto')
const input = JSON.parse(fs.readFileSync(process.argv[2]).toString())
function opt(o) { let r = {}; for (let k in o) if (o[k] !== null) r[k] = o[k]; return r }
function ids(s) { let r = []; for (let ch of s) r.push(ch.codePointAt(0) - 1); return r }
function runCase(c) {
  let t = new BPETokenizer()
  for (let s of c.samples) t.addToCorpus(s)
  let o = opt(c.opts), merges = [], maxIt = o.max_iterations
  for (let it = 1; !maxIt || it <= maxIt; it++) {
    let m = t.findNextMerge(o)
    if (!m) break
    merges.push([m[0].index, m[1].index, m[2].original_weight])
    t.applyMerge(m)
  }
  let out = { merges }
  out.final_ids = t.corpus_in_code.map(ids)
  out.token_table = t.token_table.map(x => [x.chars, x.weight, x.original_weight])
  out.vectors = c.samples.map(s => { try { return t.encodeToVector(s) } catch (e) { return 'error: ' + e.message } })
  return out
}
function xorshiftCorpus(seed, A, base, nbytes) {
  let x = seed >>> 0, codes = new Array(nbytes)
  for (let i = 0; i < nbytes; i++) {
    x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0
    codes[i] = base + Math.floor(x * A / 4294967296)
  }
  return codes
}
// config-3 scale: the corpus is generated sample by sample (a 2^30-element JS array does not fit
// V8's array limits), each sample flattened once added (the cons-string rope of core.ts:204
// otherwise exhausts the heap); only the first merges run (each is a ~2 minute scan)
function prefixRun(input) {
  let { seed, A, base, total, sample, max_iterations, min_weight } = input
  let x = seed >>> 0, t = new BPETokenizer(), t0 = Date.now()
  for (let off = 0; off < total; off += sample) {
    let n = Math.min(total, off + sample) - off, s = '', part = new Array(8192)
    for (let i = 0; i < n; i += 8192) {
      let k = Math.min(8192, n - i)
      for (let j = 0; j < k; j++) {
        x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0
        part[j] = base + Math.floor(x * A / 4294967296)
      }
      s += String.fromCharCode.apply(null, k === 8192 ? part : part.slice(0, k))
    }
    t.addToCorpus(s)
    t.corpus_in_code[t.corpus_in_code.length - 1].charCodeAt(0)
    if ((off / sample) % 64 == 0) console.error('sample', off / sample, (Date.now() - t0) / 1000, 's')
  }
  let ingest_s = (Date.now() - t0) / 1000, merges = [], merge_s = []
  for (let it = 1; it <= max_iterations; it++) {
    let t1 = Date.now()
    let m = t.findNextMerge({ min_weight })
    if (!m) break
    merges.push([m[0].index, m[1].index, m[2].original_weight])
    t.applyMerge(m)
    merge_s.push((Date.now() - t1) / 1000)
    console.error('merge', it, merges[merges.length - 1], merge_s[merge_s.length - 1], 's')
  }
  let corpus = t.corpus_in_code, live = 0
  for (let s of corpus) for (let ch of s) live++
  let sha = s => crypto.createHash('sha256').update(Buffer.from(new Int32Array(ids(s)).buffer)).digest('hex')
  return {
    seed, A, base, total, sample, max_iterations, min_weight, merges,
    char_count: Object.keys(t.char_to_token).length, live_tokens_after: live,
    first_sample_sha256: sha(corpus[0]), last_sample_sha256: sha(corpus[corpus.length - 1]),
    ingest_seconds: ingest_s, merge_seconds: merge_s,
  }
}
if (input.kind === 'prefix') {
  fs.writeFileSync(process.argv[3], JSON.stringify(prefixRun(input)))
} else if (input.kind === 'cases') {
  fs.writeFileSync(process.argv[3], JSON.stringify(input.cases.map(runCase)))
} else if (input.kind === 'synthetic') {
  let { seed, A, base, total, sample, max_iterations, min_weight } = input
  let codes = xorshiftCorpus(seed, A, base, total)
  let samples = []
  for (let off = 0; off < total; off += sample) {
    let part = codes.slice(off, Math.min(total, off + sample)), s = ''
    for (let i = 0; i < part.length; i += 8192) s += String.fromCharCode.apply(null, part.slice(i, i + 8192))
    samples.push(s)
  }
  let t = new BPETokenizer()
  for (let s of samples) { t.addToCorpus(s); t.corpus_in_code[t.corpus_in_code.length - 1].charCodeAt(0) }
  let merges = [], t0 = Date.now()
  for (let it = 1; it <= max_iterations; it++) {
    let m = t.findNextMerge({ min_weight })
    if (!m) break
    merges.push([m[0].index, m[1].index, m[2].original_weight])
    t.applyMerge(m)
    if (it % 50 == 0) console.error('iter', it, (Date.now() - t0) / 1000, 's')
  }
  let h = crypto.createHash('sha256'), hv = crypto.createHash('sha256'), n_ids = 0, n_vec = 0
  for (let s of t.corpus_in_code) {
    let a = ids(s); a.push(-1); n_ids += a.length
    h.update(Buffer.from(new Int32Array(a).buffer))
  }
  for (let s of samples) {
    let v = t.encodeToVector(s); v.push(-1); n_vec += v.length
    hv.update(Buffer.from(new Int32Array(v).buffer))
  }
  fs.writeFileSync(process.argv[3], JSON.stringify({
    seed, A, base, total, sample, max_iterations, min_weight, merges,
    token_count: t.token_table.length, char_count: Object.keys(t.char_to_token).length,
    final_ids_sha256: h.digest('hex'), final_ids_len: n_ids,
    vectors_sha256: hv.digest('hex'), vectors_len: n_vec,
    weights: t.token_table.map(x => x.weight),
    node_seconds: (Date.now() - t0) / 1000,
  }))
}
"""


def run_node(payload, name, heap_mb=16000):
    inp = os.path.join(WORK, name + '.in.json')
    out = os.path.join(WORK, name + '.out.json')
    with open(inp, 'w') as f:
        json.dump(payload, f)
    with open(os.path.join(WORK, 'harness.js'), 'w') as f:
        f.write(HARNESS)
    subprocess.check_call(['node', '--max-old-space-size=%d' % heap_mb, 'harness.js', inp, out],
                          cwd=WORK)
    with open(out) as f:
        return json.load(f)


ASTRAL = ['\U0001F600', '\U0001D11E', '\U00020000']


def random_cases(n, seed=20241024):
    rng = random.Random(seed)
    cases = []
    for i in range(n):
        kind = rng.random()
        if kind < 0.45:
            alpha = 'abcdefghij'[:rng.randint(1, 4)]          # tiny alphabets: runs + ties
        elif kind < 0.75:
            alpha = 'abcdefghijklmnopqrstuvwxyz .'[:rng.randint(5, 28)]
        elif kind < 0.9:
            alpha = 'xy' + ''.join(ASTRAL[:rng.randint(1, 3)])  # astral chars (UTF-16 length 2)
        else:
            alpha = ''.join(chr(c) for c in range(0x20, 0x7F))
        n_samples = rng.choice([1, 1, 1, 2, 3, 5, 8])
        samples = []
        for _ in range(n_samples):
            L = rng.choice([0, 1, 2, 3, rng.randint(4, 40), rng.randint(20, 160), rng.randint(20, 160),
                           rng.randint(100, 400)])
            if rng.random() < 0.15:                           # long single-char runs
                ch = rng.choice(alpha)
                s = ch * L
            else:
                s = ''.join(rng.choice(alpha) for _ in range(L))
            samples.append(s)
        opts = {
            'min_weight': rng.choice([None, None, 0, 1, 2, 3, 5, -1]),
            'max_length': rng.choice([None, None, None, 0, 2, 3, 4, 6]),
            'max_iterations': rng.choice([None, None, 1, 3, 10, 40]),
        }
        cases.append({'name': 'rand%04d' % i, 'samples': samples, 'opts': opts})
    return cases


def spec_cases():
    """The reference's own spec inputs (core.spec.ts) — outputs are taken from the reference."""
    EOF = '\x04'
    return [
        {'name': 'config1', 'samples': ['aaabdaaabac'], 'opts': {'min_weight': 2}},
        {'name': 'spec_abc_wrapped', 'samples': [EOF + 'aaabdaaabac' + EOF], 'opts': {'min_weight': 2}},
        {'name': 'spec_x9', 'samples': [EOF + 'x' * 9 + EOF], 'opts': {'min_weight': 2}},
        {'name': 'spec_x10_mw2', 'samples': [EOF + 'x' * 10 + EOF], 'opts': {'min_weight': 2}},
        {'name': 'spec_x10_mw3', 'samples': [EOF + 'x' * 10 + EOF], 'opts': {'min_weight': 3}},
        {'name': 'spec_x10_ml4', 'samples': [EOF + 'x' * 10 + EOF], 'opts': {'max_length': 4}},
        {'name': 'spec_x10_ml3', 'samples': [EOF + 'x' * 10 + EOF], 'opts': {'max_length': 3}},
        {'name': 'spec_x10_mw3_ml3', 'samples': [EOF + 'x' * 10 + EOF],
         'opts': {'min_weight': 3, 'max_length': 3}},
        {'name': 'multi_sample', 'samples': ['abab', '', 'baba', 'aaaa', 'ab'], 'opts': {}},
    ]


def gen_small():
    cases = spec_cases() + random_cases(1500)
    outs = run_node({'kind': 'cases', 'cases': cases}, 'small')
    for c, o in zip(cases, outs):
        c.update(o)
    path = os.path.join(GOLDEN, 'small_cases.json')
    with open(path, 'w') as f:
        json.dump({'generator': 'oracle/gen_golden.py', 'reference': 'beenotung/bpe-tokenizer v2.2.0 core.ts',
                   'cases': cases}, f, separators=(',', ':'))
    print('wrote', path, len(cases), 'cases', os.path.getsize(path), 'bytes')


def gen_config2():
    out = run_node({'kind': 'synthetic', 'seed': 12345, 'A': 95, 'base': 0x20, 'total': 10 << 20,
                    'sample': 1 << 20, 'max_iterations': 1000, 'min_weight': 2}, 'config2')
    path = os.path.join(GOLDEN, 'config2.json')
    with open(path, 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print('wrote', path, len(out['merges']), 'merges in', out['node_seconds'], 's')


def gen_config3_prefix():
    """BASELINE config 3 (1 GiB, 256-char alphabet, 1 MiB samples): the reference's first merges
    (SURVEY.md §8(c) golden item 5), with the live token count after them and the SHA-256 of the
    first and last samples' ids."""
    out = run_node({'kind': 'prefix', 'seed': 12345, 'A': 256, 'base': 0, 'total': 1 << 30,
                    'sample': 1 << 20, 'max_iterations': 3, 'min_weight': 2}, 'config3', 55000)
    path = os.path.join(GOLDEN, 'config3_prefix.json')
    with open(path, 'w') as f:
        json.dump(out, f, separators=(',', ':'))
    print('wrote', path, out['merges'], 'ingest', out['ingest_seconds'], 's')


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--small', action='store_true')
    ap.add_argument('--config2', action='store_true')
    ap.add_argument('--config3-prefix', action='store_true')
    args = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit('reference not present: fixtures can only be (re)generated in the build container')
    erase_reference()
    if args.small or not (args.config2 or args.config3_prefix):
        gen_small()
    if args.config2:
        gen_config2()
    if args.config3_prefix:
        gen_config3_prefix()
