// The reference's own behavioural spec (core.spec.ts:17-417) re-asserted against the drop-in
// core.js on the GPU, plus the reference-generated golden cases through the full JS surface.
// Run: node --expose-gc tests/js/spec_gpu.js
'use strict'
const assert = require('assert')
const path = require('path')
const fs = require('fs')
const { BPETokenizer, EOF, compactMerge } = require(path.join(__dirname, '..', '..', 'bpe-tokenizer_amd', 'js', 'core.js'))

const wrap = s => EOF + s + EOF
const segs = (t, s) => t.encodeToTokens(s).map(x => x.chars).join(' ')
let n_tests = 0
function it(name, f) { f(); n_tests++ }

const abc = 'aaabdaaabac'
it('abc segments (core.spec.ts:17-33)', () => {
  const t = new BPETokenizer()
  t.addToCorpus(abc)
  t.mergeUntil({ min_weight: 2 })
  assert.strictEqual(segs(t, abc), 'aaab d aaab a c')
})
it('abc vector (core.spec.ts:35-88)', () => {
  const t = new BPETokenizer()
  t.addToCorpus(wrap(abc))
  t.mergeUntil({ min_weight: 2 })
  t.compactVectorIndex()
  assert.deepStrictEqual(t.encodeToVector(abc), [4, 2, 4, 1, 3])
})
const x9 = 'xxxxxxxxx'
it('x9 segments and vector (core.spec.ts:91-140)', () => {
  let t = new BPETokenizer()
  t.addToCorpus(wrap(x9))
  t.mergeUntil({ min_weight: 2 })
  assert.strictEqual(segs(t, x9), 'xxxx xxxx x')
  t = new BPETokenizer()
  t.addToCorpus(wrap(x9))
  t.mergeUntil({ min_weight: 2 })
  t.compactVectorIndex()
  assert.deepStrictEqual(t.encodeToVector(x9), [2, 2, 1])
})
it('JSON export / import (core.spec.ts:142-165)', () => {
  const t = new BPETokenizer()
  t.addToCorpus(wrap(fs.readFileSync(__filename).toString()))
  t.mergeUntil({ min_weight: 2 })
  const json = JSON.stringify(t)
  assert(json.length > 0)
  assert(t.token_table.length > 1)
  const u = new BPETokenizer()
  u.fromJSON(JSON.parse(json))
  assert.deepStrictEqual(u.token_table, t.token_table)
})
it('resume merges after restart (core.spec.ts:167-199)', () => {
  const merges = []
  const t = new BPETokenizer()
  t.addToCorpus(wrap(abc))
  for (;;) {
    const merge = t.findNextMerge()
    if (!merge) break
    if (merge[2].weight < 2) break
    merges.push(compactMerge(merge))
    t.applyMerge(merge)
  }
  const tokens = t.token_table
  const vector = t.encodeToVector(abc)
  assert(merges.length > 0 && vector.length > 0)
  const u = new BPETokenizer()
  u.addToCorpus(wrap(abc))
  for (const m of merges) u.restoreMerge(m)
  assert.deepStrictEqual(u.token_table, tokens)
  assert.deepStrictEqual(u.encodeToVector(abc), vector)
  assert.strictEqual(u.decodeVector(vector), abc)
  assert.deepStrictEqual(u.corpus_in_code, t.corpus_in_code)
})
it('encodeToVector invalidates after each merge (core.spec.ts:201-224)', () => {
  const content = 'x'.repeat(10)
  const t = new BPETokenizer()
  t.addToCorpus(wrap(content))
  assert.deepStrictEqual(t.encodeToVector(content), [1, 1, 1, 1, 1, 1, 1, 1, 1, 1])
  let merge = t.findNextMerge({ max_length: 5 })
  t.applyMerge(merge)
  assert.deepStrictEqual(t.encodeToVector(content), [1, 1, 1, 1, 1])
  merge = t.findNextMerge({ max_length: 5 })
  t.applyMerge(merge)
  assert.deepStrictEqual(t.encodeToVector(content), [2, 2, 1])
})
function x10() { const t = new BPETokenizer(); t.addToCorpus(wrap('x'.repeat(10))); return t }
function expectMerge(m, a, b) {
  assert(m)
  assert.strictEqual(m[0].chars, a); assert.strictEqual(m[1].chars, b); assert.strictEqual(m[2].chars, a + b)
}
it('length limit (core.spec.ts:226-264)', () => {
  let t = x10()
  let m = t.findNextMerge(); expectMerge(m, 'x', 'x'); t.applyMerge(m)
  m = t.findNextMerge({ max_length: 4 }); expectMerge(m, 'xx', 'xx')
  t = x10()
  m = t.findNextMerge(); t.applyMerge(m)
  assert.strictEqual(t.findNextMerge({ max_length: 3 }), null)
})
it('weight limit (core.spec.ts:266-313)', () => {
  let t = x10()
  expectMerge(t.findNextMerge({ min_weight: 5 }), 'x', 'x')
  assert.strictEqual(x10().findNextMerge({ min_weight: 6 }), null)
  t = x10()
  let m = t.findNextMerge(); expectMerge(m, 'x', 'x'); t.applyMerge(m)
  m = t.findNextMerge(); expectMerge(m, 'xx', 'xx'); t.applyMerge(m)
  assert.strictEqual(t.findNextMerge(), null)
})
function table(t) { return t.token_table.map(x => [x.chars, x.weight]) }
it('mergeUntil limits (core.spec.ts:315-417)', () => {
  let t = x10(); t.mergeUntil({ min_weight: 2 })
  assert.deepStrictEqual(table(t), [[EOF, 2], ['x', 0], ['xx', 1], ['xxxx', 2]])
  t = x10(); t.mergeUntil({ min_weight: 3 })
  assert.deepStrictEqual(table(t), [[EOF, 2], ['x', 0], ['xx', 5]])
  t = x10(); t.mergeUntil({ max_length: 4 })
  assert.deepStrictEqual(table(t), [[EOF, 2], ['x', 0], ['xx', 1], ['xxxx', 2]])
  t = x10(); t.mergeUntil({ max_length: 3 })
  assert.deepStrictEqual(table(t), [[EOF, 2], ['x', 0], ['xx', 5]])
  t = x10(); t.mergeUntil({ min_weight: 3, max_length: 3 })
  assert.deepStrictEqual(table(t), [[EOF, 2], ['x', 0], ['xx', 5]])
})
it('corpus_in_code getter / setter (example/import-merge-log-to-ram.ts:21-22)', () => {
  const t = new BPETokenizer()
  t.addToCorpus('abab'); t.addToCorpus(''); t.addToCorpus('ba')
  const codes = t.corpus_in_code
  assert.deepStrictEqual(codes, ['\u0001\u0002\u0001\u0002', '', '\u0002\u0001'])
  t.corpus_in_code = []
  assert.deepStrictEqual(t.corpus_in_code, [])
  assert.strictEqual(t.findNextMerge(), null)
  t.corpus_in_code = codes
  assert.deepStrictEqual(t.corpus_in_code, codes)
  const m = t.findNextMerge()
  assert.deepStrictEqual([m[0].chars, m[1].chars, m[2].weight], ['a', 'b', 2])
})
it('restoreToCorpus after fromJSON continues merging', () => {
  const t = new BPETokenizer()
  t.addToCorpus('abcabcabcab'); t.mergeUntil({ max_iterations: 2 })
  const u = new BPETokenizer(); u.fromJSON(JSON.parse(JSON.stringify(t)))
  u.restoreToCorpus('abcabcabcab')
  assert.deepStrictEqual(u.corpus_in_code, t.corpus_in_code)
  t.mergeUntil({}); u.mergeUntil({})
  assert.deepStrictEqual(table(u), table(t))
})

it('mergeUntil on the device loop == findNextMerge + applyMerge one by one (core.ts:365-383)', () => {
  let seed = 7
  const rnd = () => { seed ^= seed << 13; seed >>>= 0; seed ^= seed >>> 17; seed ^= seed << 5; seed >>>= 0; return seed }
  const alpha = 'abcdefghij klmnop'
  const samples = []
  for (let s = 0; s < 12; s++) {
    let str = ''
    const n = 2000 + (rnd() % 20000)
    for (let i = 0; i < n; i++) str += (rnd() % 7 === 0 ? 'xx' : alpha[rnd() % alpha.length])
    samples.push(str)
  }
  for (const opts of [{ max_iterations: 150 }, { max_iterations: 90, max_length: 3 }, { max_iterations: 2.5, min_weight: 3 }]) {
    const t = new BPETokenizer(), u = new BPETokenizer()
    for (const s of samples) { t.addToCorpus(s); u.addToCorpus(s) }
    t.mergeUntil(opts)
    for (let it = 1; !opts.max_iterations || it <= opts.max_iterations; it++) {
      const m = u.findNextMerge(opts)
      if (!m) break
      u.applyMerge(m)
    }
    assert.deepStrictEqual(t.token_table, u.token_table)
    assert.deepStrictEqual(t.merge_codes, u.merge_codes)
    assert.deepStrictEqual(t.merge_tokens.map(m => m.map(x => x.index)), u.merge_tokens.map(m => m.map(x => x.index)))
    assert.deepStrictEqual(t.corpus_in_code, u.corpus_in_code)
    // and merging continues identically from both
    t.mergeUntil({ max_iterations: 5 }); u.mergeUntil({ max_iterations: 5 })
    assert.deepStrictEqual(t.token_table, u.token_table)
  }
  const e = new BPETokenizer()
  e.mergeUntil({})                        // empty corpus: nothing to merge (core.ts:312)
  e.addToCorpus('abab'); e.mergeUntil({ max_iterations: -1 })   // `iteration <= -1` never holds
  assert.strictEqual(e.token_table.length, 2)
})
it('long texts are encoded on the device (encodeToCode, core.ts:392-409)', () => {
  const t = new BPETokenizer()
  const alpha = 'the quick brown fox jumps over a lazy dog'
  let seed = 99, corpus = ''
  const rnd = () => { seed ^= seed << 13; seed >>>= 0; seed ^= seed >>> 17; seed ^= seed << 5; seed >>>= 0; return seed }
  for (let i = 0; i < 50000; i++) corpus += alpha[rnd() % alpha.length]
  t.addToCorpus(corpus)
  t.mergeUntil({ max_iterations: 200 })
  assert(t.merge_tokens.length >= 100)
  let text = ''
  for (let i = 0; i < 200000; i++) text += alpha[rnd() % alpha.length]
  // the reference's replay, on a JS string (core.ts:395-406)
  let want = ''
  for (const ch of text) want += t.char_to_token[ch].code
  for (const [from_code, to_code] of t.merge_codes) want = want.split(from_code).join(to_code)
  assert.strictEqual(t.encodeToCode(text), want)
  const vec = t.encodeToVector(text)
  assert.strictEqual(t.decodeVector(vec), text)
  assert.throws(() => t.encodeToCode(text + '\u00e9'), e => e.message === 'unknown token, char: "\u00e9"')
})

// the device encoder (merge-rank kernel, bpe_encode_batch) against the reference's replay for
// short and mid-length texts, a merge list grown by restoreMerge in between, and fromJSON
it('device encoder = replaceAll replay (core.ts:392-409)', () => {
  const t = new BPETokenizer()
  let x = 99
  const rnd = () => { x ^= x << 13; x ^= x >>> 17; x ^= x << 5; return (x >>> 0) / 4294967296 }
  const word = () => { let w = ''; const l = 1 + Math.floor(rnd() * 6); for (let i = 0; i < l; i++) w += 'abcdefghij'[Math.floor(rnd() * 10)]; return w }
  const text = n => { let s = ''; while (s.length < n) s += word() + ' '; return s.slice(0, n) }
  for (let i = 0; i < 40; i++) t.addToCorpus(text(2000))
  t.mergeUntil({ min_weight: 2, max_iterations: 600 })
  assert(t.merge_tokens.length >= 300, 'merges ' + t.merge_tokens.length)
  const replay = s => {
    let want = ''
    for (const ch of s) want += t.char_to_token[ch].code
    for (const [from_code, to_code] of t.merge_codes) want = want.split(from_code).join(to_code)
    return want
  }
  for (const n of [0, 1, 2, 3, 10, 100, 511, 513, 3000, 5000, 17000]) {
    const s = text(n)
    assert.strictEqual(t.encodeToCode(s), replay(s), 'len ' + n)
  }
  // restoreMerge-style growth (the encoder appends), then a fromJSON (the encoder rebuilds)
  const json = t.toJSON()
  const u = new BPETokenizer()
  u.fromJSON(json)
  for (const n of [50, 700, 4000]) {
    const s = text(n)
    assert.strictEqual(u.encodeToCode(s), replay(s))
    assert.deepStrictEqual(u.encodeToVector(s), t.encodeToVector(s))
  }
  const v = new BPETokenizer()
  v.fromJSON(Object.assign({}, json, { merge_codes: json.merge_codes.slice(0, 200) }))
  const w = new BPETokenizer()
  w.fromJSON(Object.assign({}, json, { merge_codes: json.merge_codes.slice(0, 200) }))
  const s = text(900)
  const before = v.encodeToCode(s)
  for (const [a, b, c] of json.merge_codes.slice(200, 300)) {
    const tok = u.code_to_token[c]
    v.restoreMerge([a, b, tok.original_weight])
  }
  let want = ''
  for (const ch of s) want += v.char_to_token[ch].code
  for (const [from_code, to_code] of v.merge_codes) want = want.split(from_code).join(to_code)
  assert.strictEqual(v.encodeToCode(s), want)
  assert.strictEqual(w.encodeToCode(s), before)
})

// reference-generated golden cases through the whole JS surface
const golden = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'small_cases.json')))
let g = 0
for (const c of golden.cases) {
  const t = new BPETokenizer()
  for (const s of c.samples) t.addToCorpus(s)
  const o = {}
  for (const k in c.opts) if (c.opts[k] !== null) o[k] = c.opts[k]
  t.mergeUntil(o)
  assert.deepStrictEqual(t.merge_tokens.map(([a, b, x]) => [a.index, b.index, x.original_weight]), c.merges, c.name)
  assert.deepStrictEqual(t.token_table.map(x => [x.chars, x.weight, x.original_weight]), c.token_table, c.name)
  const ids = t.corpus_in_code.map(s => Array.from(s).map(ch => ch.codePointAt(0) - 1))
  assert.deepStrictEqual(ids, c.final_ids, c.name)
  c.samples.forEach((s, i) => {
    const want = c.vectors[i]
    if (typeof want === 'string') assert.throws(() => t.encodeToVector(s), e => 'error: ' + e.message === want)
    else assert.deepStrictEqual(t.encodeToVector(s), want, c.name)
  })
  g++
  if (global.gc && g % 100 === 0) global.gc()
}
console.log('spec_gpu ok', n_tests, 'spec tests,', g, 'golden cases')
