// BASELINE config 2 through the drop-in (js/core.js on the GPU): 10 MiB of the 95-char xorshift32
// stream in 1 MiB samples, mergeUntil({min_weight: 2, max_iterations: 1000}), then encodeToVector
// of every sample (core.ts:424-445; 1 MiB texts take the device encoder, bpe_apply_merges).
// The merge list, the final corpus and the vectors are hashed exactly as oracle/gen_golden.py hashed
// the reference's own run (each sample's int32 array + a -1 separator) and compared with
// tests/golden/config2.json.
// Run: node tests/js/config2_gpu.js
'use strict'
const assert = require('assert')
const path = require('path')
const fs = require('fs')
const crypto = require('crypto')
const { BPETokenizer } = require(path.join(__dirname, '..', '..', 'bpe-tokenizer_amd', 'js', 'core.js'))

const g = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'config2.json')))

// SURVEY.md §8(d): x ^= x << 13; x ^= x >>> 17; x ^= x << 5 (uint32); char = base + floor(x * A / 2^32)
function xorshiftCodes(seed, A, base, n) {
  const out = new Uint16Array(n)
  let x = seed >>> 0
  for (let i = 0; i < n; i++) {
    x ^= x << 13; x >>>= 0
    x ^= x >>> 17
    x ^= x << 5; x >>>= 0
    out[i] = base + Math.floor(x * A / 4294967296)
  }
  return out
}

const codes = xorshiftCodes(g.seed, g.A, g.base, g.total)
const samples = []
for (let off = 0; off < g.total; off += g.sample) {
  const part = codes.subarray(off, Math.min(g.total, off + g.sample))
  let s = ''
  for (let i = 0; i < part.length; i += 8192) s += String.fromCharCode.apply(null, part.subarray(i, i + 8192))
  samples.push(s)
}

const t = new BPETokenizer()
for (const s of samples) t.addToCorpus(s)
assert.strictEqual(Object.keys(t.char_to_token).length, g.char_count)
const t0 = Date.now()
t.mergeUntil({ min_weight: g.min_weight, max_iterations: g.max_iterations })
const merge_s = (Date.now() - t0) / 1000
assert.deepStrictEqual(t.merge_tokens.map(([a, b, c]) => [a.index, b.index, c.original_weight]), g.merges)
assert.strictEqual(t.token_table.length, g.token_count)
assert.deepStrictEqual(t.token_table.map(x => x.weight), g.weights)

const h = crypto.createHash('sha256')
let n_ids = 0
for (const s of t.corpus_in_code) {
  const a = Array.from(s).map(ch => ch.codePointAt(0) - 1)
  a.push(-1)
  n_ids += a.length
  h.update(Buffer.from(new Int32Array(a).buffer))
}
assert.strictEqual(n_ids, g.final_ids_len)
assert.strictEqual(h.digest('hex'), g.final_ids_sha256)

const hv = crypto.createHash('sha256')
let n_vec = 0
const t1 = Date.now()
for (const s of samples) {
  const v = t.encodeToVector(s)
  v.push(-1)
  n_vec += v.length
  hv.update(Buffer.from(new Int32Array(v).buffer))
}
const enc_s = (Date.now() - t1) / 1000
assert.strictEqual(n_vec, g.vectors_len)
assert.strictEqual(hv.digest('hex'), g.vectors_sha256)
console.log('config2_gpu ok', JSON.stringify({ merges: g.merges.length, vectors_len: n_vec, merge_s, encode_s: enc_s }))
