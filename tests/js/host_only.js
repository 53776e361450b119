// Host-side logic of the drop-in core.js, no GPU needed: fromJSON/toJSON round trips,
// encode/decode against the reference's golden vectors, error messages (core.ts:136,226-228,399,
// 440,467,481,483) and the corpus helpers (core.ts:55-75).
'use strict'
const assert = require('assert')
const path = require('path')
const fs = require('fs')
const core = require(path.join(__dirname, '..', '..', 'bpe-tokenizer_amd', 'js', 'core.js'))
const { BPETokenizer, compactMerge, EOF, FS, LF, CR } = core

const golden = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'small_cases.json')))
let checked = 0
for (const c of golden.cases) {
  if (!c.token_table.length) continue
  // rebuild the BPETokenizerJSON the reference would have exported for this case
  let chars = new Set()
  for (const s of c.samples) for (const ch of s) chars.add(ch)
  const json = {
    version: 2,
    char_count: chars.size,
    token_table: c.token_table,
    merge_codes: c.merges.map(([a, b], k) => [String.fromCodePoint(a + 1), String.fromCodePoint(b + 1),
      String.fromCodePoint(chars.size + k + 1)]),
  }
  const t = new BPETokenizer()
  t.fromJSON(json)
  assert.deepStrictEqual(t.toJSON(), json, c.name)
  c.samples.forEach((s, i) => {
    const want = c.vectors[i]
    if (typeof want === 'string') {
      assert.throws(() => t.encodeToVector(s), e => 'error: ' + e.message === want, c.name)
    } else {
      assert.deepStrictEqual(t.encodeToVector(s), want, c.name)
      assert.strictEqual(t.decodeVector(want), s, c.name)
      assert.strictEqual(t.decodeTokens(t.encodeToTokens(s)), s, c.name)
    }
  })
  checked++
}
assert(checked > 900)

// error messages
assert.throws(() => new BPETokenizer().fromJSON({ version: 1 }), /^Error: invalid format$/)
assert.throws(() => new BPETokenizer().compactVectorIndex(),
  e => e.message === 'token table is empty, have you called tokenizer.addToCorpus()?')
const t = new BPETokenizer()
t.fromJSON({ version: 2, char_count: 2, token_table: [['a', 1, 1], ['b', 1, 1]], merge_codes: [] })
assert.throws(() => t.encodeToCode('c'), e => e.message === 'unknown token, char: "c"')
assert.throws(() => t.decodeVector([5]), e => e.message === 'unknown vector index: 5')
assert.throws(() => t.restoreMerge(['\u0009', '\u0001', 1]), e => e.message === 'unknown token, a_code: "\\t"')
assert.throws(() => t.restoreMerge(['\u0001', '\u0009', 1]), e => e.message === 'unknown token, b_code: "\\t"')
// findNextMerge on an empty corpus is null without touching a device (core.ts:312)
assert.strictEqual(new BPETokenizer().findNextMerge(), null)
assert.deepStrictEqual(new BPETokenizer().corpus_in_code, [])
// helpers
assert.strictEqual(core.fileContentToCorpus('x'), FS + 'x' + EOF)
assert.deepStrictEqual(core.linesToCorpus(' a \nb'), ['\ra\n', '\rb\n'])
assert.deepStrictEqual(core.linesTrimmedToCorpus(' a \r\nb'), ['\r a \n', '\rb\n'])
assert.strictEqual(LF, '\n')
assert.strictEqual(CR, '\r')
const m = [{ code: 'A' }, { code: 'B' }, { weight: 7 }]
assert.deepStrictEqual(compactMerge(m), ['A', 'B', 7])
console.log('host_only ok', checked)
