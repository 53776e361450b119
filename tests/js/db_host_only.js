// Host-side logic of the db.js twin (BPETokenizerDB, db/core.ts) over a real sqlite database, no
// GPU needed: schema, fromJSON/toJSON round trips and encode/decode against the reference's golden
// vectors, addToCorpus token rows and weights, the proxy views and the error messages
// (db/core.ts:171,220,273,457,498,526,540,542).
'use strict'
const assert = require('assert')
const fs = require('fs')
const os = require('os')
const path = require('path')
const { connectDB } = require('./sqlite_bridge')
const dbjs = require(path.join(__dirname, '..', '..', 'bpe-tokenizer_amd', 'js', 'db.js'))
const { BPETokenizerDB, resetBPETokenizerDB, EOF } = dbjs

const file = path.join(fs.mkdtempSync(path.join(os.tmpdir(), 'bpe-db-')), 'host.sqlite3')
const db = connectDB(file)

// golden cases: the reference's exported JSON imported into the DB twin, encode/decode vectors
const golden = JSON.parse(fs.readFileSync(path.join(__dirname, '..', 'golden', 'small_cases.json')))
let checked = 0
for (const c of golden.cases.filter((_, i) => i % 5 === 0)) {
  if (!c.token_table.length) continue
  let chars = new Set()
  for (const s of c.samples) for (const ch of s) chars.add(ch)
  const json = {
    version: 2,
    char_count: chars.size,
    token_table: c.token_table,
    merge_codes: c.merges.map(([a, b], k) => [String.fromCodePoint(a + 1), String.fromCodePoint(b + 1),
      String.fromCodePoint(chars.size + k + 1)]),
  }
  const t = new BPETokenizerDB({ db })
  t.fromJSON(json)
  assert.deepStrictEqual(t.toJSON(), json, c.name)
  c.samples.forEach((s, i) => {
    const want = c.vectors[i]
    if (typeof want === 'string') {
      // (the DB twin names ids where core.ts names indices: db/core.ts:498 vs core.ts:440)
      assert.throws(() => t.encodeToVector(s), c.name)
    } else {
      assert.deepStrictEqual(t.encodeToVector(s), want, c.name)
      assert.strictEqual(t.decodeVector(want), s, c.name)
      assert.strictEqual(t.decodeTokens(t.encodeToTokens(s)), s, c.name)
    }
  })
  // a second instance on the same database sees the same tables (db/core.ts:121-132)
  const u = new BPETokenizerDB({ db })
  assert.deepStrictEqual(u.toJSON(), json, c.name)
  assert.deepStrictEqual(u.merge_codes, t.merge_codes, c.name)
  checked++
}
assert(checked > 150, checked)

// addToCorpus without a device: token rows, char rows, weights (db/core.ts:216-246)
resetBPETokenizerDB(db)
let t = new BPETokenizerDB({ db })
t.addToCorpus(1, EOF + 'abca' + EOF)
t.addToCorpus(7, 'b')
assert.throws(() => t.addToCorpus(7, 'x'), e => e.message === 'corpus already added to database')
assert.strictEqual(t.getLastCorpusId(), 7)
assert.strictEqual(t.hasCorpus(1), true)
assert.strictEqual(t.hasCorpus(2), false)
const tokens = t.proxy.token
assert.strictEqual(tokens.length, 4)
assert.deepStrictEqual(
  [1, 2, 3, 4].map(i => [tokens[i].chars, tokens[i].weight, tokens[i].original_weight, tokens[i].code]),
  [[EOF, 2, 2, '\u0001'], ['a', 2, 2, '\u0002'], ['b', 2, 2, '\u0003'], ['c', 1, 1, '\u0004']],
)
assert.strictEqual(t.proxy.char_token.length, 4)
assert.deepStrictEqual(Array.from(t.proxy.corpus).map(r => [r.id, r.content_code]),
  [[1, '\u0001\u0002\u0003\u0004\u0002\u0001'], [7, '\u0003']])
assert.strictEqual(1 in t.proxy.corpus, true)
assert.strictEqual(2 in t.proxy.corpus, false)
// writes through a proxy row reach the table, as better-sqlite3-proxy rows do
tokens[4].weight = 9
assert.strictEqual(new BPETokenizerDB({ db }).char_to_token['c'].weight, 9)
tokens[4].weight = 1
// restoreToCorpus encodes with the current tables and leaves the weights alone (db/core.ts:252-256)
t.restoreToCorpus(9, 'cab')
assert.strictEqual(t.proxy.corpus[9].content_code, '\u0004\u0002\u0003')
assert.strictEqual(tokens[2].weight, 2)
// encode before any merge: the vector index skips nothing
assert.deepStrictEqual(t.encodeToVector('abc'), [1, 2, 3])
assert.strictEqual(t.decodeVector([3, 0]), 'c' + EOF)

// error messages
assert.throws(() => t.fromJSON({ version: 1 }), e => e.message === 'invalid format')
resetBPETokenizerDB(db)
assert.throws(() => new BPETokenizerDB({ db }).compactVectorIndex(),
  e => e.message === 'token table is empty, have you called tokenizer.addToCorpus()?')
t = new BPETokenizerDB({ db })
t.fromJSON({ version: 2, char_count: 2, token_table: [['a', 1, 1], ['b', 1, 1]], merge_codes: [] })
assert.throws(() => t.encodeToCode('c'), e => e.message === 'unknown token, char: "c"')
assert.throws(() => t.decodeVector([5]), e => e.message === 'unknown vector index: 5')
assert.throws(() => t.restoreMerge(['\u0009', '\u0001', 1]), e => e.message === 'unknown token, a_code: "\\t"')
assert.throws(() => t.restoreMerge(['\u0001', '\u0009', 1]), e => e.message === 'unknown token, b_code: "\\t"')
assert.throws(() => t.applyMerge([t.char_to_token.a, t.char_to_token.b, { chars: 'ab', weight: 1 }]),
  e => e.message === 'missing id in token c')
// a failed transaction leaves the tables as they were
assert.strictEqual(t.proxy.merge.length, 0)
assert.strictEqual(t.char_to_token.a.weight, 1)

db.close()
console.log('db_host_only ok', checked)
