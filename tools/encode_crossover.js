// Where encodeToCode (core.ts:392-409) should leave the reference's JS replay for the device
// encoder: one text per call through the drop-in, both ways, for merge lists of several lengths
// and texts of several lengths.  The tokenizer is trained through the drop-in on words of a
// 10-letter alphabet (xorshift32), as a tokenizer for text would be.  Prints one JSON object:
// per (merges, chars) the microseconds per call of the JS replay (split/join per merge, as
// core.ts:404-406) and of the device path (bpe_encode_batch: copy in, merge-rank kernel, copy out).
// Usage: node tools/encode_crossover.js
'use strict'
const path = require('path')
const { BPETokenizer } = require(path.join(__dirname, '..', 'bpe-tokenizer_amd', 'js', 'core.js'))
const nat = require(path.join(__dirname, '..', 'bpe-tokenizer_amd', 'js', 'native.js'))

let x = 4242
const rnd = () => { x ^= x << 13; x ^= x >>> 17; x ^= x << 5; return (x >>> 0) / 4294967296 }
const word = () => { let w = ''; const l = 1 + Math.floor(rnd() * 7); for (let i = 0; i < l; i++) w += 'abcdefghij'[Math.floor(rnd() * 10)]; return w }
const text = n => { let s = ''; while (s.length < n) s += word() + ' '; return s.slice(0, n) }

const t = new BPETokenizer()
for (let i = 0; i < 512; i++) t.addToCorpus(text(1 << 14))
t.mergeUntil({ min_weight: 2, max_iterations: 4096 })
const all = t.merge_tokens.slice()
const codes = t.merge_codes.slice()

function time(f) {
  f()
  const t0 = process.hrtime.bigint()
  let reps = 0
  while (Number(process.hrtime.bigint() - t0) < 2e8) { f(); reps++ }
  return Number(process.hrtime.bigint() - t0) / reps / 1e3
}

const rows = []
for (const m of [16, 32, 64, 128, 256, 1024, 4096]) {
  if (m > all.length) break
  const holder = {}
  const list = all.slice(0, m)
  const mc = codes.slice(0, m)
  for (const n of [16, 64, 256, 1024, 4096, 16384]) {
    const s = text(n)
    const js = time(() => {
      let c = ''
      for (const ch of s) c += t.char_to_token[ch].code
      for (const [f, to] of mc) c = c.split(f).join(to)
      return c
    })
    const dev = time(() => {
      const ids = []
      for (const ch of s) ids.push(t.char_to_token[ch].index)
      const out = nat.encodeIdsOnDevice(holder, list, mt => [mt[0].index, mt[1].index, mt[2].index], ids)
      return nat.idsToCode(out, 0, out.length)
    })
    rows.push({ merges: m, chars: n, js_us: +js.toFixed(2), device_us: +dev.toFixed(2), device_wins: dev < js })
  }
}
console.log(JSON.stringify({ what: 'encodeToCode per call: JS replay vs device encoder', trained_merges: all.length, rows }))
