// Throughput of the drop-in (bpe-tokenizer_amd/js/core.js) on the GPU: the reference's own
// surface end to end — addToCorpus of 1 MiB latin1 samples (xorshift32 seed 12345, 256-char
// alphabet, SURVEY.md §8(d)), then mergeUntil({min_weight: 2}) timed after a few warmup merges.
// Usage: node tools/bench_js.js [MiB=256] [merges=2000] [warmup=5]
'use strict'
const path = require('path')
const { BPETokenizer } = require(path.join(__dirname, '..', 'bpe-tokenizer_amd', 'js', 'core.js'))
const native = require(path.join(__dirname, '..', 'bpe-tokenizer_amd', 'addon', 'bpe_napi.node'))

const mib = +(process.argv[2] || 256), merges = +(process.argv[3] || 2000), warmup = +(process.argv[4] || 5)
let x = 12345
const t = new BPETokenizer()
const t0 = Date.now()
const part = new Array(8192)
for (let s = 0; s < mib; s++) {
  let str = ''
  for (let i = 0; i < (1 << 20); i += 8192) {
    for (let j = 0; j < 8192; j++) {
      x ^= x << 13; x >>>= 0; x ^= x >>> 17; x ^= x << 5; x >>>= 0
      part[j] = Math.floor(x * 256 / 4294967296)
    }
    str += String.fromCharCode.apply(null, part)
  }
  t.addToCorpus(str)
}
const ingest_s = (Date.now() - t0) / 1000
t.mergeUntil({ min_weight: 2, max_iterations: warmup })
const live0 = native.corpusSize(t.engine())[1]
const t1 = process.hrtime.bigint()
t.mergeUntil({ min_weight: 2, max_iterations: merges })
const dt = Number(process.hrtime.bigint() - t1) / 1e9
const done = t.merge_tokens.length - warmup
let scans = 0, live = live0
for (const [, , c] of t.merge_tokens.slice(warmup)) { scans += live; live -= c.original_weight }
console.log(JSON.stringify({
  what: 'drop-in core.js mergeUntil (device loop through N-API)', corpus_mib: mib,
  ingest_s, merges: done, warmup, seconds: dt, ms_per_merge: 1000 * dt / done,
  pair_scans_per_s: scans / dt, tokens: t.token_table.length,
}))
