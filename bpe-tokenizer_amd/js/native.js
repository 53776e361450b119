'use strict'
/**
 * native.js — internal: the N-API addon (addon/bpe_napi.node) and the option conventions shared
 * by the two drop-ins, core.js (BPETokenizer) and db.js (BPETokenizerDB).
 */
const path = require('path')

let native = null
function loadNative() {
  if (!native) native = require(path.join(__dirname, '..', 'addon', 'bpe_napi.node'))
  return native
}

/** Texts at least this long, with at least this many merges, are encoded on the GPU. */
const ENCODE_ON_DEVICE_CHARS = 1 << 16
const ENCODE_ON_DEVICE_MERGES = 16

/** JS `x || fallback` for numeric options, mapped onto the C ABI's int64 conventions. */
function maxLengthArg(max_length) {
  // core.ts:255,272: falsy -> unlimited; otherwise `len <= max_length`
  if (!max_length) return 0
  if (max_length === Infinity) return 0
  if (max_length === -Infinity) return -1
  let v = Math.floor(max_length) // integer lengths: len <= x  <=>  len <= floor(x)
  return v === 0 ? -1 : v // 0 < x < 1: nothing fits, but 0 means "unlimited" in the C ABI
}

function minWeightArg(options) {
  // core.ts:256: options?.min_weight || 2 ; core.ts:313: W < min_weight -> null
  let min_weight = (options && options.min_weight) || 2
  if (min_weight === Infinity) return Number.MAX_SAFE_INTEGER
  if (min_weight === -Infinity) return -Number.MAX_SAFE_INTEGER
  let v = Math.ceil(min_weight) // integer W: W < x  <=>  W < ceil(x)
  return v === 0 ? -1 : v // 0 would mean "default" in the C ABI; W >= 1 always passes -1
}

module.exports = {
  loadNative,
  maxLengthArg,
  minWeightArg,
  ENCODE_ON_DEVICE_CHARS,
  ENCODE_ON_DEVICE_MERGES,
}
