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

/**
 * encodeToCode (core.ts:392-409) runs on the GPU (the merge-rank encoder, bpe_encode_batch) for a
 * merge list of at least ENCODE_ON_DEVICE_MERGES merges, or a text of at least
 * ENCODE_ON_DEVICE_CHARS chars with at least ENCODE_ON_DEVICE_MIN_MERGES merges.  Below that the
 * reference's own replay (one split/join per merge, ~0.45 us per merge on a short text in Node)
 * finishes before one device round trip would (profiles/r04_encode_crossover.json).
 * BPE_ENCODE_MIN_MERGES overrides the first threshold (e.g. host-only runs without a device).
 */
const ENCODE_ON_DEVICE_CHARS = 1 << 16
const ENCODE_ON_DEVICE_MIN_MERGES = 16
const ENCODE_ON_DEVICE_MERGES = +process.env.BPE_ENCODE_MIN_MERGES || 128

function encodeOnDevice(n_chars, n_merges) {
  if (n_chars < 2 || n_merges < ENCODE_ON_DEVICE_MIN_MERGES) return false
  return n_merges >= ENCODE_ON_DEVICE_MERGES || n_chars >= ENCODE_ON_DEVICE_CHARS
}

/**
 * The owner's device encoder (bpe_encoder_*), holding the merge list `list` as a rank table; the
 * merges appended to the list since the last call are appended to it (applyMerge, restoreMerge,
 * mergeUntil), and a replaced or shortened list (fromJSON) rebuilds it.  tripleOf(entry) -> the
 * entry's (a, b, c) token indices.  The owner keeps the handle in non-enumerable fields.
 */
function syncEncoder(owner, list, tripleOf) {
  let n = loadNative()
  if (!owner._encoder) {
    for (let k of ['_encoder', '_enc_list', '_enc_n', '_enc_last'])
      if (!Object.prototype.hasOwnProperty.call(owner, k))
        Object.defineProperty(owner, k, { value: null, writable: true, enumerable: false })
    owner._encoder = n.createEncoder(0)
    owner._enc_list = null
  }
  let have = owner._enc_n || 0
  if (owner._enc_list !== list || have > list.length || (have && list[have - 1] !== owner._enc_last)) {
    n.encoderClear(owner._encoder)
    owner._enc_list = list
    have = 0
  }
  if (have < list.length) {
    let k = list.length - have
    let abc = new Int32Array(3 * k)
    for (let i = 0; i < k; i++) {
      let t = tripleOf(list[have + i])
      abc[3 * i] = t[0]
      abc[3 * i + 1] = t[1]
      abc[3 * i + 2] = t[2]
    }
    n.encoderAddMerges(owner._encoder, abc)
  }
  owner._enc_n = list.length
  owner._enc_last = list.length ? list[list.length - 1] : null
  return owner._encoder
}

/** one text's token ids through the owner's merges on the device -> Int32Array of ids */
function encodeIdsOnDevice(owner, list, tripleOf, ids) {
  let enc = syncEncoder(owner, list, tripleOf)
  let res = loadNative().encodeBatch(enc, Int32Array.from(ids), Float64Array.of(0, ids.length))
  return res[0]
}

/** engine ids -> code point string (code = index + 1, core.ts:149) */
function idsToCode(ids, begin, end) {
  let parts = []
  for (let i = begin; i < end; i += 8192) {
    let part = []
    let stop = Math.min(end, i + 8192)
    for (let j = i; j < stop; j++) part.push(ids[j] + 1)
    parts.push(String.fromCodePoint.apply(null, part))
  }
  return parts.join('')
}

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
  encodeOnDevice,
  encodeIdsOnDevice,
  idsToCode,
}
