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
 * encodeToCode (core.ts:392-409) runs on the GPU (bpe_encode_batch: the merge-rank encoder for
 * texts up to ENCODE_LDS_TOKENS tokens, apply-only replay passes above) when a per-call cost model
 * fitted to the measured crossover (profiles/r04_encode_crossover.json, MI355X + Node on the box's
 * host) says it beats the reference's own replay (one split/join per merge, kept below):
 *   JS replay     ~ 0.11 us per merge + chars x (0.03 + 0.00005 x merges) us
 *   device (LDS)  ~ 30 us per call + 1.6 us per greedy step (at most min(merges, 0.4 x chars))
 *                   + 0.05 us per char (id and code conversions, copies)
 *   device (long) ~ 10 us per merge (one replay pass each) + 0.05 us per char
 * In practice: long merge lists with short texts, and long texts.  BPE_ENCODE_DEVICE=0 keeps every
 * call on the JS replay, =1 sends every call with a merge to the device and lets its errors through
 * (tests).  By default a call the device cannot take falls back to the JS replay
 * (encodeIdsMaybeOnDevice): no addon or no HIP device (remembered for the owner's lifetime), or a
 * merge list with a token id the device encoder does not hold (>= BPE_MAX_VOCAB: remembered while
 * the owner keeps that list), so the drop-in encodes wherever the reference does.
 */
const ENCODE_LDS_TOKENS = 16384
const ENCODE_DEVICE = process.env.BPE_ENCODE_DEVICE

function encodeOnDevice(n_chars, n_merges) {
  if (n_chars < 2 || n_merges < 1 || ENCODE_DEVICE === '0') return false
  if (ENCODE_DEVICE === '1') return true
  const js = 0.11 * n_merges + n_chars * (0.03 + 0.00005 * n_merges)
  const dev =
    n_chars <= ENCODE_LDS_TOKENS
      ? 30 + 1.6 * Math.min(n_merges, 0.4 * n_chars) + 0.05 * n_chars
      : 10 * n_merges + 0.05 * n_chars
  return dev < js
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

/**
 * encodeIdsMaybeOnDevice when the cost model sends the call to the device and the device can take it,
 * else null (the caller then runs the reference's replay).  Only what the device cannot do is
 * remembered on the owner (non-enumerable `_enc_failed`): `true` when the encoder itself cannot be
 * made (no addon, no HIP device), the list when one of its merges has a token id the encoder does not
 * hold (the list keeps that merge: fromJSON replaces the list).  A text with such an id replays alone.
 * Any other failure (a device fault, out of memory) is reported once as a process warning and not
 * remembered: that call replays, and the next one tries the device again with its encoder rebuilt.
 */
const CAPABILITY_LIST = /merge token id out of range|more merges than token ids/
const CAPABILITY_TEXT = /token id out of range in text/
let warned = false
function encodeIdsMaybeOnDevice(owner, list, tripleOf, ids) {
  if (!encodeOnDevice(ids.length, list.length)) return null
  if (ENCODE_DEVICE !== '1' && (owner._enc_failed === true || owner._enc_failed === list))
    return null
  try {
    return encodeIdsOnDevice(owner, list, tripleOf, ids)
  } catch (e) {
    if (ENCODE_DEVICE === '1') throw e
    if (!Object.prototype.hasOwnProperty.call(owner, '_enc_failed'))
      Object.defineProperty(owner, '_enc_failed', { value: null, writable: true, enumerable: false })
    let msg = String((e && e.message) || e)
    if (!owner._encoder) {
      owner._enc_failed = true
    } else {
      // (the encoder may hold part of the list: the next call loads it again from the start)
      owner._enc_list = null
      if (CAPABILITY_LIST.test(msg)) owner._enc_failed = list
      else if (!CAPABILITY_TEXT.test(msg) && !warned) {
        warned = true
        process.emitWarning('bpe device encoder failed, this call replays the merges in JS: ' + msg)
      }
    }
    return null
  }
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
  encodeIdsMaybeOnDevice,
  idsToCode,
}
