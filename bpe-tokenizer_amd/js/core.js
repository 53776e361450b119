'use strict'
/**
 * core.js — drop-in replacement for beenotung/bpe-tokenizer's in-memory `BPETokenizer`
 * (reference: /root/reference/core.ts, v2.2.0), running the merge-training hot path on MI355X.
 *
 * Same exports, class surface, fields, options semantics and error messages as core.ts.  What
 * changes is where the corpus lives: `corpus_in_code` is not an array of JS strings but a flat
 * int32 token-id array in HBM, owned by libbpe (include/bpe.h) through the N-API addon
 * (addon/bpe_napi.node).  findNextMerge / applyMerge / mergeUntil / addToCorpus /
 * restoreToCorpus / restoreMerge drive the GPU; the token table, codes, JSON and encode/decode
 * bookkeeping stay here in JS exactly as in the reference.
 *
 * There is no CPU fallback: the first corpus operation creates the HIP engine and throws
 * `bpe native: ...` when no device is available.  Methods that never touch the corpus
 * (fromJSON, toJSON, encode*, decode*, compactVectorIndex) work without a GPU.
 *
 * Node 12 compatible (no `?.`, `??`, `String.prototype.replaceAll`).
 */
const {
  loadNative,
  maxLengthArg,
  minWeightArg,
  encodeIdsMaybeOnDevice,
  idsToCode,
} = require('./native')

/** @description file separator (core.ts:36) */
let FS = String.fromCharCode(28)
/** @description end of file (core.ts:39) */
let EOF = String.fromCharCode(4)
/** @description "\n" line feed, new line (core.ts:42) */
let LF = '\n'
/** @description "\r" carriage return (core.ts:45) */
let CR = '\r'

/** @description wrap with FS and EOF (core.ts:55-58) */
function fileContentToCorpus(content) {
  let text = content.toString()
  return FS + text + EOF
}

/** @description split into lines, wrap with \r and \n (core.ts:61-64) */
function linesToCorpus(text) {
  let lines = text.split('\n')
  return lines.map(line => '\r' + line.trim() + '\n')
}

/** @description split into lines, wrap with \r and \n, keep inner spaces (core.ts:67-75) */
function linesTrimmedToCorpus(text) {
  let lines = text.split('\n')
  return lines.map(line => {
    if (line.endsWith('\r')) {
      line = line.slice(0, line.length - 1)
    }
    return '\r' + line + '\n'
  })
}

/** `String.prototype.replaceAll(p, r)` for the single-code-point replacements used here. */
function replaceAll(s, from, to) {
  return s.split(from).join(to)
}

/** a merge_tokens entry [a, b, c] -> its token indices (the encoder's (a, b, c) triple) */
function tokenTriple(merge) {
  return [merge[0].index, merge[1].index, merge[2].index]
}

class BPETokenizer {
  constructor() {
    /** @description index for lookup (core.ts:79) */
    this.char_to_token = {}
    /** @description index for lookup (core.ts:82) */
    this.code_to_token = {}
    /** @description token.index -> Token (core.ts:85) */
    this.token_table = []
    /** @description for export (core.ts:88) */
    this.merge_tokens = []
    /** @description for encode (core.ts:91) */
    this.merge_codes = []
    /** @description for encode; skips zero-weight tokens (core.ts:97) */
    this.to_vector_index = null
    /** @description for decode; skips zero-weight tokens (core.ts:103) */
    this.from_vector_index = null
    Object.defineProperty(this, '_engine', { value: null, writable: true, enumerable: false })
    Object.defineProperty(this, '_registered', { value: 0, writable: true, enumerable: false })
    // applyMerge rewrites queued for the engine, as (a, b, c) index triples
    Object.defineProperty(this, '_pending', { value: [], writable: true, enumerable: false })
  }

  /**
   * @description the HIP engine holding the corpus (created on first use).  The corpus spans
   * several GPUs when BPE_NUM_GPUS > 1 (devices 0..n-1) or BPE_DEVICES lists device indices
   * ("0,1,2,3"); BPE_REDUCE=host exchanges the pair counts through host copies instead of RCCL
   * (any placement, e.g. two shards on one device).  The class surface does not change.
   */
  engine() {
    if (!this._engine) {
      let n = loadNative()
      let devices = null
      if (process.env.BPE_DEVICES) {
        devices = process.env.BPE_DEVICES.split(',').map(s => Number(s.trim()))
        if (devices.some(d => !Number.isInteger(d) || d < 0))
          throw new Error('bpe native: BPE_DEVICES must list device indices, e.g. "0,1,2,3"')
      } else if (+process.env.BPE_NUM_GPUS > 1) {
        devices = []
        for (let i = 0; i < +process.env.BPE_NUM_GPUS; i++) devices.push(i)
      }
      let reduce = process.env.BPE_REDUCE === 'host' ? 1 : 0
      if (devices && devices.length > 1) this._engine = n.createEngine(0, Int32Array.from(devices), reduce)
      else this._engine = n.createEngine(devices ? devices[0] : 0)
      this._registered = 0
    }
    this.flushMerges()
    this.registerTokens()
    return this._engine
  }

  /**
   * @description runs the queued applyMerge rewrites on the engine: a run of them (restoreMerge
   * replay) takes one apply-only pass each, the last one fused with the next count.
   */
  flushMerges() {
    let pending = this._pending
    if (pending.length === 0) return
    this._pending = []
    loadNative().applyMerges(this._engine, Int32Array.from(pending), 1)
  }

  /** @description tells the engine the UTF-16 length of every token it has not seen yet */
  registerTokens() {
    let { token_table } = this
    let n = loadNative()
    for (let i = this._registered; i < token_table.length; i++) {
      n.setTokenLen16(this._engine, token_table[i].index, token_table[i].chars.length)
    }
    this._registered = token_table.length
  }

  /**
   * @description added by this.addToCorpus() (core.ts:106).
   * Materialised from HBM on read; assigning replaces the device corpus (`= []` clears it).
   */
  get corpus_in_code() {
    if (!this._engine) return []
    let [ids, offsets] = loadNative().readCorpus(this.engine())
    let samples = []
    for (let s = 0; s + 1 < offsets.length; s++) {
      let code = ''
      for (let i = offsets[s]; i < offsets[s + 1]; i += 8192) {
        let end = Math.min(offsets[s + 1], i + 8192)
        let part = []
        for (let j = i; j < end; j++) part.push(ids[j] + 1)
        code += String.fromCodePoint.apply(null, part)
      }
      samples.push(code)
    }
    return samples
  }

  set corpus_in_code(samples) {
    if (!this._engine && (!samples || samples.length === 0)) return
    let engine = this.engine()
    let n = loadNative()
    n.clearCorpus(engine)
    for (let sample of samples || []) {
      let ids = []
      for (let code of sample) ids.push(code.codePointAt(0) - 1)
      n.addSample(engine, Int32Array.from(ids))
    }
  }

  /**
   * @description export token tables and merge list (core.ts:112-127).
   */
  toJSON() {
    return {
      version: 2,
      char_count: Object.keys(this.char_to_token).length,
      token_table: this.token_table.map(token => [
        token.chars,
        token.weight,
        token.original_weight,
      ]),
      merge_codes: this.merge_tokens.map(([a, b, c]) => [a.code, b.code, c.code]),
    }
  }

  /** @description restore from json (core.ts:130-171) */
  fromJSON(json) {
    if (
      json.version !== 2 ||
      !Array.isArray(json.token_table) ||
      !Array.isArray(json.merge_codes)
    )
      throw new Error('invalid format')
    let { char_count } = json
    let newInstance = new BPETokenizer()
    let { char_to_token, code_to_token, token_table, merge_tokens, merge_codes } = newInstance
    this.char_to_token = char_to_token
    this.code_to_token = code_to_token
    this.token_table = token_table
    this.merge_tokens = merge_tokens
    this.merge_codes = merge_codes
    this.to_vector_index = null
    this.from_vector_index = null
    this._pending = []
    if (this._engine) loadNative().clearCorpus(this._engine)
    this._registered = 0
    for (let [chars, weight, original_weight] of json.token_table) {
      let index = token_table.length
      let code = String.fromCodePoint(index + 1)
      let token = { chars, weight, original_weight, code, index }
      if (index < char_count) {
        char_to_token[chars] = token
      }
      code_to_token[code] = token
      token_table[index] = token
    }
    for (let [a_code, b_code, c_code] of json.merge_codes) {
      let a = code_to_token[a_code]
      let b = code_to_token[b_code]
      let c = code_to_token[c_code]
      merge_tokens.push([a, b, c])
      merge_codes.push([a.code + b.code, c.code])
    }
    if (this._engine) this.registerTokens()
    this.compactVectorIndex()
  }

  invalidateVectorIndex() {
    this.to_vector_index = null
    this.from_vector_index = null
  }

  /**
   * @description add new content to corpus (core.ts:182-207).
   * Token weights are updated when adding content.
   */
  addToCorpus(content) {
    let { char_to_token, code_to_token, token_table } = this
    let ids = []
    for (let char of content) {
      let token = char_to_token[char]
      if (!token) {
        let index = token_table.length
        let code = String.fromCodePoint(index + 1)
        token = { chars: char, weight: 1, original_weight: 1, code, index }
        char_to_token[char] = token
        code_to_token[code] = token
        token_table.push(token)
      } else {
        token.weight++
        token.original_weight++
      }
      ids.push(token.index)
    }
    let engine = this.engine()
    loadNative().addSample(engine, Int32Array.from(ids))
  }

  /**
   * @description restore content to corpus (after restart) for continuous merging
   * (core.ts:213-216).  Token weights are not updated when restoring content.
   */
  restoreToCorpus(content) {
    let content_in_code = this.encodeToCode(content)
    let ids = []
    for (let code of content_in_code) ids.push(code.codePointAt(0) - 1)
    let engine = this.engine()
    loadNative().addSample(engine, Int32Array.from(ids))
  }

  /**
   * @description skip zero-weight tokens to reduce range of vector index (core.ts:222-241).
   */
  compactVectorIndex() {
    let { token_table } = this
    let token_count = token_table.length
    if (token_count == 0) {
      throw new Error(`token table is empty, have you called tokenizer.addToCorpus()?`)
    }
    let to_vector_index = (this.to_vector_index = [])
    let from_vector_index = (this.from_vector_index = [])
    let vector_index = 0
    for (let index = 0; index < token_count; index++) {
      let token = token_table[index]
      if (token.weight > 0) {
        to_vector_index[index] = vector_index
        from_vector_index[vector_index] = index
        vector_index++
      }
    }
  }

  /**
   * @description one full pass over the corpus on the GPU (core.ts:247-326): the most frequent
   * adjacent pair under the reference's tie-break, or null.
   */
  findNextMerge(options) {
    let max_length = options && options.max_length
    if (!this._engine) return null
    let engine = this.engine()
    let found = loadNative().findNextMerge(engine, maxLengthArg(max_length), minWeightArg(options))
    if (!found) return null
    let [a_index, b_index, weight] = found
    let max_a = this.token_table[a_index]
    let max_b = this.token_table[b_index]
    let new_index = this.token_table.length
    let new_code = String.fromCodePoint(new_index + 1)
    let max_c = {
      chars: max_a.chars + max_b.chars,
      weight: weight,
      original_weight: weight,
      code: new_code,
      index: new_index,
    }
    return [max_a, max_b, max_c]
  }

  /**
   * @description applies a merge to the tables and rewrites the corpus in HBM (core.ts:332-360).
   */
  applyMerge(merge) {
    let { code_to_token, token_table, merge_tokens, merge_codes } = this
    let [a, b, c] = merge

    let from_code = a.code + b.code
    let to_code = c.code

    a.weight -= c.weight
    b.weight -= c.weight

    this.invalidateVectorIndex()

    code_to_token[c.code] = c
    token_table.push(c)

    merge_tokens.push(merge)
    merge_codes.push([from_code, to_code])

    if (this._engine) {
      // (queued: the engine rewrites the corpus at its next use, see flushMerges)
      this._pending.push(a.index, b.index, c.index)
    }
  }

  /**
   * @description call `findNextMerge()` and `applyMerge()` in loop (core.ts:365-383).
   * The loop runs on the device (bpe_merge_until: the merge decisions stay in HBM, one host round
   * trip per batch of iterations); the merges it made are then entered into the tables exactly as
   * findNextMerge + applyMerge would have, in order.
   */
  mergeUntil(options) {
    let max_iterations = options && options.max_iterations
    // core.ts:376: `!max_iterations || iteration <= max_iterations`
    let it_arg = 0
    if (max_iterations && max_iterations !== Infinity) {
      if (!(max_iterations >= 1)) return
      it_arg = Math.floor(max_iterations)
    }
    if (!this._engine) return // an empty corpus: findNextMerge returns null (core.ts:312)
    let engine = this.engine()
    let max_length = options && options.max_length
    let abw = loadNative().mergeUntil(engine, maxLengthArg(max_length), minWeightArg(options), it_arg)
    let { code_to_token, token_table, merge_tokens, merge_codes } = this
    for (let i = 0; i < abw.length; i += 3) {
      let a = token_table[abw[i]]
      let b = token_table[abw[i + 1]]
      let weight = abw[i + 2]
      let index = token_table.length
      let c = {
        chars: a.chars + b.chars,
        weight: weight,
        original_weight: weight,
        code: String.fromCodePoint(index + 1),
        index: index,
      }
      // applyMerge's bookkeeping (core.ts:345-354); the corpus is already rewritten
      a.weight -= c.weight
      b.weight -= c.weight
      code_to_token[c.code] = c
      token_table.push(c)
      merge_tokens.push([a, b, c])
      merge_codes.push([a.code + b.code, c.code])
    }
    if (abw.length) this.invalidateVectorIndex()
    // the engine registered the UTF-16 length of every token it created (core.ts:318)
    this._registered = token_table.length
  }

  /**
   * @description encode to binary string (core.ts:392-409).
   * With enough merges the text is encoded on the GPU by the merge-rank encoder (bpe_encode_batch:
   * the lowest-ranked merge present is rewritten until none is, which equals the reference's
   * in-order replaceAll of every merge; texts over ENCODE_LDS_TOKENS tokens are replayed by apply-only passes
   * over HBM).  Short merge lists keep the reference's replay here (see native.js).
   */
  encodeToCode(content) {
    let { char_to_token } = this

    let content_in_code = ''
    let ids = []
    for (let char of content) {
      let token = char_to_token[char]
      if (!token) {
        throw new Error('unknown token, char: ' + JSON.stringify(char))
      }
      ids.push(token.index)
      content_in_code += token.code
    }

    let out = encodeIdsMaybeOnDevice(this, this.merge_tokens, tokenTriple, ids)
    if (out) return idsToCode(out, 0, out.length)

    for (let [from_code, to_code] of this.merge_codes) {
      content_in_code = replaceAll(content_in_code, from_code, to_code)
    }

    return content_in_code
  }

  /** core.ts:411-422 */
  encodeToTokens(content) {
    let { code_to_token } = this
    let content_in_code = this.encodeToCode(content)
    let tokens = []
    for (let code of content_in_code) {
      tokens.push(code_to_token[code])
    }
    return tokens
  }

  /** core.ts:424-445 */
  encodeToVector(content) {
    let { code_to_token, to_vector_index } = this

    if (!to_vector_index) {
      this.compactVectorIndex()
      to_vector_index = this.to_vector_index
    }

    let content_in_code = this.encodeToCode(content)

    let vector = []
    for (let code of content_in_code) {
      let index = code_to_token[code].index
      if (index in to_vector_index) {
        vector.push(to_vector_index[index])
      } else {
        throw new Error(`unknown token index: ${index}`)
      }
    }

    return vector
  }

  /** core.ts:447-453 */
  decodeTokens(tokens) {
    let content = ''
    for (let token of tokens) {
      content += token.chars
    }
    return content
  }

  /** core.ts:455-471 */
  decodeVector(vector) {
    let { from_vector_index, token_table } = this
    if (!from_vector_index) {
      this.compactVectorIndex()
      from_vector_index = this.from_vector_index
    }
    let content = ''
    for (let vector_index of vector) {
      if (vector_index in from_vector_index) {
        let index = from_vector_index[vector_index]
        content += token_table[index].chars
      } else {
        throw new Error(`unknown vector index: ${vector_index}`)
      }
    }
    return content
  }

  /**
   * @description restore merge produced from `compactMerge(this.findNextMerge())`
   * (core.ts:477-494).  To be used after restart for continuous merging.
   */
  restoreMerge(compactMerge) {
    let { code_to_token } = this
    let [a_code, b_code, c_weight] = compactMerge
    let a = code_to_token[a_code]
    if (!a) throw new Error(`unknown token, a_code: ${JSON.stringify(a_code)}`)
    let b = code_to_token[b_code]
    if (!b) throw new Error(`unknown token, b_code: ${JSON.stringify(b_code)}`)
    let index = this.token_table.length
    let code = String.fromCodePoint(index + 1)
    let c = {
      chars: a.chars + b.chars,
      weight: c_weight,
      original_weight: c_weight,
      code,
      index,
    }
    this.applyMerge([a, b, c])
  }
}

/**
 * @description to store MergeToken in compact format (core.ts:500-503)
 */
function compactMerge(merge) {
  let [a, b, c] = merge
  return [a.code, b.code, c.weight]
}

module.exports = {
  FS,
  EOF,
  LF,
  CR,
  fileContentToCorpus,
  linesToCorpus,
  linesTrimmedToCorpus,
  BPETokenizer,
  compactMerge,
}
