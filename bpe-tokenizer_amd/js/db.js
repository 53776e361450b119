'use strict'
/**
 * db.js — drop-in replacement for beenotung/bpe-tokenizer's sqlite-backed `BPETokenizerDB`
 * (reference: /root/reference/db/core.ts, db/proxy.ts, db/migration.ts), with the merge-training
 * hot path on MI355X (SURVEY.md §8(f) rank 4).
 *
 * The database stays the system of record, with the reference's schema (corpus, token,
 * char_token, merge), so a database written by the reference opens here and the other way round.
 * What moves is the work of findNextMerge / applyMerge / mergeUntil (db/core.ts:290-441):
 *   - the corpus rows are loaded once, in id order, into the HIP engine (libbpe through the N-API
 *     addon, the same engine as core.js); ids are code points (db/core.ts:226-227), engine ids
 *     are code point - 1, so the tie-break on a.id + b.id (db/core.ts:337) orders alike;
 *   - findNextMerge is one pass on the device (bpe_find_next_merge);
 *   - applyMerge rewrites the corpus in HBM (bpe_apply_merge), then writes back exactly the rows
 *     the merge changed: a rewrite shortens every row it touches, so the rows whose length fell
 *     (bpe_sample_lengths) are read back (bpe_read_samples) and updated, in place of the
 *     reference's `like '%code%'` scan + `replaceAll` (db/core.ts:399-417);
 *   - mergeUntil runs the device-resident loop (bpe_merge_until) and writes the token table, the
 *     merge rows and the changed corpus rows once at the end, in one transaction.
 * Token rows, weights, merge rows, JSON import/export, encode/decode keep the reference's
 * semantics and error messages.  There is no CPU fallback for the corpus work: without a device
 * the first corpus operation throws `bpe native: ...`.
 *
 * `db` is a better-sqlite3-helper instance, as for the reference (prepare / transaction /
 * migrate).  The engine mirrors the corpus table from its first use on: rows must be changed
 * through this object (addToCorpus / restoreToCorpus / applyMerge ...), as with the reference's
 * cached merge_codes and char_to_token.
 *
 * Node 12 compatible.
 */
const {
  loadNative,
  maxLengthArg,
  minWeightArg,
  encodeIdsMaybeOnDevice,
  idsToCode,
} = require('./native')
const { EOF } = require('./core')

/** @description the reference's schema (db/migration.ts), so either side opens the other's file */
const migrationSQL = /* sql */ `
-- Up
create table if not exists corpus (
  id integer primary key
, content_code text not null
, created_at text not null default CURRENT_TIMESTAMP
, updated_at text null
);
create table if not exists token (
  id integer primary key
, chars text not null
, weight integer not null
, original_weight integer not null
, code text not null
, created_at text not null default CURRENT_TIMESTAMP
, updated_at text null
);
create table if not exists char_token (
  id integer primary key
, created_at text not null default CURRENT_TIMESTAMP
, updated_at text null
);
create table if not exists merge (
  id integer primary key
, a_id integer not null references token(id)
, b_id integer not null references token(id)
, c_id integer not null references token(id)
, created_at text not null default CURRENT_TIMESTAMP
, updated_at text null
);

-- Down
drop table if exists merge;
drop table if exists char_token;
drop table if exists token;
drop table if exists corpus;
`

const COLUMNS = {
  corpus: ['id', 'content_code'],
  token: ['id', 'chars', 'weight', 'original_weight', 'code'],
  char_token: ['id'],
  merge: ['id', 'a_id', 'b_id', 'c_id'],
}
const REFS = {
  char_token: { token: ['id', 'token'] },
  merge: { a: ['a_id', 'token'], b: ['b_id', 'token'], c: ['c_id', 'token'] },
}

/**
 * A live row: reads hit the database, writes are `update` statements (the row objects of
 * better-sqlite3-proxy that db/proxy.ts hands out).
 */
function liveRow(db, table, id) {
  let row = {}
  for (let col of COLUMNS[table]) {
    if (col === 'id') {
      Object.defineProperty(row, 'id', { value: id, enumerable: true })
      continue
    }
    let get = db.prepare(`select ${col} from ${table} where id = ?`).pluck()
    let set = db.prepare(`update ${table} set ${col} = ? where id = ?`)
    Object.defineProperty(row, col, {
      enumerable: true,
      get: () => get.get(id),
      set: v => set.run(v, id),
    })
  }
  let refs = REFS[table] || {}
  for (let name of Object.keys(refs)) {
    let [field, target] = refs[name]
    Object.defineProperty(row, name, {
      enumerable: false,
      get: () => liveRow(db, target, row[field]),
    })
  }
  return row
}

/**
 * A table as an array indexed by id (db/proxy.ts createProxy): `t[id]`, `t[id] = row`,
 * `id in t`, `t.length`, `t.length = 0`, `t.push(row)`, `for (row of t)` (id order).
 */
function tableProxy(db, table) {
  let cols = COLUMNS[table]
  let count = db.prepare(`select count(*) from ${table}`).pluck()
  let has = db.prepare(`select count(*) from ${table} where id = ?`).pluck()
  let ids = db.prepare(`select id from ${table} order by id asc`).pluck()
  let upsert = db.prepare(
    `insert or replace into ${table} (${cols.join(', ')}) values (${cols.map(c => ':' + c).join(', ')})`,
  )
  let insert = db.prepare(
    `insert into ${table} (${cols.slice(1).join(', ')}) values (${cols.slice(1).map(c => ':' + c).join(', ')})`,
  )
  let clear = db.prepare(`delete from ${table}`)
  let bind = (row, id) => {
    let b = {}
    for (let c of cols) b[c] = c === 'id' ? id : row[c] === undefined ? null : row[c]
    return b
  }
  let target = []
  return new Proxy(target, {
    get(_, key) {
      if (key === 'length') return count.get()
      if (key === 'push')
        return (...rows) => {
          for (let row of rows) insert.run(bind(row, null))
          return count.get()
        }
      if (key === Symbol.iterator)
        return function* () {
          for (let id of ids.all()) yield liveRow(db, table, id)
        }
      if (typeof key === 'string' && /^\d+$/.test(key)) {
        let id = +key
        return has.get(id) ? liveRow(db, table, id) : undefined
      }
      return target[key]
    },
    set(_, key, value) {
      if (key === 'length') {
        if (value !== 0) throw new Error('only `length = 0` is supported on a table proxy')
        clear.run()
        return true
      }
      if (typeof key === 'string' && /^\d+$/.test(key)) {
        upsert.run(bind(value, +key))
        return true
      }
      target[key] = value
      return true
    },
    has(_, key) {
      if (typeof key === 'string' && /^\d+$/.test(key)) return has.get(+key) > 0
      return key in target
    },
  })
}

function createProxy(options) {
  let { db } = options
  return {
    corpus: tableProxy(db, 'corpus'),
    token: tableProxy(db, 'token'),
    char_token: tableProxy(db, 'char_token'),
    merge: tableProxy(db, 'merge'),
  }
}

/** code point string -> engine ids (code point - 1) */
function codeToIds(code) {
  let ids = []
  for (let ch of code) ids.push(ch.codePointAt(0) - 1)
  return Int32Array.from(ids)
}

/** a merge_codes entry [from_code, to_code] -> its (a, b, c) token indices (id - 1) */
function codeTriple(merge) {
  let pair = Array.from(merge[0])
  return [pair[0].codePointAt(0) - 1, pair[1].codePointAt(0) - 1, merge[1].codePointAt(0) - 1]
}

class BPETokenizerDB {
  constructor(options) {
    let { db } = options
    db.migrate({ migrations: [migrationSQL] })
    this.db = db
    this.proxy = createProxy({ db })
    /** @description index for lookup (db/core.ts:21) */
    this.char_to_token = {}
    /** @description index for lookup (db/core.ts:24) */
    this.code_to_token = {}
    /** @description for encode (db/core.ts:27) */
    this.merge_codes = []
    this.to_vector_index = null
    this.from_vector_index = null

    this.select_last_corpus_id = db.prepare(`select max(id) from corpus`).pluck()
    this.select_corpus_rows = db.prepare(`select id, content_code from corpus order by id asc`)
    this.select_token_table = db.prepare(
      `select id, chars, weight, original_weight, code from token order by id asc`,
    )
    this.select_char_ids = db.prepare(`select id from char_token order by id asc`).pluck()
    this.select_merge = db.prepare(`select a_id, b_id, c_id from merge order by id asc`)
    this.select_weighted_token = db.prepare(`select id from token where weight > 0 order by id asc`).pluck()
    this.count_token = db.prepare(`select count(*) from token`).pluck()
    this.has_corpus = db.prepare(`select count(*) from corpus where id = ?`).pluck()
    this.insert_corpus = db.prepare(`insert into corpus (id, content_code) values (:id, :content_code)`)
    this.upsert_corpus = db.prepare(`insert or replace into corpus (id, content_code) values (:id, :content_code)`)
    this.update_corpus = db.prepare(`update corpus set content_code = :content_code where id = :id`)
    this.insert_token = db.prepare(
      `insert or replace into token (id, chars, weight, original_weight, code) values (:id, :chars, :weight, :original_weight, :code)`,
    )
    this.update_weight = db.prepare(`update token set weight = :weight where id = :id`)
    this.update_weights = db.prepare(
      `update token set weight = :weight, original_weight = :original_weight where id = :id`,
    )
    this.insert_char = db.prepare(`insert or replace into char_token (id) values (?)`)
    this.insert_merge = db.prepare(`insert into merge (a_id, b_id, c_id) values (:a_id, :b_id, :c_id)`)

    Object.defineProperty(this, '_engine', { value: null, writable: true, enumerable: false })
    Object.defineProperty(this, '_rows', { value: [], writable: true, enumerable: false })
    Object.defineProperty(this, '_lens', { value: [], writable: true, enumerable: false })
    Object.defineProperty(this, '_registered', { value: 0, writable: true, enumerable: false })
    Object.defineProperty(this, '_tokens', { value: [], writable: true, enumerable: false })

    // the token table, cached as write-through rows (db/core.ts:121-132)
    let char_ids = new Set(this.select_char_ids.all())
    for (let row of this.select_token_table.all()) {
      let token = this.tokenRow(row)
      if (char_ids.has(token.id)) this.char_to_token[token.chars] = token
      this.code_to_token[token.code] = token
    }
    for (let m of this.select_merge.all()) {
      let a = this._tokens[m.a_id]
      let b = this._tokens[m.b_id]
      let c = this._tokens[m.c_id]
      this.merge_codes.push([a.code + b.code, c.code])
    }

    // db/core.ts:134-138
    this.addToCorpus = db.transaction(this.addToCorpus)
    this.findNextMerge = db.transaction(this.findNextMerge)
    this.applyMerge = db.transaction(this.applyMerge)
    this.mergeUntil = db.transaction(this.mergeUntil)
    this.toJSON = db.transaction(this.toJSON)
    this.fromJSON = db.transaction(this.fromJSON)
  }

  /**
   * @description a token held in memory whose `weight` / `original_weight` writes go to the
   * token table (the proxy rows of db/core.ts:386-387 do the same).
   */
  tokenRow(row) {
    let { update_weight, update_weights } = this
    let weight = row.weight
    let original_weight = row.original_weight
    let token = {}
    Object.defineProperty(token, 'id', { value: row.id, enumerable: true })
    Object.defineProperty(token, 'chars', { value: row.chars, enumerable: true })
    Object.defineProperty(token, 'weight', {
      enumerable: true,
      get: () => weight,
      set: v => {
        weight = v
        update_weight.run({ id: row.id, weight: v })
      },
    })
    Object.defineProperty(token, 'original_weight', {
      enumerable: true,
      get: () => original_weight,
      set: v => {
        original_weight = v
        update_weights.run({ id: row.id, weight, original_weight: v })
      },
    })
    Object.defineProperty(token, 'code', { value: row.code, enumerable: true })
    this._tokens[row.id] = token
    return token
  }

  /** @description delete all tokens and corpus from database, called by fromJSON() (db/core.ts:142-147) */
  reset() {
    let { db } = this
    this.dropEngine()
    resetBPETokenizerDB(db)
    let that = new BPETokenizerDB({ db })
    Object.assign(this, that)
    this._tokens = that._tokens
  }

  /** @description for in-memory BPETokenizer (db/core.ts:150-162) */
  toJSON() {
    let token_table = this.select_token_table.all()
    let code = []
    for (let t of token_table) code[t.id] = t.code
    return {
      version: 2,
      char_count: this.select_char_ids.all().length,
      token_table: token_table.map(token => [token.chars, token.weight, token.original_weight]),
      merge_codes: this.select_merge.all().map(m => [code[m.a_id], code[m.b_id], code[m.c_id]]),
    }
  }

  /** @description delete all existing tokens and corpus, then import tokens from the json (db/core.ts:165-201) */
  fromJSON(json) {
    if (json.version !== 2 || !Array.isArray(json.token_table) || !Array.isArray(json.merge_codes))
      throw new Error('invalid format')
    let { char_count } = json
    this.reset()
    let code_to_id = {}
    let token_id = 0
    for (let [chars, weight, original_weight] of json.token_table) {
      token_id++
      let code = String.fromCodePoint(token_id)
      this.insert_token.run({ id: token_id, chars, weight, original_weight, code })
      if (token_id <= char_count) this.insert_char.run(token_id)
      code_to_id[code] = token_id
    }
    for (let [a_code, b_code, c_code] of json.merge_codes) {
      this.insert_merge.run({ a_id: code_to_id[a_code], b_id: code_to_id[b_code], c_id: code_to_id[c_code] })
    }
    let that = new BPETokenizerDB({ db: this.db })
    Object.assign(this, that)
    this._tokens = that._tokens
  }

  /** @description to enable adding more corpus without duplication (db/core.ts:204-206) */
  getLastCorpusId() {
    return this.select_last_corpus_id.get()
  }

  hasCorpus(id) {
    return this.has_corpus.get(id) > 0
  }

  // ---- the device engine ----------------------------------------------------------------------

  /** @description the HIP engine holding the corpus rows in id order (loaded on first use) */
  engine() {
    if (!this._engine) {
      let n = loadNative()
      this._engine = n.createEngine(0)
      this._registered = 0
      this.registerTokens()
      this._rows = []
      this._lens = []
      for (let row of this.select_corpus_rows.all()) {
        let ids = codeToIds(row.content_code)
        n.addSample(this._engine, ids)
        this._rows.push(row.id)
        this._lens.push(ids.length)
      }
    }
    this.registerTokens()
    return this._engine
  }

  dropEngine() {
    // (the context and its device memory go now, not when the garbage collector finds the handle)
    if (this._engine) loadNative().destroyEngine(this._engine)
    this._engine = null
    this._rows = []
    this._lens = []
  }

  /** @description tells the engine the UTF-16 length of every token it has not seen yet */
  registerTokens() {
    let n = loadNative()
    let tokens = this._tokens
    for (let id = this._registered + 1; id < tokens.length; id++) {
      if (tokens[id]) n.setTokenLen16(this._engine, id - 1, tokens[id].chars.length)
      this._registered = id
    }
  }

  /** @description a new corpus row: appended to the engine when it comes last in id order */
  engineAdd(id, content_code) {
    if (!this._engine) return
    let rows = this._rows
    if (rows.length && id <= rows[rows.length - 1]) {
      this.dropEngine() // reloaded in id order at the next merge
      return
    }
    let ids = codeToIds(content_code)
    this.registerTokens()
    loadNative().addSample(this._engine, ids)
    rows.push(id)
    this._lens.push(ids.length)
  }

  /**
   * @description writes back the corpus rows a rewrite changed: exactly those whose length fell
   * (db/core.ts:399-417 finds them with `like '%from_code%'` and `replaceAll`)
   */
  syncRows() {
    let n = loadNative()
    let lens = n.sampleLengths(this._engine)
    let changed = []
    for (let i = 0; i < lens.length; i++) if (lens[i] !== this._lens[i]) changed.push(i)
    if (changed.length === 0) return
    let [ids, off] = n.readSamples(this._engine, Float64Array.from(changed))
    for (let k = 0; k < changed.length; k++) {
      let i = changed[k]
      this.update_corpus.run({ id: this._rows[i], content_code: idsToCode(ids, off[k], off[k + 1]) })
      this._lens[i] = lens[i]
    }
  }

  invalidateVectorIndex() {
    this.to_vector_index = null
    this.from_vector_index = null
  }

  /**
   * @description add new content to corpus (db/core.ts:216-246).
   * Token weights are updated when adding content.
   */
  addToCorpus(id, content) {
    let { char_to_token, code_to_token } = this
    if (this.hasCorpus(id)) {
      throw new Error('corpus already added to database')
    }
    let content_code = ''
    let counts = new Map()
    for (let char of content) {
      let token = char_to_token[char]
      if (!token) {
        let new_id = this.count_token.get() + 1
        let code = String.fromCodePoint(new_id)
        this.insert_token.run({ id: new_id, chars: char, weight: 1, original_weight: 1, code })
        this.insert_char.run(new_id)
        token = this.tokenRow({ id: new_id, chars: char, weight: 1, original_weight: 1, code })
        char_to_token[char] = token
        code_to_token[code] = token
      } else {
        counts.set(token, (counts.get(token) || 0) + 1)
      }
      content_code += token.code
    }
    // the per-char increments of db/core.ts:240-241, one update per token
    for (let [token, k] of counts) {
      token.weight += k
      token.original_weight += k
    }
    this.insert_corpus.run({ id, content_code })
    this.engineAdd(id, content_code)
  }

  /**
   * @description restore content to corpus (after import tokens with fromJSON()) for continuous
   * merging (db/core.ts:252-256).  Token weights are not updated when restoring content.
   */
  restoreToCorpus(id, content) {
    let content_code = this.encodeToCode(content)
    let existed = this.hasCorpus(id)
    this.upsert_corpus.run({ id, content_code })
    if (existed) this.dropEngine()
    else this.engineAdd(id, content_code)
  }

  /**
   * @description skip zero-weight tokens to reduce range of vector index (db/core.ts:267-284).
   * Auto called by `encodeToVector()` and `decodeVector()`
   */
  compactVectorIndex() {
    let token_count = this.count_token.get()
    if (token_count == 0) {
      throw new Error(`token table is empty, have you called tokenizer.addToCorpus()?`)
    }
    let to_vector_index = (this.to_vector_index = [])
    let from_vector_index = (this.from_vector_index = [])
    let vector_index = 0
    for (let id of this.select_weighted_token.all()) {
      to_vector_index[id] = vector_index
      from_vector_index[vector_index] = id
      vector_index++
    }
  }

  /**
   * @description one pass over the corpus rows on the GPU (db/core.ts:290-369): the most frequent
   * adjacent pair under the reference's tie-break, or null.
   */
  findNextMerge(options) {
    let max_length = options && options.max_length
    let engine = this.engine()
    let found = loadNative().findNextMerge(engine, maxLengthArg(max_length), minWeightArg(options))
    if (!found) return null
    let [a_index, b_index, weight] = found
    let max_a = this._tokens[a_index + 1]
    let max_b = this._tokens[b_index + 1]
    let new_id = this.count_token.get() + 1
    let max_c = {
      chars: max_a.chars + max_b.chars,
      weight: weight,
      original_weight: weight,
      code: String.fromCodePoint(new_id),
      id: new_id,
    }
    return [max_a, max_b, max_c]
  }

  /** @description the table side of applyMerge (db/core.ts:379-397) */
  recordMerge(a, b, c) {
    if (!c.id) {
      throw new Error('missing id in token c')
    }
    let from_code = a.code + b.code
    let to_code = c.code
    a.weight -= c.weight
    b.weight -= c.weight
    this.invalidateVectorIndex()
    this.insert_token.run({
      id: c.id,
      chars: c.chars,
      weight: c.weight,
      original_weight: c.original_weight,
      code: c.code,
    })
    let row = this.tokenRow(c)
    this.code_to_token[row.code] = row
    this.insert_merge.run({ a_id: a.id, b_id: b.id, c_id: c.id })
    this.merge_codes.push([from_code, to_code])
    return row
  }

  /**
   * @description applies a merge to the tables, rewrites the corpus in HBM and writes back the
   * rows it changed (db/core.ts:375-418).
   */
  applyMerge(merge) {
    let [a, b, c] = merge
    this.recordMerge(a, b, c)
    let engine = this.engine()
    loadNative().applyMerge(engine, a.id - 1, b.id - 1, c.id - 1)
    this.syncRows()
  }

  /**
   * @description call `findNextMerge()` and `applyMerge()` in loop (db/core.ts:423-441), as the
   * device-resident loop; the tables and the changed rows are written once, at the end.
   */
  mergeUntil(options) {
    let max_iterations = options && options.max_iterations
    let it_arg = 0
    if (max_iterations && max_iterations !== Infinity) {
      if (!(max_iterations >= 1)) return
      it_arg = Math.floor(max_iterations)
    }
    let engine = this.engine()
    let max_length = options && options.max_length
    let abw = loadNative().mergeUntil(engine, maxLengthArg(max_length), minWeightArg(options), it_arg)
    let next_id = this.count_token.get() + 1
    for (let i = 0; i < abw.length; i += 3) {
      let a = this._tokens[abw[i] + 1]
      let b = this._tokens[abw[i + 1] + 1]
      let weight = abw[i + 2]
      let id = next_id++
      this.recordMerge(a, b, {
        chars: a.chars + b.chars,
        weight,
        original_weight: weight,
        code: String.fromCodePoint(id),
        id,
      })
    }
    // the engine registered the UTF-16 length of every token it created
    this._registered = this._tokens.length - 1
    if (abw.length) this.syncRows()
  }

  /**
   * @description encode to binary string (db/core.ts:450-467); with enough merges on the GPU's
   * merge-rank encoder, as in core.js.
   */
  encodeToCode(content) {
    let { char_to_token } = this
    let ids = []
    let content_in_code = ''
    for (let char of content) {
      let token = char_to_token[char]
      if (!token) {
        throw new Error('unknown token, char: ' + JSON.stringify(char))
      }
      ids.push(token.id - 1)
      content_in_code += token.code
    }
    let out = encodeIdsMaybeOnDevice(this, this.merge_codes, codeTriple, ids)
    if (out) return idsToCode(out, 0, out.length)
    for (let [from_code, to_code] of this.merge_codes) {
      content_in_code = content_in_code.split(from_code).join(to_code)
    }
    return content_in_code
  }

  /** db/core.ts:469-480 */
  encodeToTokens(content) {
    let { code_to_token } = this
    let content_in_code = this.encodeToCode(content)
    let tokens = []
    for (let code of content_in_code) {
      tokens.push(code_to_token[code])
    }
    return tokens
  }

  /** db/core.ts:482-503 */
  encodeToVector(content) {
    let { code_to_token, to_vector_index } = this
    if (!to_vector_index) {
      this.compactVectorIndex()
      to_vector_index = this.to_vector_index
    }
    let content_in_code = this.encodeToCode(content)
    let vector = []
    for (let code of content_in_code) {
      let id = code_to_token[code].id
      if (id in to_vector_index) {
        vector.push(to_vector_index[id])
      } else {
        throw new Error(`unknown token id: ${id}`)
      }
    }
    return vector
  }

  /** db/core.ts:505-511 */
  decodeTokens(tokens) {
    let content = ''
    for (let token of tokens) {
      content += token.chars
    }
    return content
  }

  /** db/core.ts:513-530 */
  decodeVector(vector) {
    let { from_vector_index } = this
    if (!from_vector_index) {
      this.compactVectorIndex()
      from_vector_index = this.from_vector_index
    }
    let content = ''
    for (let vector_index of vector) {
      if (vector_index in from_vector_index) {
        let id = from_vector_index[vector_index]
        content += this._tokens[id].chars
      } else {
        throw new Error(`unknown vector index: ${vector_index}`)
      }
    }
    return content
  }

  /**
   * @description restore merge produced from `compactMerge(BPETokenizer.findNextMerge())`
   * (db/core.ts:536-553).  To be used after restart for continuous merging.
   */
  restoreMerge(compactMerge) {
    let { code_to_token } = this
    let [a_code, b_code, c_weight] = compactMerge
    let a = code_to_token[a_code]
    if (!a) throw new Error(`unknown token, a_code: ${JSON.stringify(a_code)}`)
    let b = code_to_token[b_code]
    if (!b) throw new Error(`unknown token, b_code: ${JSON.stringify(b_code)}`)
    let new_id = this.count_token.get() + 1
    let c = {
      chars: a.chars + b.chars,
      weight: c_weight,
      original_weight: c_weight,
      code: String.fromCodePoint(new_id),
      id: new_id,
    }
    this.applyMerge([a, b, c])
  }
}

/** @description delete all tokens and corpus from database (db/core.ts:557-564) */
function resetBPETokenizerDB(db) {
  db.migrate({ migrations: [migrationSQL] })
  let proxy = createProxy({ db })
  proxy.char_token.length = 0
  proxy.merge.length = 0
  proxy.corpus.length = 0
  proxy.token.length = 0
}

/** @description db/core.ts:566-571 (needs @beenotung/better-sqlite3-helper, as the reference) */
function connectDB(path) {
  const DB = require('@beenotung/better-sqlite3-helper')
  return (DB.default || DB)({ path, migrate: false })
}

module.exports = {
  BPETokenizerDB,
  resetBPETokenizerDB,
  connectDB,
  createProxy,
  migrationSQL,
  EOF,
}
