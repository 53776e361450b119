'use strict'
/**
 * Test infrastructure: the subset of the better-sqlite3-helper API that BPETokenizerDB uses
 * (prepare -> all / get / run / pluck, transaction, migrate, exec, close), synchronous, over a
 * real sqlite3 database served by tests/js/sqlite_server.py through two FIFOs.  Node 12 in this
 * image has no sqlite binding of its own.
 */
const fs = require('fs')
const os = require('os')
const path = require('path')
const { spawn, execFileSync } = require('child_process')
const { StringDecoder } = require('string_decoder')

function connectDB(dbPath) {
  const dir = fs.mkdtempSync(path.join(os.tmpdir(), 'bpe-sqlite-'))
  const reqPath = path.join(dir, 'req')
  const resPath = path.join(dir, 'res')
  execFileSync('mkfifo', [reqPath, resPath])
  const child = spawn('python3', [path.join(__dirname, 'sqlite_server.py'), dbPath, reqPath, resPath], {
    stdio: ['ignore', 'inherit', 'inherit'],
  })
  child.unref()
  // the server opens the request FIFO first, then the reply FIFO: open them in the same order
  const reqFd = fs.openSync(reqPath, 'w')
  const resFd = fs.openSync(resPath, 'r')
  const decoder = new StringDecoder('utf8')
  const buf = Buffer.alloc(1 << 16)
  let pending = ''
  let closed = false

  function call(msg) {
    if (closed) throw new Error('The database connection is not open')
    fs.writeSync(reqFd, JSON.stringify(msg) + '\n')
    for (;;) {
      const i = pending.indexOf('\n')
      if (i >= 0) {
        const line = pending.slice(0, i)
        pending = pending.slice(i + 1)
        const out = JSON.parse(line)
        if (!out.ok) throw new Error(out.error)
        return out
      }
      const n = fs.readSync(resFd, buf, 0, buf.length, null)
      if (n === 0) throw new Error('sqlite server closed the connection')
      pending += decoder.write(buf.slice(0, n))
    }
  }

  function bindings(args) {
    if (args.length === 1 && args[0] !== null && typeof args[0] === 'object' && !Array.isArray(args[0]))
      return args[0]
    return args
  }

  function toRow(cols, r) {
    const o = {}
    cols.forEach((c, k) => (o[c] = r[k]))
    return o
  }

  let depth = 0
  const db = {
    prepare(sql) {
      let pluck = false
      const stmt = {
        pluck(on) {
          pluck = on !== false
          return stmt
        },
        all(...args) {
          const out = call({ op: 'all', sql, params: bindings(args) })
          return out.rows.map(r => (pluck ? r[0] : toRow(out.cols, r)))
        },
        get(...args) {
          const out = call({ op: 'get', sql, params: bindings(args) })
          if (!out.rows.length) return undefined
          return pluck ? out.rows[0][0] : toRow(out.cols, out.rows[0])
        },
        run(...args) {
          const out = call({ op: 'run', sql, params: bindings(args) })
          return { changes: out.changes, lastInsertRowid: out.lastInsertRowid }
        },
      }
      return stmt
    },
    exec(sql) {
      call({ op: 'exec', sql })
      return db
    },
    transaction(fn) {
      return function (...args) {
        if (depth === 0) call({ op: 'run', sql: 'begin' })
        depth++
        let result
        try {
          result = fn.apply(this, args)
        } catch (e) {
          depth--
          if (depth === 0) call({ op: 'run', sql: 'rollback' })
          throw e
        }
        depth--
        if (depth === 0) call({ op: 'run', sql: 'commit' })
        return result
      }
    },
    migrate(options) {
      for (const m of options.migrations) {
        const up = m.split('-- Down')[0].replace('-- Up', '')
        call({ op: 'exec', sql: up })
      }
    },
    close() {
      if (closed) return
      call({ op: 'close' })
      closed = true
      fs.closeSync(reqFd)
      fs.closeSync(resFd)
      fs.rmSync ? fs.rmSync(dir, { recursive: true, force: true }) : fs.rmdirSync(dir, { recursive: true })
    },
  }
  return db
}

module.exports = { connectDB }
