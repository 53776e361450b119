"""Test infrastructure: a sqlite3 database served over two FIFOs, one JSON request / reply per
line, for tests/js/sqlite_bridge.js.  Node 12 in this image has no sqlite binding, and the
reference's BPETokenizerDB (db/core.ts) needs one; Python's sqlite3 module is the real engine
behind the bridge.

Usage: sqlite_server.py DB_PATH REQUEST_FIFO REPLY_FIFO"""
import json
import sqlite3
import sys


def main():
    db_path, req_path, res_path = sys.argv[1:4]
    con = sqlite3.connect(db_path, isolation_level=None)   # transactions are explicit
    req = open(req_path, 'r', encoding='utf-8')
    res = open(res_path, 'w', encoding='utf-8')
    while True:
        line = req.readline()
        if not line:
            break
        m = json.loads(line)
        op = m['op']
        out = {'ok': True}
        try:
            if op == 'close':
                res.write(json.dumps(out) + '\n')
                res.flush()
                break
            if op == 'exec':
                # statement by statement: executescript would commit an open transaction
                for stmt in m['sql'].split(';'):
                    if stmt.strip():
                        con.execute(stmt)
            else:
                params = m.get('params')
                cur = con.execute(m['sql'], params if params is not None else ())
                if op == 'run':
                    out['changes'] = cur.rowcount
                    out['lastInsertRowid'] = cur.lastrowid
                else:
                    out['cols'] = [d[0] for d in cur.description] if cur.description else []
                    if op == 'get':
                        row = cur.fetchone()
                        out['rows'] = [list(row)] if row is not None else []
                    else:
                        out['rows'] = [list(r) for r in cur.fetchall()]
        except Exception as e:   # reported to the JS caller as a thrown Error
            out = {'ok': False, 'error': '%s: %s' % (type(e).__name__, e)}
        res.write(json.dumps(out) + '\n')
        res.flush()
    con.close()


if __name__ == '__main__':
    main()
