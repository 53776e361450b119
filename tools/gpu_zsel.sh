#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-zsel}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/zipf_sel.py 1024 2000 2000 > "$OUT/incr.json" 2>&1 || { cat "$OUT/incr.json"; exit 1; }
cat "$OUT/incr.json"
BPE_SEL_FULL=1 timeout -k 10 200 python3 tools/zipf_sel.py 1024 2000 2000 > "$OUT/full.json" 2>&1 || { cat "$OUT/full.json"; exit 1; }
cat "$OUT/full.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/tr" -o run --output-format csv \
    -- python3 tools/zipf_sel.py 1024 2000 2000 > "$OUT/tr.log" 2>&1 || { tail "$OUT/tr.log"; exit 1; }
python3 tools/trace_gaps.py "$OUT/tr" "$OUT/gaps.json" > /dev/null
python3 - "$OUT" <<'PY'
import csv, sys, glob, collections
rows = []
for f in glob.glob(sys.argv[1] + '/tr/**/*kernel_trace.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_select_maint' in r['Kernel_Name']:
            rows.append((int(r['Start_Timestamp']), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
rows.sort()
d = [x for _, x in rows[-2000:]]
d.sort()
print('k_select_maint last 2000: median %.1f us, p10 %.1f, p90 %.1f, max %.1f' % (d[len(d)//2], d[len(d)//10], d[9*len(d)//10], d[-1]))
PY
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
