set -eo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ic
timeout -s KILL 200 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH -d gpurun_out/ic/p1 -o run --output-format csv -- python3 tools/microbench.py 1024 256 10 1000 > gpurun_out/ic/p1.log 2>&1
python3 - <<'PY'
import csv, glob, collections
v = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob('gpurun_out/ic/p1/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        kn = r['Kernel_Name'].split('(')[0]
        if 'k_step' in kn:
            v[(kn, r['Counter_Name'])] += float(r['Counter_Value']); n[(kn, r['Counter_Name'])] += 1
for k in sorted(v): print(k, v[k] / n[k])
PY
