#!/bin/bash
# The one GPU-box driver script (run from the repo root on the box, e.g. through gpurun):
#   tools/gpu_run.sh TAG step [step ...]
# Every step runs under its own time limit; the script stops at the first failing step.
# Steps:
#   tests      pytest -m gpu (PYTEST_PATHS: test paths, PYTEST_K: a -k expression; default all)
#   smoke      __graft_entry__.smoke()
#   driver     the driver's exact bench command (bench.py --gpus 1 --steps 20 --warmup 5), timed
#   bench      full C3 bench line + the incremental mode's and the encoder's lines
#              (bench.py --incremental --encode)
#   zipf       full zipf C3 bench line (bench.py --corpus zipf)
#   prof       rocprofv3 --kernel-trace --stats of the full C3 bench (kernel stats CSV)
#   profzipf   the same for zipf C3
#   profpix    the same for the incremental mode (tools/pix_bench.py, full C3)
#   pmc        FETCH_SIZE and WRITE_SIZE passes (PMC_STEPS C3 merges, default 300; the bench's own
#              7995 give per-launch bytes comparable with its roofline), by tools/pmc_summary.py
#   sq         two SQ counter passes (300 C3 merges), summarised by tools/sq_loop_summary.py
#   probe      tools/probe/bin/stream_probe3 (loads in flight x VALU work per chunk)
#   rccl       the RCCL legs at world 1: tools/sharded_overhead.py (per-iteration cost)
#   encode     the device encoder: tools/encode_bench.py (uniform and zipf merges, 100k short
#              texts) and tools/encode_crossover.js (JS replay vs device per call)
#   enclat     tools/encode_latency.py (one text per call: wall and kernel time per call)
#   profenc    rocprofv3 --kernel-trace --stats of tools/encode_bench.py (zipf)
#   multi      8 shards of the C5 stream (512 MiB) on one device to the 32k vocabulary, the mode left
#              to the engine (auto: the stream, switching past 18 432 ids) then the incremental mode
#              (tools/multi_pix_probe.py; MULTI_MODES="stream ..." adds the stream kept by the caller)
#   profmulti  rocprofv3 --kernel-trace --stats of the streaming leg of `multi`
#   profmultipix  the same for the incremental leg
#   sqenc      SQ counter passes and FETCH_SIZE of the device encoder (tools/encode_bench.py, zipf
#              merges, 20 000 texts), summarised per k_encode launch (tools/sq_loop_summary.py),
#              under TAG/enc (apart from the sq / pmc steps' directories)
# Environment: BENCH_EXTRA (extra bench.py flags), PMC_CORPUS (uniform|zipf), PMC_STEPS, BPE_LIB (A/B builds)
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "step $1 failed"; tail -40 "$2"; exit 1; }
prof_stats() {  # $1 dir: print the top kernels of the stats CSV
  find "$1" -name '*kernel_stats.csv' -exec head -14 {} \;
}
PMC_BENCH="bench.py --steps ${PMC_STEPS:-300} --warmup 5 --no-cpu-baseline ${PMC_CORPUS:+--corpus $PMC_CORPUS}"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
  tests)
    # (a heartbeat under gpurun_out/ while a long test runs: pytest -v prints only at a test's end;
    # each test still has its own 400 s limit)
    ( while sleep 50; do date +%T >> "$OUT/heartbeat"; done ) & HB=$!
    # (RCCL's warnings to a file: a communicator that fails to come up leaves its reason there)
    export NCCL_DEBUG=${NCCL_DEBUG:-WARN} NCCL_DEBUG_FILE=${NCCL_DEBUG_FILE:-$PWD/$OUT/nccl.%p.log}
    timeout -k 10 1100 python3 -u -m pytest ${PYTEST_PATHS:-tests} ${PYTEST_K:+-k "$PYTEST_K"} -m gpu -v --durations=40 \
        --maxfail=5 --timeout 400 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
    rc=$?; kill $HB 2>/dev/null
    [ $rc -eq 0 ] || fail tests "$OUT/pytest_gpu.log"
    tail -3 "$OUT/pytest_gpu.log" ;;
  smoke)
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || fail smoke "$OUT/smoke.log"
    cat "$OUT/smoke.log" ;;
  driver)
    t0=$(date +%s.%N)
    timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/driver.jsonl" 2> "$OUT/driver.err" \
        || fail driver "$OUT/driver.err"
    t1=$(date +%s.%N)
    cat "$OUT/driver.jsonl"; python3 -c "print('driver wall: %.1f s' % ($t1 - $t0))" | tee "$OUT/driver.wall" ;;
  bench)
    timeout -k 10 700 python3 bench.py --incremental --encode $BENCH_EXTRA > "$OUT/bench.jsonl" 2> "$OUT/bench.err" \
        || fail bench "$OUT/bench.err"
    cat "$OUT/bench.jsonl" ;;
  zipf)
    timeout -k 10 600 python3 bench.py --corpus zipf --no-cpu-baseline $BENCH_EXTRA > "$OUT/zipf.jsonl" \
        2> "$OUT/zipf.err" || fail zipf "$OUT/zipf.err"
    head -c 1500 "$OUT/zipf.jsonl" ;;
  prof)
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline $BENCH_EXTRA > "$OUT/trace.jsonl" 2> "$OUT/trace.err" \
        || fail prof "$OUT/trace.err"
    head -c 600 "$OUT/trace.jsonl"; echo; prof_stats "$OUT/trace" ;;
  profzipf)
    timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/tracez" -o run --output-format csv \
        -- python3 bench.py --corpus zipf --no-cpu-baseline > "$OUT/tracez.jsonl" 2> "$OUT/tracez.err" \
        || fail profzipf "$OUT/tracez.err"
    head -c 600 "$OUT/tracez.jsonl"; echo; prof_stats "$OUT/tracez" ;;
  profpix)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pix" -o run --output-format csv \
        -- python3 tools/pix_bench.py 1024 7995 --no-stream > "$OUT/pix.json" 2> "$OUT/pix.err" \
        || fail profpix "$OUT/pix.err"
    cat "$OUT/pix.json"
    python3 tools/trace_gaps.py "$OUT/pix" "$OUT/gaps_pix.json" --from-kernel k_pix_select > /dev/null \
        || fail gaps "$OUT/pix.err" ;;
  pmc)
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
        -- python3 $PMC_BENCH > "$OUT/fetch.log" 2>&1 || fail fetch "$OUT/fetch.log"
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
        -- python3 $PMC_BENCH > "$OUT/write.log" 2>&1 || fail write "$OUT/write.log"
    python3 tools/pmc_summary.py "$OUT" "$OUT/pmc_summary.json" > /dev/null && echo "pmc summary written" ;;
  sq)
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        -d "$OUT/sq" -o run --output-format csv -- python3 $PMC_BENCH > "$OUT/sq.log" 2>&1 || fail sq "$OUT/sq.log"
    timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
        -d "$OUT/sq2" -o run --output-format csv -- python3 $PMC_BENCH > "$OUT/sq2.log" 2>&1 || fail sq2 "$OUT/sq2.log"
    python3 tools/sq_loop_summary.py "$OUT" > "$OUT/sq_summary.txt" && cat "$OUT/sq_summary.txt" ;;
  probe)
    timeout -k 10 300 tools/probe/bin/stream_probe3 > "$OUT/probe3.jsonl" 2>&1 || fail probe "$OUT/probe3.jsonl"
    cat "$OUT/probe3.jsonl" ;;
  rccl)
    for sz in "64 300" "1024 300"; do
      timeout -k 10 400 python3 -u tools/sharded_overhead.py $sz >> "$OUT/rccl_overhead.jsonl" 2>> "$OUT/rccl.err" \
          || fail rccl "$OUT/rccl.err"
    done
    cat "$OUT/rccl_overhead.jsonl" ;;
  encode)
    for c in uniform zipf; do
      timeout -k 10 300 python3 -u tools/encode_bench.py --corpus $c >> "$OUT/encode.jsonl" 2>> "$OUT/encode.err" \
          || fail encode "$OUT/encode.err"
    done
    cat "$OUT/encode.jsonl"
    timeout -k 10 300 node tools/encode_crossover.js > "$OUT/crossover.json" 2>> "$OUT/encode.err" \
        || fail crossover "$OUT/encode.err"
    cat "$OUT/crossover.json" ;;
  enclat)
    timeout -k 10 300 python3 -u tools/encode_latency.py > "$OUT/latency.json" 2> "$OUT/latency.err" \
        || fail enclat "$OUT/latency.err"
    cat "$OUT/latency.json" ;;
  profenc)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/enc" -o run --output-format csv \
        -- python3 tools/encode_bench.py --corpus zipf > "$OUT/enc.jsonl" 2> "$OUT/enc.err" \
        || fail profenc "$OUT/enc.err"
    cat "$OUT/enc.jsonl"; prof_stats "$OUT/enc" ;;
  multi)
    for mode in ${MULTI_MODES:-auto incremental}; do
      timeout -k 10 500 python3 -u tools/multi_pix_probe.py 512 8 32512 4096 $mode > "$OUT/multi8_$mode.jsonl" \
          2> "$OUT/multi8_$mode.err" || fail multi "$OUT/multi8_$mode.err"
      tail -2 "$OUT/multi8_$mode.jsonl"
    done ;;
  profmulti)
    BPE_MULTI_ONE_THREAD=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$OUT/multi" -o run --output-format csv \
        -- python3 tools/multi_pix_probe.py 512 8 32512 4096 auto > "$OUT/pmulti.jsonl" 2> "$OUT/pmulti.err" \
        || fail profmulti "$OUT/pmulti.err"
    tail -2 "$OUT/pmulti.jsonl"; prof_stats "$OUT/multi" ;;
  profmultipix)
    # (one enqueue thread: rocprofv3's kernel trace crashed in hipEventRecord with the
    # per-shard threads, gpurun_out/r05i; the kernels are the same)
    BPE_MULTI_ONE_THREAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/multipix" -o run --output-format csv \
        -- python3 tools/multi_pix_probe.py 512 8 32512 4096 incremental > "$OUT/pmultipix.jsonl" 2> "$OUT/pmultipix.err" \
        || fail profmultipix "$OUT/pmultipix.err"
    tail -2 "$OUT/pmultipix.jsonl"; prof_stats "$OUT/multipix"
    python3 tools/trace_gaps.py "$OUT/multipix" "$OUT/gaps_multipix.json" > /dev/null || true ;;
  sqenc)
    E="$OUT/enc"; mkdir -p "$E"
    ENC="tools/encode_bench.py --corpus zipf --texts 20000 --reps 1 --cpu-texts 20"
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
        -d "$E/sq" -o run --output-format csv -- python3 $ENC > "$E/sq.log" 2>&1 || fail sqenc "$E/sq.log"
    timeout -s KILL 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
        -d "$E/sq2" -o run --output-format csv -- python3 $ENC > "$E/sq2.log" 2>&1 || fail sqenc2 "$E/sq2.log"
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$E/fetch" -o run --output-format csv \
        -- python3 $ENC > "$E/fetch.log" 2>&1 || fail sqenc3 "$E/fetch.log"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$E/trace" -o run --output-format csv \
        -- python3 $ENC > "$E/trace.log" 2>&1 || fail sqenc4 "$E/trace.log"
    python3 tools/sq_loop_summary.py "$E" > "$E/sq_summary.txt" && grep -A30 k_encode "$E/sq_summary.txt" | head -80
    prof_stats "$E/trace" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
# keep the merged-back output small (the raw per-dispatch CSVs are tens of MB)
find "$OUT" \( -name "*kernel_trace.csv" -o -name "*counter_collection.csv" \) -delete
exit 0
