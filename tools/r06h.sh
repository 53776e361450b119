# round-6: where the pass's time goes: count-only pass (recount) vs merge pass, and the count-free
# ring (BPE_PROBE_NOCOUNT timing build: the ring, its loads and bookkeeping, no counting)
export TMPDIR=/tmp
mkdir -p gpurun_out/r06h
for lib in bpe-tokenizer_amd/libbpe.so gpurun_exp/nocount.so; do
  BPE_LIB=$lib timeout -k 10 300 python3 tools/microbench.py 1024 256 3 >> gpurun_out/r06h/mb.jsonl 2>> gpurun_out/r06h/mb.err || exit 1
done
cat gpurun_out/r06h/mb.jsonl
