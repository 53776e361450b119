# round-6: the host path's merge pass (k_step<MERGE_XY, MODE_TABLE>, engine TU) on the round-5 build,
# the unscreened build and the current one
export TMPDIR=/tmp
mkdir -p gpurun_out/r06i
for lib in gpurun_exp/base.so gpurun_exp/prep.so bpe-tokenizer_amd/libbpe.so gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so; do
  BPE_LIB=$lib timeout -k 10 300 python3 tools/microbench.py 1024 256 20 >> gpurun_out/r06i/mb.jsonl 2>> gpurun_out/r06i/mb.err || exit 1
done
cat gpurun_out/r06i/mb.jsonl
