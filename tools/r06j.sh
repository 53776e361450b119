# round-6: host-path table passes built in the step TU: parity of the host path, then its merge pass
export TMPDIR=/tmp
mkdir -p gpurun_out/r06j
timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "host" tests/test_sharded_gpu.py tests/test_capi.py > gpurun_out/r06j/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r06j/pytest.log
[ $rc -eq 0 ] || exit $rc
for lib in gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so; do
  BPE_LIB=$lib timeout -k 10 300 python3 tools/microbench.py 1024 256 20 >> gpurun_out/r06j/mb.jsonl 2>> gpurun_out/r06j/mb.err || exit 1
done
cat gpurun_out/r06j/mb.jsonl
