# round-6: MODE_INCR's cold adds out of line through the table's device copy (ctp2): parity of the
# maintained state and the incremental mode, then a zipf A/B against the current build
export TMPDIR=/tmp
mkdir -p gpurun_out/r06l
BPE_LIB=gpurun_exp/ctp2.so timeout -k 10 900 python3 -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "zipf or cold or only_cold or ties_of_cold" tests/test_incremental.py \
  tests/test_scale_configs.py::test_zipf_2000_merges_vs_cpu_restatement tests/test_sharded_gpu.py > gpurun_out/r06l/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r06l/pytest.log
[ $rc -eq 0 ] || exit $rc
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06l 3000 bpe-tokenizer_amd/libbpe.so gpurun_exp/ctp2.so
