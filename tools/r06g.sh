# round-6: slot 0 of each chunk loaded a stage ahead (BPE_EARLY_FIRST) against the current build
export TMPDIR=/tmp
mkdir -p gpurun_out/r06g
BPE_LIB=gpurun_exp/early.so timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "loop or host" > gpurun_out/r06g/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r06g/pytest.log
[ $rc -eq 0 ] || exit $rc
AB_REPS=2 tools/ab_exp.sh r06g 2000 bpe-tokenizer_amd/libbpe.so gpurun_exp/early.so
