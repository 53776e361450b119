# round-6: the unscreened-pass test, then ring depth / load lead of the step TU on the unscreened build
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_unscreened_passes_from_the_counts_bound > gpurun_out/r06c/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r06c/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_REPS=2 tools/ab_exp.sh r06c 2000 bpe-tokenizer_amd/libbpe.so gpurun_exp/r6l3.so gpurun_exp/r7l3.so gpurun_exp/r6l2.so
