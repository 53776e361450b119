# round-6 check: the unscreened passes' parity tests, the ADVICE fixes' tests, then a 3-way A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/r06b
timeout -k 10 700 python3 -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_unscreened_passes_from_the_counts_bound \
  tests/test_gpu_parity.py::test_lds_counters_past_16_bits \
  tests/test_gpu_parity.py::test_small_golden_cases \
  tests/test_gpu_parity.py::test_random_vs_oracle \
  tests/test_gpu_parity.py::test_c3_dynamics_through_the_device_loop \
  tests/test_multi_device.py::test_automatic_switch_to_the_incremental_mode_and_its_fallback \
  tests/test_sharded_gpu.py::test_incremental_rank_loop_automatic_switch_and_fallback \
  tests/test_js_dropin.py > gpurun_out/r06b/pytest.log 2>&1
rc=$?
tail -12 gpurun_out/r06b/pytest.log
# (1: test failures, the A/B still runs; anything else: stop)
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_REPS=2 tools/ab_exp.sh r06b 2000 gpurun_exp/base.so bpe-tokenizer_amd/libbpe.so gpurun_exp/noscreen.so
