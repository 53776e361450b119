# round-6: k_runs_reduce (the stitch folded into the reduce launch) parity, then A/B of the reduce's
# lane groups (8 / 16 / 32) and of the fused launch
export TMPDIR=/tmp
mkdir -p gpurun_out/r06f
BPE_LIB=gpurun_exp/fused.so timeout -k 10 600 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "loop" tests/test_scale_configs.py::test_config3_1000_merges_vs_cpu_restatement > gpurun_out/r06f/pytest.log 2>&1
rc=$?
tail -4 gpurun_out/r06f/pytest.log
[ $rc -eq 0 ] || exit $rc
AB_REPS=2 tools/ab_exp.sh r06f 2000 gpurun_exp/prep.so gpurun_exp/rg16.so gpurun_exp/rg32.so gpurun_exp/fused.so gpurun_exp/fused.so:BPE_RUNS_SEPARATE=1
