# round-6: the maintained selection's tail (k_select_maint's last workgroup) with each thread's
# record and its block maxima in one batch of loads (sel1) against HEAD, zipf C3 (7995 merges);
# then the maintained-state parity tests on sel1 (the current tree)
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06u 7995 gpurun_exp/head.so gpurun_exp/sel1.so
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py "tests/test_scale_configs.py::test_zipf_2000_merges_vs_cpu_restatement" tests/test_sharded_gpu.py -k "maintained or zipf or parity or merges" > gpurun_out/r06u/tests.txt 2>&1
