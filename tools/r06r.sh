# round-6: per-launch kernel trace of the zipf maintained state (2000 merges) for the selection
# kernels' duration distribution; and the guarded-Prep build (g_guard) against c_60afc15 on zipf
export TMPDIR=/tmp
mkdir -p gpurun_out/r06r
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06r/trace -o zipf -- python3 bench.py --corpus zipf --steps 2000 --no-cpu-baseline > gpurun_out/r06r/bench_trace.json
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06r 7995 gpurun_exp/c_60afc15.so gpurun_exp/g_guard.so
