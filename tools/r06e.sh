# round-6: the reduce's lane groups per block (8 / 16 / 32), on the Prep build
export TMPDIR=/tmp
mkdir -p gpurun_out/r06e
AB_REPS=2 tools/ab_exp.sh r06e 2000 gpurun_exp/prep.so gpurun_exp/rg16.so gpurun_exp/rg32.so || exit 1
for v in prep rg32; do
  BPE_LIB=gpurun_exp/$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06e/tr_$v -o run --output-format csv \
    -- python3 bench.py --steps 1000 --no-cpu-baseline > gpurun_out/r06e/tr_$v.jsonl 2> gpurun_out/r06e/tr_$v.err || exit 1
  find gpurun_out/r06e/tr_$v -name '*kernel_stats.csv' -exec head -8 {} \;
done
