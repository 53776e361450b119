# round-6: the full GPU suite, smoke and the driver's command on the current build, then a zipf A/B
# of the maintained-state pass: current / cold table through a device pointer (ctp) / no cold adds
# in the pass at all (noct: a timing build, wrong where the LDS hash overflows)
export TMPDIR=/tmp
bash tools/gpu_run.sh r06k tests smoke driver || exit 1
AB_EXTRA="--corpus zipf" AB_REPS=1 tools/ab_exp.sh r06k_zipf 2000 bpe-tokenizer_amd/libbpe.so gpurun_exp/ctp.so gpurun_exp/noct.so
