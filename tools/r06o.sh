# round-6: C3 2000 merges, HEAD against the Prep commit (is the gate's 1.7 % the gate alone?)
export TMPDIR=/tmp
AB_REPS=2 tools/ab_exp.sh r06o 2000 gpurun_exp/c_fdfcd1e.so gpurun_exp/head.so
