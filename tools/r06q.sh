# round-6: scheduler strategies on the two passes' translation units.  zipf C3 (7995 merges) for
# the maintained-state pass (INCR_FLAGS), C3 (2000 merges) for the table pass (STEP_FLAGS + x)
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=1 tools/ab_exp.sh r06q 7995 gpurun_exp/c_60afc15.so gpurun_exp/i_r5.so gpurun_exp/i_r5trk.so gpurun_exp/i_r5mmc.so gpurun_exp/i_r5ilp.so gpurun_exp/i_trk.so
AB_REPS=2 tools/ab_exp.sh r06q_c3 2000 gpurun_exp/i_base.so gpurun_exp/s_trk.so gpurun_exp/s_mmc.so gpurun_exp/s_ilp.so gpurun_exp/s_iter.so
