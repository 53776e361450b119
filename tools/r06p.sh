# round-6: the maintained-state pass (k_step_loop<MODE_INCR>) in its own TU, by its flags
# (Makefile INCR_FLAGS), on zipf C3 (7995 merges); c_60afc15 = the round's best zipf build
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06p 7995 gpurun_exp/c_60afc15.so gpurun_exp/i_base.so gpurun_exp/i_pm.so gpurun_exp/i_r5.so gpurun_exp/i_r5pm.so gpurun_exp/i_r7.so
