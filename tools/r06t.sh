# round-6: heavy merges (W * 16 >= chunks, screened) without the apply-time slots (h_heavy) against
# HEAD and c_60afc15, on zipf C3 (7995 merges) and C3 (2000 merges)
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06t 7995 gpurun_exp/c_60afc15.so gpurun_exp/head.so gpurun_exp/h_heavy.so
AB_REPS=2 tools/ab_exp.sh r06t_c3 2000 gpurun_exp/head.so gpurun_exp/h_heavy.so
