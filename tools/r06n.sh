# round-6: zipf C3 (7995 merges) across the round's builds: round 5, unscreened, Prep, current
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06n 7995 gpurun_exp/base.so gpurun_exp/c_60afc15.so gpurun_exp/c_fdfcd1e.so bpe-tokenizer_amd/libbpe.so
