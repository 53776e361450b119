# round-6: the Prep gated on the merge's weight (current tree) against the builds before it, on
# zipf C3 (7995 merges) and C3 (2000 merges); then the parity file on the current tree
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06n 7995 gpurun_exp/c_60afc15.so gpurun_exp/c_fdfcd1e.so bpe-tokenizer_amd/libbpe.so
AB_REPS=2 tools/ab_exp.sh r06n_c3 2000 gpurun_exp/c_fdfcd1e.so bpe-tokenizer_amd/libbpe.so
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/r06n/parity.txt 2>&1
