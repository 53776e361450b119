# round-6: the incremental selection's grid (k_select_maint, BPE_SEL_GRID) on zipf C3 (7995 merges)
# (BPE_SEL_GRID was an A/B-only knob of that build, not kept: profiles/r06_ab_incr_codegen.txt)
export TMPDIR=/tmp
AB_EXTRA="--corpus zipf" AB_REPS=2 tools/ab_exp.sh r06s 7995 bpe-tokenizer_amd/libbpe.so:BPE_SEL_GRID=256 bpe-tokenizer_amd/libbpe.so:BPE_SEL_GRID=128 bpe-tokenizer_amd/libbpe.so:BPE_SEL_GRID=64 bpe-tokenizer_amd/libbpe.so:BPE_SEL_GRID=32 bpe-tokenizer_amd/libbpe.so:BPE_SEL_GRID=16
