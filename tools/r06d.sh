# round-6: the apply-time pair slots (Prep) build: parity subset, A/B against the current build, full C3
export TMPDIR=/tmp
mkdir -p gpurun_out/r06d
BPE_LIB=gpurun_exp/prep.so timeout -k 10 900 python3 -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "not config2" > gpurun_out/r06d/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r06d/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
AB_REPS=2 tools/ab_exp.sh r06d 2000 bpe-tokenizer_amd/libbpe.so gpurun_exp/prep.so || exit 1
BPE_LIB=gpurun_exp/prep.so timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/r06d/full_prep.jsonl 2> gpurun_out/r06d/full_prep.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r06d/full_prep.jsonl').readline()); print('full C3 prep', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['fixture_check'], d['breakdown_ms_per_step'])"
