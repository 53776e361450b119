# round-6 final measurements on the current build: the full C3 bench (+ incremental mode, encoder),
# the zipf bench, rocprofv3 kernel stats (C3, zipf), FETCH/WRITE over the full C3 run, SQ counters
export TMPDIR=/tmp
bash tools/gpu_run.sh r06m bench zipf prof profzipf sq || exit 1
PMC_STEPS=7995 bash tools/gpu_run.sh r06m pmc || exit 1
