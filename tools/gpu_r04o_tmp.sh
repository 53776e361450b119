set -o pipefail
tools/gpu_run.sh r04o bench profpix || exit 1
timeout -k 10 400 python3 -u tools/pix_bench.py 2048 32507 --no-stream > gpurun_out/r04o/c5shard_pix.json 2> gpurun_out/r04o/c5shard_pix.err || { tail -5 gpurun_out/r04o/c5shard_pix.err; exit 1; }
tail -1 gpurun_out/r04o/c5shard_pix.json
