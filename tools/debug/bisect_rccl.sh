mkdir -p gpurun_out/r04n4
for grp in "tests/test_encoder.py" "tests/test_js_dropin.py" "tests/test_gpu_parity.py" "tests/test_incremental.py" "tests/test_capi.py"; do
  timeout -k 10 500 python3 -m pytest $grp tests/test_multi_device.py tests/test_sharded_gpu.py -m gpu -q -x \
     -k "not test_multi_device or rccl_one_device" --deselect tests/test_sharded_gpu.py > gpurun_out/r04n4/$(basename $grp .py).log 2>&1
  echo "$grp rc=$? $(tail -1 gpurun_out/r04n4/$(basename $grp .py).log)"
done
