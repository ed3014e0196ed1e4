export ESGD_TIMEOUT_S=60
O=gpurun_out/r05af
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "400 ESGD_IDLE_SKIP=1 python -u -m pytest tests/test_caller_gpu.py tests/test_example_gpu.py tests/test_dataplane_gpu.py -x -v --timeout 170 --timeout-method thread -k 'caller or example or post_io or wait_on or release or consumer or producer'" \
  "600 bash tools/bench_round.sh r05af n2c4 n4c4"
