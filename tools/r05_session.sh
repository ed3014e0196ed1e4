export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ab
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "400 python -u -m pytest tests/test_caller_gpu.py tests/test_example_gpu.py -x -v --timeout 170 --timeout-method thread" \
  "600 bash tools/bench_round.sh r05ab n2c4 n4c4"
