export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ac
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "300 ESGD_SNAPSHOT_WORKERS=256 python -u -m pytest tests/test_caller_gpu.py -x -v --timeout 170 --timeout-method thread" \
  "600 bash tools/bench_round.sh r05ac n2c4 n4c4"
