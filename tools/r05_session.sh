export ESGD_TIMEOUT_S=60
O=gpurun_out/r05aj
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "400 bash tools/bench_round.sh r05aj n2 n4c4" \
  "650 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread"
