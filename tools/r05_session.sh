export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ad
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "800 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread" \
  "300 python -c 'import __graft_entry__ as g; g.smoke()'" \
  "400 bash tools/bench_round.sh r05ad n1 prof"
