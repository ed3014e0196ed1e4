export ESGD_TIMEOUT_S=60
O=gpurun_out/r05k
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "600 bash tools/bench_round.sh r05k n1 prof"
