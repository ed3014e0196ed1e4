export ESGD_TIMEOUT_S=60
O=gpurun_out/r05r
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "600 bash tools/bench_round.sh r05r n1 prof"
