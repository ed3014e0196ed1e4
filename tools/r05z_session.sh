export ESGD_TIMEOUT_S=60
O=gpurun_out/r05z
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread" \
 "300 bash tools/bench_round.sh r05z n2c4" \
 "400 bash tools/bench_round.sh r05z n4c4"
