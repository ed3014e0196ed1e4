export ESGD_TIMEOUT_S=60
O=gpurun_out/r05l
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "900 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread" \
 "900 bash tools/bench_round.sh r05l n2 profopt"
