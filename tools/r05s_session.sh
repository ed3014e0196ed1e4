export ESGD_TIMEOUT_S=60
O=gpurun_out/r05s
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "300 python -u -m pytest tests/test_c_caller_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread" \
 "700 bash tools/bench_round.sh r05s n2 n4c4"
