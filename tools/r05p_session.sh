export ESGD_TIMEOUT_S=60
O=gpurun_out/r05p
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "500 python -u -m pytest tests/test_caller_gpu.py tests/test_example_gpu.py tests/test_c_caller_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread" \
 "300 bash tools/bench_round.sh r05p n2c4" \
 "400 bash tools/bench_round.sh r05p n4c4"
