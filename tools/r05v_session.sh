export ESGD_TIMEOUT_S=60
O=gpurun_out/r05v
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "500 python -u -m pytest tests/test_example_gpu.py tests/test_caller_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread -k 'example or backward or resnet'"
