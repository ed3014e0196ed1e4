export ESGD_TIMEOUT_S=60
O=gpurun_out/r05b
bash tools/gpu_steps.sh $O \
 "600 python -u -m pytest tests/test_dataplane_gpu.py tests/test_caller_gpu.py -v --timeout 240 --timeout-method thread -k 'post_io or residency or finalize_with or refused or group_post or eager_sgd_optimizer or late_gradient or shadowed'" \
 "500 python -u -m pytest tests/test_dataplane_gpu.py -v --timeout 300 --timeout-method thread -k 'batched or pipelined_stress'"
