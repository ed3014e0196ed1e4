export ESGD_TIMEOUT_S=60
O=gpurun_out/r05j
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "600 python -u -m pytest tests/test_caller_gpu.py tests/test_example_gpu.py tests/test_dataplane_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k 'optimizer or op_group or post_io or example'" \
 "300 env ESGD_BENCH_LEGS=optimizer_resnet50_161,c4_resnet50_161_vs_fused ESGD_BENCH_RCCL=0 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_c4.json" \
 "400 env ESGD_BENCH_LEGS=optimizer_resnet50_161,c4_resnet50_161_vs_fused ESGD_BENCH_RCCL=0 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_n4_c4.json"
