export ESGD_TIMEOUT_S=60
O=gpurun_out/r05f
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "400 python -u -m pytest tests/test_caller_gpu.py tests/test_example_gpu.py -v --timeout 240 --timeout-method thread -k 'optimizer or resnet50 or group_post'" \
 "300 env ESGD_BENCH_LEGS=optimizer_resnet50_161,c4_resnet50_161_vs_fused ESGD_BENCH_RCCL=0 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_c4.json" \
 "300 env ESGD_BENCH_LEGS=optimizer_resnet50_161,c4_resnet50_161_vs_fused ESGD_BENCH_RCCL=0 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_n4_c4.json"
