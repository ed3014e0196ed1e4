export ESGD_TIMEOUT_S=60
O=gpurun_out/r05d
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "500 python -u -m pytest tests/test_dataplane_gpu.py tests/test_c_caller_gpu.py -v --timeout 240 --timeout-method thread -k 'wrong_mapping or refused or c_caller or post_io or residency'" \
 "300 env ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161 ESGD_BENCH_RCCL=0 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_c4.json" \
 "300 env ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161 ESGD_BENCH_RCCL=0 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_n4_c4.json"
