export ESGD_TIMEOUT_S=60
O=gpurun_out/r05x
mkdir -p $O
L=ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161
bash tools/gpu_steps.sh $O \
 "300 env $L ESGD_BENCH_RCCL=0 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2_default.json" \
 "300 env $L ESGD_BENCH_RCCL=0 ESGD_SMALL_ROUND_BYTES=16777216 ESGD_BATCH_WORKERS=256 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2_16mib_w256.json" \
 "400 env $L ESGD_BENCH_RCCL=0 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4_default.json" \
 "400 env $L ESGD_BENCH_RCCL=0 ESGD_SMALL_ROUND_BYTES=16777216 ESGD_BATCH_WORKERS=256 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4_16mib_w256.json"
