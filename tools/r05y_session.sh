export ESGD_TIMEOUT_S=60
O=gpurun_out/r05y
mkdir -p $O
L=ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161
B="python bench.py --steps 20 --warmup 5"
bash tools/gpu_steps.sh $O \
 "300 env $L ESGD_BENCH_RCCL=0 ESGD_SMALL_ROUND_BYTES=16777216 $B --gpus 2 > $O/n2_16mib_w64.json" \
 "300 env $L ESGD_BENCH_RCCL=0 ESGD_BATCH_WORKERS=256 $B --gpus 2 > $O/n2_4mib_w256.json" \
 "300 env $L ESGD_BENCH_RCCL=0 ESGD_SMALL_ROUND_BYTES=16777216 ESGD_BATCH_WORKERS=512 $B --gpus 2 > $O/n2_16mib_w512.json" \
 "300 env $L ESGD_BENCH_RCCL=0 ESGD_SMALL_ROUND_BYTES=16777216 ESGD_BATCH_WORKERS=256 $B --gpus 2 > $O/n2_16mib_w256_again.json" \
 "400 env $L ESGD_BENCH_RCCL=0 ESGD_SMALL_ROUND_BYTES=16777216 $B --gpus 4 > $O/n4_16mib_w64.json" \
 "400 env $L ESGD_BENCH_RCCL=0 ESGD_BATCH_WORKERS=256 $B --gpus 4 > $O/n4_4mib_w256.json"
