export ESGD_TIMEOUT_S=30
O=gpurun_out/r05c
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "500 python -u tools/mapping_probe.py $O/probe 3 > $O/probe.jsonl" \
 "300 env ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161 ESGD_BENCH_RCCL=0 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_c4.json" \
 "300 env ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161 ESGD_BENCH_RCCL=0 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_n4_c4.json"
