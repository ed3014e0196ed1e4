export ESGD_TIMEOUT_S=60
O=gpurun_out/r05g
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300 python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300 env ESGD_BENCH_LEGS=optimizer_resnet50_161,c4_resnet50_161_vs_fused ESGD_BENCH_RCCL=0 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2_c4.json"
