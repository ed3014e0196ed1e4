export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ae
mkdir -p $O
bash tools/gpu_steps.sh $O "700 bash tools/bench_round.sh r05ae n2 n4c4"
