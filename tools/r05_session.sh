export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ao
mkdir -p $O
bash tools/gpu_steps.sh $O "500 bash tools/bench_round.sh r05ao n2c4 n4c4"
