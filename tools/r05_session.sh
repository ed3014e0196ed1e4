export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ah
mkdir -p $O
bash tools/gpu_steps.sh $O "400 bash tools/bench_round.sh r05ah n2c4"
