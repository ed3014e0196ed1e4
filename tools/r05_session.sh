export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ap
mkdir -p $O
bash tools/gpu_steps.sh $O "400 bash tools/bench_round.sh r05ap smoke n1 n2c4"
