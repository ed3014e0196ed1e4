export ESGD_TIMEOUT_S=60
O=gpurun_out/r05aa
mkdir -p $O
bash tools/gpu_steps.sh $O "700 bash tools/bench_round.sh r05aa n2 n4c4"
