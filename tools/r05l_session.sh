export ESGD_TIMEOUT_S=60
O=gpurun_out/r05l
mkdir -p $O
bash tools/gpu_steps.sh $O \
 "1000 bash tools/bench_round.sh r05l n2 profopt"
