export ESGD_TIMEOUT_S=60
O=gpurun_out/r05an
mkdir -p $O
bash tools/gpu_steps.sh $O "450 bash tools/bench_round.sh r05an profopt"
