# The N > 1 bench with 2 and 4 ranks sharing the box's one GPU (HBM numbers, not xGMI).
# usage: tools/rehearse.sh TAG [extra env assignments are inherited]
export ESGD_TIMEOUT_S=60
O=gpurun_out/${1:-rehearse}; mkdir -p $O
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510+n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_n$n.json 2> $O/bench_n$n.err || exit $?
done
