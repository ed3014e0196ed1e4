# Rehearse the N>1 bench path with several ranks on the box's single GPU (timings
# are NOT xGMI numbers: all ranks share one device's HBM).
set -e
O=gpurun_out/$1; mkdir -p $O
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500+n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_n$n.json 2> $O/bench_n$n.err
done
