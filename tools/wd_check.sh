# bench.py N=2 twice: once with a 4 s budget for the extra legs (the watchdog must still
# print the headline line and exit 0), once in full.
O=gpurun_out/${1:-wd}; mkdir -p $O
ESGD_BENCH_EXTRAS_S=${WD_BUDGET:-4} timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 > $O/short.json 2> $O/short.err
echo "rc=$?" >> $O/short.json
[ -n "$WD_ONLY" ] || timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 20 --warmup 5 > $O/full.json 2> $O/full.err
