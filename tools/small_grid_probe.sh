mkdir -p gpurun_out/sg
export LAT_KEEP=1 ESGD_TIMEOUT_S=30 LAT_SIZES=4194304,16777216,67108864 LAT_ITERS=40
for n in 2 4; do
  timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29571 tools/lat_probe.py > gpurun_out/sg/five_n$n.txt 2>&1 || exit 1
  for g in 64 256; do
    ESGD_SMALL_ROUND_BYTES=67108864 ESGD_SMALL_GRID=$g timeout -k 10 100 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29571 tools/lat_probe.py > gpurun_out/sg/one_g${g}_n$n.txt 2>&1 || exit 1
  done
done
