set -e
O=gpurun_out/lat; mkdir -p $O
export ESGD_TIMEOUT_S=30 ESGD_GPU_TRACE=1
export LAT_SIZES=65536,262144,1048576,67108864
ESGD_SHADOW=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29546 tools/lat_probe.py > $O/n2s.txt 2>&1
