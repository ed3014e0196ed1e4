# Per-round latency decomposition (tools/lat_probe.py) on the box's GPU.
#   bash tools/lat.sh OUT [kinds] [rank counts]
set -e
O=gpurun_out/${1:-lat}; mkdir -p $O
KINDS=${2:-allreduce}
NS=${3:-"1 2"}
export ESGD_TIMEOUT_S=30 ESGD_GPU_TRACE=1
export LAT_SIZES=${LAT_SIZES:-65536,1048576,67108864}
for k in $KINDS; do
  for n in $NS; do
    LAT_KIND=$k timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29540+n)) tools/lat_probe.py > $O/${k}_n$n.txt 2>&1
  done
done
