# esgd_reduce_host at the C2 shape: zero-copy (default for pinned buckets) vs chunked DMA
# at several chunk sizes; one JSON line per process (the env knobs are read once)
set -e
O=gpurun_out/${1:-hostred}; mkdir -p $O
timeout -k 10 120 python tools/host_reduce_sweep.py >> $O/sweep.jsonl
for c in 8 16 32; do
  ESGD_HOST_REDUCE_MODE=dma ESGD_HOST_REDUCE_CHUNK=$((c<<20)) timeout -k 10 120 python tools/host_reduce_sweep.py >> $O/sweep.jsonl
done
timeout -k 10 120 python tools/host_reduce_sweep.py >> $O/sweep.jsonl
