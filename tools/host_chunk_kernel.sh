# C3 with 256 MiB HOST buckets per rank (chunked host rounds) at 2 ranks: DMA copies (0)
# vs kernel copies through the pinned buckets' device views with 16 / 32 / 64 workgroups
set -e
O=gpurun_out/${1:-hck}; mkdir -p $O
for kb in 0 16 32 64 0; do
  ESGD_HOST_CHUNK_KERNEL=$kb ESGD_BENCH_LEGS=c3_host_buckets timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 > $O/n2_kb$kb.json 2> $O/n2_kb$kb.err
  python -c "import json,sys; d=json.loads(open('$O/n2_kb$kb.json').read().strip().splitlines()[-1]); print($kb, json.dumps(d.get('c3_host_buckets')))" >> $O/summary.txt
done
