# Windowed launches (policies 21-23: slices of 32 / 64 / 96 MiB per bucket) vs one launch.
set -e
O=gpurun_out/${1:-window}; mkdir -p $O
for m in 64 128 256 1024; do
  timeout -k 10 300 python tools/sweep_reduce.py --k 8 --mib $m --grids 0 --unrolls 4 --nts 1 --policies=-1,21,22,23 --rounds 5 --iters 20 > $O/sweep_$m.jsonl 2>&1
done
