# Tree kernel (production policy) per-launch time vs bucket size, 8 inputs, one session.
set -e
O=gpurun_out/${1:-size_trend}; mkdir -p $O
for m in 16 32 64 128 256 512; do
  timeout -k 10 120 python tools/sweep_reduce.py --k 8 --mib $m --grids 0 --unrolls 4 --nts 1 --policies=-1 --rounds 5 --iters 20 > $O/sweep_$m.jsonl 2>&1
done
