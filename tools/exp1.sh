set -e
O=gpurun_out/exp1; mkdir -p $O
for k in 1 2 4 8; do
  for st in 0 4352; do
    timeout -k 10 120 python tools/sweep_reduce.py --k $k --mib 64 --rounds 5 --iters 20 --unrolls 2,4,8 --nts 1 --grids 0,16384 --stagger $st >> $O/sweep.log 2>/dev/null
  done
done
timeout -k 10 120 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 4 --iters 10 --unrolls 4 --nts 1 --grids 0,16384,32768 --stagger 4352 >> $O/sweep.log 2>/dev/null
