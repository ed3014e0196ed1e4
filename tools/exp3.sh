set -e
O=gpurun_out/exp3; mkdir -p $O
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 5 --iters 8 --unrolls 4 --nts 1 --grids 2048,4096,8192 --policies 1,2,3,4,5,6,7,8 > $O/p256.log 2>/dev/null
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 64 --rounds 6 --iters 20 --unrolls 4 --nts 1 --grids 2048,4096,8192 --policies 0,1,2,3,4,5,6,7,8 > $O/p64.log 2>/dev/null
timeout -k 10 200 python tools/sweep_reduce.py --k 2 --mib 256 --rounds 5 --iters 10 --unrolls 2,4 --nts 1 --grids 0,4096 --policies 0,1,3,5 > $O/k2.log 2>/dev/null
timeout -k 10 200 python tools/sweep_reduce.py --k 4 --mib 256 --rounds 5 --iters 10 --unrolls 2,4 --nts 1 --grids 0,4096 --policies 0,1,3,5 > $O/k4.log 2>/dev/null
