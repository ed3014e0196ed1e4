set -e
O=gpurun_out/exp2; mkdir -p $O
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 4 --iters 8 --unrolls 2,4 --nts 1 --grids 0,4096,16384 --policies 0,1,2,3,4,5,6,7,8 --contigs 0 > $O/p256.log 2>/dev/null
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 4 --iters 8 --unrolls 2,4 --nts 1 --grids 512,1024,2048 --policies 1,4,5 --contigs 1 > $O/c256.log 2>/dev/null
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 64 --rounds 5 --iters 20 --unrolls 2,4 --nts 1 --grids 0,16384 --policies 0,1,2,3,4,5,6,7,8 --contigs 0 > $O/p64.log 2>/dev/null
