set -e
O=gpurun_out/exp4; mkdir -p $O
for st in 0 256 4096 8192 65536 1052672 2162688 16777216; do
timeout -k 10 100 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 4 --iters 8 --unrolls 4 --nts 1 --grids 0,4096,8192 --stagger $st >> $O/st.log 2>/dev/null
done
timeout -k 10 100 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 6 --iters 8 --unrolls 2,4 --nts 1 --grids 1024,2048,3072,4096,6144,8192,16384 >> $O/grid.log 2>/dev/null
timeout -k 10 100 python tools/sweep_reduce.py --k 8 --mib 64 --rounds 6 --iters 20 --unrolls 2,4 --nts 1 --grids 1024,2048,3072,4096,6144,8192,16384 >> $O/grid64.log 2>/dev/null
