set -e
O=gpurun_out/exp5; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -q -x > $O/pytest.log 2>&1
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 64 --rounds 6 --iters 20 --unrolls 4 --nts 1 --grids 0 --policies=-1,9,10,11,12,13 > $O/p64.log 2>/dev/null
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 256 --rounds 5 --iters 8 --unrolls 4 --nts 1 --grids 0 --policies=-1,9,10,11,12,13 > $O/p256.log 2>/dev/null
bash tools/rehearse_n.sh reh2
