# data plane after a protocol change: multi-rank GPU tests, then the N=4 rehearsal
set -e
O=gpurun_out/dpc; mkdir -p $O
export ESGD_TIMEOUT_S=30
timeout -k 10 500 python -m pytest tests/test_dataplane_gpu.py tests/test_caller_gpu.py tests/test_c_caller_gpu.py -x -q > $O/dp.txt 2>&1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 4 --steps 10 --warmup 3 > $O/bench_n4.json 2> $O/bench_n4.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29545 bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_n2.json 2> $O/bench_n2.err
