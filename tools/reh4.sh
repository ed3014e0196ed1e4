# one-GPU rehearsal of the N>1 bench path (4 ranks share device 0; never N=8)
set -e
O=gpurun_out/reh4; mkdir -p $O
export ESGD_TIMEOUT_S=60
timeout -k 10 60 ./tools/bin/probe_ipc > $O/probe.txt 2>&1
timeout -k 10 400 python -m pytest tests/test_dataplane_gpu.py -x -q > $O/dp.txt 2>&1
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 4 --steps 10 --warmup 3 > $O/bench_n4.json 2> $O/bench_n4.err
