# Data-plane check on the GPU box: the multi-rank GPU tests, then the 2/4-rank rehearsals
# of the N>1 bench (ranks share the box's one GPU: HBM numbers, not xGMI).
export ESGD_TIMEOUT_S=60
O=gpurun_out/${1:-r2b}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_dataplane_gpu.py tests/test_caller_gpu.py tests/test_c_caller_gpu.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_dp.log 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc     # a hang / crash ends the session here
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510+n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_n$n.json 2> $O/bench_n$n.err || exit $?
done
exit $rc
