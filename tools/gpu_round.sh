# One GPU session: parity tests, bench (with PMC traffic), rocprof kernel stats,
# and 2/4-rank rehearsals of the N>1 path on the single GPU.
set -e
export ESGD_TIMEOUT_S=60
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510+n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_n$n.json 2> $O/bench_n$n.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu-baseline --no-gate --steps 100 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2>&1
