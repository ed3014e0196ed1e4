# Round-end validation on the GPU box: the whole -m gpu suite, smoke(), the N = 1 bench,
# the 2/4-rank rehearsals of the N > 1 bench, and rocprofv3 kernel statistics of the
# bench.  Each GPU step has its own time limit; the first failure ends the session.
set -e
export ESGD_TIMEOUT_S=60
O=gpurun_out/${1:-validate}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $O/pytest_gpu_full.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510+n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_n$n.json 2> $O/bench_n$n.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-pmc --no-trace --no-cpu-baseline --steps 100 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2>&1
