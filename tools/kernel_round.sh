# Local tree kernel session: its GPU tests, the window sweep, the N = 1 bench and its
# rocprofv3 kernel statistics.
set -e
O=gpurun_out/${1:-kernel}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_reduce_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_reduce.log 2>&1
for m in 128 256 1024; do
  timeout -k 10 300 python tools/sweep_reduce.py --k 8 --mib $m --grids 0 --unrolls 4 --nts 1 --policies=-1,21,22,23,24 --rounds 5 --iters 20 > $O/sweep_$m.jsonl 2>&1
done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-pmc --no-trace --no-cpu-baseline --steps 100 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2>&1
