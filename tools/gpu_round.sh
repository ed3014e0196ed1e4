# One GPU session: parity tests, bench (with PMC traffic), rocprof kernel stats.
set -e
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 500 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu-baseline --steps 100 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2>&1
