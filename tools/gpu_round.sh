# One GPU session: parity tests, bench (with PMC traffic), rocprof kernel stats,
# and a 2-rank rehearsal of the N>1 path on the single GPU.
set -e
export ESGD_TIMEOUT_S=60
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2.json 2> $O/bench_n2.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu-baseline --no-gate --steps 100 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2>&1
