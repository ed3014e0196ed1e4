# One GPU session: kernel sweep (with bit-exactness vs the production variant), the N=1
# bench (PMC traffic, gate shape, CPU baselines), 2/4-rank rehearsals of the N>1 path on
# the single GPU, and rocprofv3 kernel statistics of the bench.
set -e
export ESGD_TIMEOUT_S=60
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 256 --grids 0,512 --unrolls 4 --nts 1 --policies=${POLICIES:--1,17,18,19,20} --rounds 5 --iters 20 > $O/sweep_256.jsonl 2>&1
timeout -k 10 200 python tools/sweep_reduce.py --k 8 --mib 64 --grids 0 --unrolls 4 --nts 1 --policies=${POLICIES:--1,17,18,19,20} --rounds 5 --iters 40 > $O/sweep_64.jsonl 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510+n)) bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_n$n.json 2> $O/bench_n$n.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-pmc --no-trace --no-cpu-baseline --steps 100 > $GRAFT_REPO_ROOT/$O/bench_prof.json 2>&1
