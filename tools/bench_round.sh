# One GPU session of bench work (round 3): the N = 1 line (PMC + kernel-trace passes), the
# N = 2 line started the way a bare `bench.py --gpus 2` starts it (self-launched ranks,
# sharing the box's one GPU: a rehearsal) and rocprofv3 kernel statistics of the N = 1 bench.  Each GPU step has its own time limit; the first
# failure ends the session.
#   bash tools/bench_round.sh <tag> [steps...]   steps: smoke n1 n2 n4 n2c4 n4c4 prof profopt sweep (default: n1 n2 prof)
set -e
export ESGD_TIMEOUT_S=60
O=gpurun_out/${1:-bench_round}; shift || true
STEPS=${*:-n1 n2 prof}
mkdir -p $O
R=$PWD
for s in $STEPS; do
  case $s in
  smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 ;;
  n1) timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
      cp -r gpurun_out/bench_kernel_trace_split.json $O/ 2>/dev/null || true ;;
  n2) timeout -k 10 600 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench_n2.json 2> $O/bench_n2.err ;;
  n4) timeout -k 10 600 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/bench_n4.json 2> $O/bench_n4.err ;;
  n2c4|n4c4) n=${s:1:1}   # the headline N > 1 line plus only the 161-bucket legs
      ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused,optimizer_resnet50_161 ESGD_BENCH_RCCL=0 timeout -k 10 300 python bench.py --gpus $n \
          --steps 20 --warmup 5 > $O/bench_n${n}_c4.json 2> $O/bench_n${n}_c4.err ;;
  prof) (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run \
          --output-format csv -- python $R/bench.py --no-pmc --no-trace --no-cpu-baseline --steps 100 \
          > $R/$O/bench_prof.json 2>&1) ;;
  profopt) (cd /tmp && export TMPDIR=/tmp && ESGD_BENCH_LEGS=optimizer_resnet50_161 ESGD_BENCH_RCCL=0 \
          timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/profopt -o run_%pid% --output-format csv \
          -- python $R/bench.py --gpus 2 --steps 20 --warmup 5 > $R/$O/bench_profopt_n2.json 2>&1) ;;
  sweep) test -f tools/bin/libesgd_sweeps.so   # built here by `make sweeps` (build() does it)
      for m in 64 256 1024; do
        timeout -k 10 240 python tools/sweep_reduce.py --mib $m --grids 0 --unrolls 4 --nts 1 \
            --policies=-1,25,26,27,28,29 --rounds 5 --iters 20 > $O/sweep_streams_$m.jsonl 2>&1
      done ;;
  esac
done
