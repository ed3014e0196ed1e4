export ESGD_TIMEOUT_S=60
O=gpurun_out/r05w
mkdir -p $O
R=$PWD
bash tools/gpu_steps.sh $O \
 "400 cd /tmp && export TMPDIR=/tmp && ESGD_BENCH_LEGS=c4_resnet50_161_vs_fused ESGD_BENCH_RCCL=0 rocprofv3 --hip-trace --stats -d $R/$O/hip -o run_%pid% --output-format csv -- python $R/bench.py --gpus 2 --steps 20 --warmup 5 > $R/$O/bench_n2_hiptrace.json 2> $R/$O/bench_n2_hiptrace.err"
