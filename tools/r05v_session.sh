export ESGD_TIMEOUT_S=60
O=gpurun_out/r05v
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
E="python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29613 examples/resnet50_eager_sgd.py --mode allreduce --delay 0 --warmup 3 --steps 20"
bash tools/gpu_steps.sh $O \
 "500 python -u -m pytest tests/test_example_gpu.py tests/test_caller_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread -k 'example or backward or resnet'" \
 "300 $E --fuse --overlap > $O/ex_full_fused_overlap25.json" \
 "300 $E --fuse > $O/ex_full_fused.json" \
 "300 $E --overlap > $O/ex_full_overlap.json" \
 "300 $E --fuse --overlap --bucket-mb 10 > $O/ex_full_fused_overlap10.json"
