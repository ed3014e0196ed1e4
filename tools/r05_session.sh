export ESGD_TIMEOUT_S=60
O=gpurun_out/r05al
mkdir -p $O
L="python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 examples/resnet50_eager_sgd.py --mode allreduce --steps 20 --batch 64 --image 224 --delay 0 --warmup 3"
bash tools/gpu_steps.sh $O \
  "240 $L > $O/example_full_after.json" \
  "240 $L --overlap > $O/example_full_overlap.json" \
  "240 $L --fuse > $O/example_full_fused.json"
