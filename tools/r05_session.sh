export ESGD_TIMEOUT_S=60
O=gpurun_out/r05am
mkdir -p $O
L="python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 examples/resnet50_eager_sgd.py --steps 20 --batch 64 --image 224 --warmup 3"
bash tools/gpu_steps.sh $O \
  "240 $L --mode majority > $O/majority_delay032_after.json" \
  "240 $L --mode majority --overlap > $O/majority_delay032_overlap.json" \
  "240 $L --mode solo --overlap > $O/solo_delay032_overlap.json"
