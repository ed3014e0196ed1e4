export ESGD_TIMEOUT_S=60
O=gpurun_out/r05u
mkdir -p $O
E="python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29612 examples/resnet50_eager_sgd.py --mode allreduce --delay 0 --warmup 3"
bash tools/gpu_steps.sh $O \
 "240 $E --steps 30 --image 64 --batch 4 --overlap > $O/ex_small_overlap_grouped.json" \
 "240 $E --steps 30 --image 64 --batch 4 > $O/ex_small_after.json" \
 "300 $E --steps 20 > $O/ex_full_after.json" \
 "300 $E --steps 20 --overlap > $O/ex_full_overlap.json" \
 "300 $E --steps 20 --fuse > $O/ex_full_fused.json"
