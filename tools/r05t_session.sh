export ESGD_TIMEOUT_S=60
O=gpurun_out/r05t
mkdir -p $O
E="python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29611 examples/resnet50_eager_sgd.py --mode allreduce --delay 0 --steps 30 --warmup 3"
bash tools/gpu_steps.sh $O \
 "240 $E --image 64 --batch 4 > $O/ex_small_after.json" \
 "240 $E --image 64 --batch 4 --overlap > $O/ex_small_overlap.json" \
 "240 $E --image 64 --batch 4 --fuse > $O/ex_small_fused.json" \
 "300 $E --image 128 --batch 16 > $O/ex_mid_after.json" \
 "300 $E --image 128 --batch 16 --overlap > $O/ex_mid_overlap.json" \
 "300 $E --image 128 --batch 16 --fuse > $O/ex_mid_fused.json"
