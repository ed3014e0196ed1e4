export ESGD_TIMEOUT_S=60
O=gpurun_out/r05q
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60
bash tools/gpu_steps.sh $O \
 "300 python -u -m pytest tests/test_dataplane_gpu.py -m gpu -x -v --timeout 170 --timeout-method thread -k 'post_iov or post_io or wait_on'" \
 "300 bash tools/bench_round.sh r05q n2c4" \
 "400 bash tools/bench_round.sh r05q n4c4"
