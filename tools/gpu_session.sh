# One GPU session: the -m gpu suite (durations kept), then tools/bench_round.sh steps.
# Test FAILURES (pytest rc 1) do not stop the session; a fault, abort, segfault or a time
# limit (rc 124 / 134 / 137 / 139, or any other) does: nothing more runs on the GPU.
#   bash tools/gpu_session.sh <tag> [bench_round steps...]
T=${1:-session}; shift || true
O=gpurun_out/$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    --durations=60 -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/pytest_gpu.log
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $# -eq 0 ] && exit $rc
bash tools/bench_round.sh $T "$@"
