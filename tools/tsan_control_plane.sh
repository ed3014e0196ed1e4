# ThreadSanitizer over the engine (progress thread, activation, issue ring, hold/release,
# delete-while-in-flight) through the multi-process CPU control-plane tests.  torch's
# gloo is not instrumented and reports races in its own destructors: only reports with a
# libesgd frame count.
set -e
cd "$(dirname "$0")/.."
make -j8 tsan > /dev/null
RT=/opt/rocm/lib/llvm/lib/clang/22/lib/linux/libclang_rt.tsan-x86_64.so
D=$(mktemp -d)
LD_PRELOAD=$RT ESGD_LIB=$PWD/build/tsan/libesgd.so TSAN_OPTIONS="report_signal_unsafe=0 log_path=$D/rep" \
    python -m pytest tests/test_control_plane.py -q -m "not gpu" 2>&1 | tail -1
n=$(cat $D/rep.* 2>/dev/null | grep -c "^WARNING: ThreadSanitizer" || true)
e=$(grep -l "esgd" $D/rep.* 2>/dev/null | wc -l)
echo "ThreadSanitizer: $n reports in total, $e with a libesgd frame"
[ "$e" -eq 0 ]
