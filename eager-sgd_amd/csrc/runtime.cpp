// runtime.cpp — device, memory, stream and event plumbing of the C ABI (esgd.h).
//
// fflib2 has no device layer at all (it reduces host buffers on a pthread,
// SURVEY.md §0.1); these entry points exist so that callers without PyTorch
// (the ff.h drop-in, the deep500 op, plain C tests) can drive the HIP path.
#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>

#include "esgd_internal.h"

namespace esgd {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = 0; }

// ESGD_TEST: "key=value,key=value" (see esgd_internal.h); read at each call -- the hooks
// that must stay fixed for the process keep their first value themselves
int64_t test_knob(const char *key, int64_t dflt) {
    const char *e = getenv("ESGD_TEST");
    if (!e || !*e) return dflt;
    const std::string spec(e);
    const size_t klen = std::strlen(key);
    size_t i = 0;
    while (i < spec.size()) {
        size_t j = spec.find(',', i);
        if (j == std::string::npos) j = spec.size();
        if (j - i > klen && spec.compare(i, klen, key) == 0 && spec[i + klen] == '=')
            return int64_t(strtoll(spec.c_str() + i + klen + 1, nullptr, 10));
        i = j + 1;
    }
    return dflt;
}

int hip_fail(hipError_t e, const char *what, const char *file, int line) {
    (void)hipGetLastError();   // reported here: not again by the thread's next launch check
    set_error("%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    if (e == hipErrorOutOfMemory) return ESGD_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice) return ESGD_NO_DEVICE;
    if (e == hipErrorInvalidValue) return ESGD_INVALID_ARG;
    return ESGD_ERROR;
}

// Every data call checks for a device first.  hipGetDeviceCount takes the runtime's lock and
// cost ~15 us a call under rocprofv3's HIP trace -- 4 300 calls in one 161-bucket bench leg,
// one per tree / pack launch (r05w) -- so a device once seen is remembered (devices do not
// go away under a running process); a missing one is asked about again each time.
static std::atomic<bool> g_device_seen{false};

int require_device() {
    if (g_device_seen.load(std::memory_order_relaxed)) return ESGD_SUCCESS;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        set_error("no HIP device available (hipGetDeviceCount: %s, n=%d)",
                  hipGetErrorString(e), n);
        return ESGD_NO_DEVICE;
    }
    g_device_seen.store(true, std::memory_order_relaxed);
    return ESGD_SUCCESS;
}

static std::mutex g_stream_mu;
static hipStream_t g_streams[64] = {};

hipStream_t default_stream() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if (!g_streams[dev]) {
        hipStream_t s = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess) g_streams[dev] = s;
    }
    return g_streams[dev];
}

}  // namespace esgd

using namespace esgd;

extern "C" {

const char *esgd_last_error(void) { return g_err; }

int esgd_version(void) { return 100; }

size_t esgd_dtype_size(int dtype) {
    switch (dtype) {
    case ESGD_INT32: return 4;
    case ESGD_INT64: return 8;
    case ESGD_DOUBLE: return 8;
    case ESGD_FLOAT: return 4;
    case ESGD_BF16: return 2;
    default: return 0;
    }
}

int esgd_device_count(int *n) {
    ESGD_ARG(n, "esgd_device_count: null pointer");
    hipError_t e = hipGetDeviceCount(n);
    if (e != hipSuccess) { *n = 0; }
    return ESGD_SUCCESS;
}

int esgd_set_device(int dev) { ESGD_HIP(hipSetDevice(dev)); return ESGD_SUCCESS; }

int esgd_get_device(int *dev) {
    ESGD_ARG(dev, "esgd_get_device: null pointer");
    ESGD_HIP(hipGetDevice(dev));
    return ESGD_SUCCESS;
}

int esgd_device_arch(int dev, char *name, size_t len) {
    ESGD_ARG(name && len > 0, "esgd_device_arch: bad buffer");
    if (int rc = require_device()) return rc;
    hipDeviceProp_t p;
    ESGD_HIP(hipGetDeviceProperties(&p, dev));
    snprintf(name, len, "%s", p.gcnArchName);
    return ESGD_SUCCESS;
}

// Buckets come from the IPC arena (arena.cpp): a freed bucket is recycled in this
// process, never handed back to the driver while peers may map it.
int esgd_malloc(void **ptr, size_t bytes) {
    ESGD_ARG(ptr, "esgd_malloc: null pointer");
    return arena_alloc(bytes ? bytes : 256, ptr, true);
}

// hipFree's contract is kept: the block is reused only after the work queued on its
// device so far has finished (a kernel still reading or writing it on any stream), so
// the device is synchronised before the block goes back to the free list.
int esgd_free(void *ptr) {
    if (!ptr) return ESGD_SUCCESS;
    const int dev = arena_device(ptr);
    if (dev < 0) {
        ESGD_HIP(hipFree(ptr));
        return ESGD_SUCCESS;
    }
    int cur = -1;
    ESGD_HIP(hipGetDevice(&cur));
    if (cur != dev) ESGD_HIP(hipSetDevice(dev));
    const hipError_t e = hipDeviceSynchronize();
    if (cur != dev) hip_ignore(hipSetDevice(cur));
    if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize (esgd_free)", __FILE__, __LINE__);
    arena_free(ptr);
    return ESGD_SUCCESS;
}

int esgd_memory_stats(uint64_t *reserved, uint64_t *in_use, uint64_t *exported) {
    arena_stats(reserved, in_use, exported);
    return ESGD_SUCCESS;
}

int esgd_host_alloc(void **ptr, size_t bytes) {
    ESGD_ARG(ptr, "esgd_host_alloc: null pointer");
    if (int rc = require_device()) return rc;
    ESGD_HIP(hipHostMalloc(ptr, bytes ? bytes : 256, hipHostMallocDefault));
    return ESGD_SUCCESS;
}

int esgd_host_free(void *ptr) {
    if (!ptr) return ESGD_SUCCESS;
    ESGD_HIP(hipHostFree(ptr));
    return ESGD_SUCCESS;
}

int esgd_host_register(void *ptr, size_t bytes) {
    ESGD_ARG(ptr && bytes, "esgd_host_register: bad range");
    if (int rc = require_device()) return rc;
    ESGD_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return ESGD_SUCCESS;
}

int esgd_host_unregister(void *ptr) {
    ESGD_ARG(ptr, "esgd_host_unregister: null pointer");
    ESGD_HIP(hipHostUnregister(ptr));
    return ESGD_SUCCESS;
}

int esgd_memcpy_async(void *dst, const void *src, size_t bytes, int kind, void *stream) {
    ESGD_ARG(kind >= 0 && kind <= 3, "esgd_memcpy_async: bad kind %d", kind);
    if (!bytes) return ESGD_SUCCESS;
    ESGD_ARG(dst && src, "esgd_memcpy_async: null pointer");
    static const hipMemcpyKind kinds[4] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost,
                                           hipMemcpyDeviceToDevice, hipMemcpyDefault};
    ESGD_HIP(hipMemcpyAsync(dst, src, bytes, kinds[kind], as_stream(stream)));
    return ESGD_SUCCESS;
}

int esgd_memset_async(void *dst, int value, size_t bytes, void *stream) {
    if (!bytes) return ESGD_SUCCESS;
    ESGD_ARG(dst, "esgd_memset_async: null pointer");
    ESGD_HIP(hipMemsetAsync(dst, value, bytes, as_stream(stream)));
    return ESGD_SUCCESS;
}

int esgd_stream_create(void **stream) {
    ESGD_ARG(stream, "esgd_stream_create: null pointer");
    if (int rc = require_device()) return rc;
    hipStream_t s;
    ESGD_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return ESGD_SUCCESS;
}

int esgd_stream_destroy(void *stream) {
    if (!stream) return ESGD_SUCCESS;
    ESGD_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
    return ESGD_SUCCESS;
}

int esgd_stream_synchronize(void *stream) {
    ESGD_HIP(hipStreamSynchronize(as_stream(stream)));
    return ESGD_SUCCESS;
}

int esgd_device_synchronize(void) {
    ESGD_HIP(hipDeviceSynchronize());
    return ESGD_SUCCESS;
}

int esgd_event_create(void **event) {
    ESGD_ARG(event, "esgd_event_create: null pointer");
    if (int rc = require_device()) return rc;
    hipEvent_t e;
    ESGD_HIP(hipEventCreate(&e));
    *event = e;
    return ESGD_SUCCESS;
}

int esgd_event_destroy(void *event) {
    if (!event) return ESGD_SUCCESS;
    ESGD_HIP(hipEventDestroy(static_cast<hipEvent_t>(event)));
    return ESGD_SUCCESS;
}

int esgd_event_record(void *event, void *stream) {
    ESGD_ARG(event, "esgd_event_record: null event");
    ESGD_HIP(hipEventRecord(static_cast<hipEvent_t>(event), as_stream(stream)));
    return ESGD_SUCCESS;
}

int esgd_event_synchronize(void *event) {
    ESGD_ARG(event, "esgd_event_synchronize: null event");
    ESGD_HIP(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    return ESGD_SUCCESS;
}

int esgd_event_elapsed_ms(void *start, void *stop, float *ms) {
    ESGD_ARG(start && stop && ms, "esgd_event_elapsed_ms: null argument");
    ESGD_HIP(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)));
    return ESGD_SUCCESS;
}

int esgd_stream_wait_event(void *stream, void *event) {
    ESGD_ARG(event, "esgd_stream_wait_event: null event");
    ESGD_HIP(hipStreamWaitEvent(as_stream(stream), static_cast<hipEvent_t>(event), 0));
    return ESGD_SUCCESS;
}

}  // extern "C"
