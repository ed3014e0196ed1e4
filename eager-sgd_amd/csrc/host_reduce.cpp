// host_reduce.cpp — the local reduction on the reference's own contract: buckets that
// start and end in host memory (the wrapper's calloc'd buckets,
// T/utils/opt_esgd_solo_imagenet_imbalance.py:288-298; fflib2 sums them on the CPU,
// src/components/gcomp/ffop_gcomp_operator.c:33-58).
//
// Pinned, mapped buckets (the usual case: hipHostMalloc / hipHostRegister) are reduced in
// place: the tree kernel reads the k inputs and writes the output through their device
// views, over PCIe in both directions at once, no staging and no DMA commands.  Measured at
// C2's shape (8 x 64 MiB, profiles/r02/host_reduce_sweep.jsonl): 9.7-9.8 ms = 55 GB/s of
// buckets, 62 GB/s over the link, against 10.8 ms for H2D + tree + D2H in sequence and
// 10.5 ms for the chunked DMA pipeline below (16-32 MiB chunks; 1-4 MiB chunks are slower
// than the sequence: 17 / 13 / 11.5 ms, the per-copy cost).
// Other buckets (pageable memory) run in chunks through
// three process-wide streams so the PCIe link works in both directions at once:
//   copy stream 1: H2D of chunk c of every input into staging set c % kStages
//   compute stream: the tree kernel (esgd_reduce) of chunk c, staging -> staged output
//   copy stream 2: D2H of chunk c's output while chunks c+1, c+2 upload.
// A staging set is reused only after the kernel that read it (inputs) and the D2H that
// drained it (output) have finished; successive calls queue on the same streams, so the
// reuse order holds across calls too.  The result is the tree of esgd_reduce, element
// for element (the sum is element-wise: chunking cannot change a bit).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "esgd.h"
#include "esgd_internal.h"

namespace esgd {
namespace {

constexpr int kStages = 3;

struct HostReduce {
    std::mutex mu;
    int device = -1;
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    char *stage = nullptr;          // kStages x (kMaxFanin + 1) x chunk bytes
    size_t chunk = 0;               // bytes per input per chunk
    // per staging set: its inputs uploaded / reduced (inputs free again) / output drained
    hipEvent_t uploaded[kStages] = {}, reduced[kStages] = {}, out_free[kStages] = {};
    hipEvent_t start = nullptr, done = nullptr;
    uint64_t seq = 0;               // chunks issued so far (picks the staging set)
};

HostReduce g_hr;

// bytes per input per chunk of the DMA pipeline: 16 MiB (16-32 MiB chunks measured best,
// profiles/r02/host_reduce_sweep.jsonl)
constexpr size_t kChunkBytes = size_t(16) << 20;

// the device address of pinned, mapped host memory; nullptr otherwise
void *mapped(void *host) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}

int ensure(HostReduce &h) {
    int dev = 0;
    ESGD_HIP(hipGetDevice(&dev));
    if (h.stage && h.device == dev) return ESGD_SUCCESS;
    if (h.stage) {
        set_error("esgd_reduce_host: first used on device %d, now called on device %d", h.device, dev);
        return ESGD_INVALID_ARG;
    }
    // streams and events first (created once, kept on failure), the staging last: a
    // call that fails part way leaves nothing half-initialised behind `stage`
    for (hipStream_t *s : {&h.h2d, &h.comp, &h.d2h})
        if (!*s) ESGD_HIP(hipStreamCreateWithFlags(s, hipStreamNonBlocking));
    for (int i = 0; i < kStages; ++i)
        for (hipEvent_t *e : {&h.uploaded[i], &h.reduced[i], &h.out_free[i]})
            if (!*e) ESGD_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    for (hipEvent_t *e : {&h.start, &h.done})
        if (!*e) ESGD_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    h.chunk = kChunkBytes;
    ESGD_HIP(hipMalloc(reinterpret_cast<void **>(&h.stage), size_t(kStages) * (ESGD_MAX_FANIN + 1) * h.chunk));
    h.device = dev;
    return ESGD_SUCCESS;
}

}  // namespace

}  // namespace esgd

using namespace esgd;

extern "C" int esgd_reduce_host(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                                void *stream) {
    ESGD_ARG(k >= 1 && k <= ESGD_MAX_FANIN, "esgd_reduce_host: fan-in %d outside [1, %d]", k, ESGD_MAX_FANIN);
    ESGD_ARG(inputs && out, "esgd_reduce_host: null inputs/out");
    const int es = esgd_dtype_size(dtype);
    ESGD_ARG(es > 0, "esgd_reduce_host: unsupported dtype %d", dtype);
    for (int j = 0; j < k; ++j) ESGD_ARG(inputs[j], "esgd_reduce_host: input %d is null", j);
    if (count == 0) return ESGD_SUCCESS;
    if (int rc = require_device()) return rc;
    hipStream_t cs = stream == ESGD_STREAM_NULL ? nullptr : as_stream(stream);
    // pinned and mapped buckets: the tree kernel reads and writes them in place over
    // PCIe (zero-copy)
    {
        const void *view[ESGD_MAX_FANIN];
        void *oview = mapped(out);
        bool all = oview != nullptr;
        for (int j = 0; all && j < k; ++j) all = (view[j] = mapped(const_cast<void *>(inputs[j]))) != nullptr;
        if (all) return esgd_reduce(dtype, k, view, oview, count, cs);
    }
    HostReduce &h = g_hr;
    std::lock_guard<std::mutex> lk(h.mu);
    if (int rc = ensure(h)) return rc;
    // work the caller queued on `stream` before this call (e.g. writes of the host
    // buckets through a device view) comes first
    ESGD_HIP(hipEventRecord(h.start, cs));
    ESGD_HIP(hipStreamWaitEvent(h.h2d, h.start, 0));
    const uint64_t per = h.chunk / size_t(es);   // elements per input per chunk
    for (uint64_t o = 0; o < count; o += per) {
        const uint64_t n = std::min(per, count - o);
        const int st = int(h.seq++ % kStages);
        char *base = h.stage + size_t(st) * (ESGD_MAX_FANIN + 1) * h.chunk;
        const void *dev_in[ESGD_MAX_FANIN];
        // inputs of this staging set: free once the kernel that read them last finished
        ESGD_HIP(hipStreamWaitEvent(h.h2d, h.reduced[st], 0));
        for (int j = 0; j < k; ++j) {
            dev_in[j] = base + size_t(j) * h.chunk;
            ESGD_HIP(hipMemcpyAsync(const_cast<void *>(dev_in[j]), static_cast<const char *>(inputs[j]) + o * es,
                                    n * es, hipMemcpyHostToDevice, h.h2d));
        }
        ESGD_HIP(hipEventRecord(h.uploaded[st], h.h2d));
        char *dev_out = base + size_t(ESGD_MAX_FANIN) * h.chunk;
        ESGD_HIP(hipStreamWaitEvent(h.comp, h.uploaded[st], 0));
        ESGD_HIP(hipStreamWaitEvent(h.comp, h.out_free[st], 0));   // last D2H of this output drained
        if (int rc = esgd_reduce(dtype, k, dev_in, dev_out, n, h.comp)) return rc;
        ESGD_HIP(hipEventRecord(h.reduced[st], h.comp));
        ESGD_HIP(hipStreamWaitEvent(h.d2h, h.reduced[st], 0));
        ESGD_HIP(hipMemcpyAsync(static_cast<char *>(out) + o * es, dev_out, n * es, hipMemcpyDeviceToHost, h.d2h));
        ESGD_HIP(hipEventRecord(h.out_free[st], h.d2h));
    }
    // the caller's stream continues once the last D2H has landed
    ESGD_HIP(hipEventRecord(h.done, h.d2h));
    ESGD_HIP(hipStreamWaitEvent(cs, h.done, 0));
    return ESGD_SUCCESS;
}
