// esgd_internal.h — shared helpers for libesgd.so (not installed).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "esgd.h"

namespace esgd {

// Per-thread message of the last failure; esgd_last_error() returns it.
void set_error(const char *fmt, ...);
void clear_error();

// Map a HIP status onto the ABI's codes, recording where it failed.
int hip_fail(hipError_t e, const char *what, const char *file, int line);

// A HIP call whose failure is tolerated (teardown, best-effort restores).  HIP keeps the
// thread's last error until hipGetLastError() reads it, and every kernel launch here is
// checked with hipGetLastError(): an ignored failure left in place would be reported by
// the thread's next, unrelated launch.  So a tolerated failure is cleared at once.
inline void hip_ignore(hipError_t e) {
    if (e != hipSuccess) (void)hipGetLastError();
}

// Lazily-created library stream for the current device (NULL stream argument).
hipStream_t default_stream();

// Fails with ESGD_NO_DEVICE (and a message) if no HIP device is usable.
int require_device();

// A stream argument of the ABI: NULL is the library's own stream, ESGD_STREAM_NULL the
// legacy default stream (stream 0, e.g. torch's default stream), anything else a stream.
inline hipStream_t as_stream(void *s) {
    if (s == ESGD_STREAM_NULL) return nullptr;
    return s ? static_cast<hipStream_t>(s) : default_stream();
}

// Device memory that peers may map (arena.cpp): never given back while it may be mapped.
// Where the flags of one rank pairing live (data plane -> round kernels).  A rank
// publishes a round by storing it at dst[0..ndst-1] and waits until mine[0..world-1] have
// all reached it.  Host flags (default): one shared array in the node segment, so dst is
// this rank's own word and mine the array.  Device flags (ESGD_DEVICE_FLAGS=1): every
// rank owns a page of uncached HBM holding one word per peer; dst is this rank's word in
// every rank's page (peers' pages mapped over IPC), mine this rank's own words.
constexpr int kPairMax = 16;   // = kMaxRanks
struct PairFlags {
    uint32_t *mine;
    uint32_t *dst[kPairMax];
    int ndst;
};

// ESGD_TEST (tests and diagnostics only; one variable for every fault hook): comma-separated
// key=value pairs, e.g. ESGD_TEST=fail_exports=2,piece_bytes=65536 (fail_connect is read
// at every creation, the others once per process)
//   fail_exports=N      the process's first N chunk exports are refused as the runtime does
//   fail_maps=N         its first N sealed mappings read back as another chunk's
//   fail_connect=R      rank R's connect fails (the creation vote fails on every rank)
//   arena_bypass=1|2    every bucket its own allocation (2: freed once peers closed their
//                       mappings) -- the ROCm IPC re-export probe
//   piece_bytes=B       remote launches in B-byte pieces (default 64 MiB)
//   shadow=1            every device bucket reduced through an arena shadow
//   host_chunk_bytes=B  host buckets of at least 2 x B bytes run chunked (default 16 MiB)
int64_t test_knob(const char *key, int64_t dflt);

// release_idle_chunks: a new chunk may first give idle never-exported chunks back to the
// driver (hipFree synchronises the device: callers' threads only, never the progress thread);
// fresh_chunk: the block comes from a chunk allocated now (never one a peer has opened)
int arena_alloc(size_t bytes, void **out, bool release_idle_chunks = false, bool fresh_chunk = false);
bool arena_free(void *p);
int arena_device(const void *p);   // device of an arena block, -1 if p is not one
bool arena_unexportable(const void *p);   // p's chunk: the runtime refused its IPC export
void arena_stats(uint64_t *reserved, uint64_t *live, uint64_t *exported);
// export p's chunk: its base, p's offset, the handle; seal (may be null): the chunk's
// usable bytes and seal nonce (ChunkSeal, below)
struct SealInfo {
    uint64_t chunk_bytes, chunk_base, nonce;
};
int arena_export(const void *p, size_t bytes, void **base, uint64_t *off, uint8_t handle[64],
                 SealInfo *seal = nullptr);
// The seal: 32 bytes written right behind an exported chunk's usable bytes before its
// first export.  Read back through a peer's fresh mapping, it proves the mapping shows
// the exporter's chunk (round 4: a suite's job came out wrong with the runtime mapping
// a peer's chunk to other memory).
struct ChunkSeal {
    uint64_t magic;
    uint64_t base;    // the exporter's VA of the chunk
    uint64_t nonce;
    uint32_t pid;
    uint32_t pad;
};
constexpr uint64_t kSealMagic = 0x4c41455344475345ull;   // "ESGDSEAL"
// written / read by kernels (reduce_kernels.hip), synchronously: 4 words
int seal_write(void *dst, const uint64_t w[4]);
int seal_read(const void *src, uint64_t w[4]);
// the stream they run on (dataplane.cpp)
int seal_stream(hipStream_t *out);
// diagnostics: "yes" while a seal read / write waits for the round stream, else nullptr
const char *seal_io_busy();
constexpr size_t kSealBytes = 4096;                      // allocated behind every chunk
void arena_trim();
// a multi-process job's first export: one chunk exported (or quarantined if refused)
// before its buckets are allocated
void arena_warm();
// deep500 group entry points (reduce_kernels.hip): copy-in of n tensors (/ divisor) into
// n buckets, copy-out of n buckets into n tensors -- one launch per 48
int pack_scatter(int n, const float *const *src, float *const *dst, const uint64_t *count, float divisor,
                 void *stream);
int unpack_gather(int n, float *const *dst, const float *const *src, const uint64_t *count, void *stream);

}  // namespace esgd

#define ESGD_HIP(call)                                                          \
    do {                                                                        \
        hipError_t esgd_e_ = (call);                                            \
        if (esgd_e_ != hipSuccess) return esgd::hip_fail(esgd_e_, #call, __FILE__, __LINE__); \
    } while (0)

#define ESGD_ARG(cond, ...)                                                     \
    do {                                                                        \
        if (!(cond)) { esgd::set_error(__VA_ARGS__); return ESGD_INVALID_ARG; } \
    } while (0)
