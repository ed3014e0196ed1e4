// reduce_kernels.hip — the gradient-bucket reduction entry points and the data plane's
// kernels, hand-written for gfx950.
//
// The tree-order reduction kernel itself (k_tree_sum_buf: k inputs folded in the
// hypercube order of fflib2's recursive doubling, src/colls/ffallreduce.c:138-171, one
// HBM pass) and its launch sizing live in reduce_core.h, shared with the tools-only sweep
// library (tools/sweeps/reduce_sweeps.hip).  This file holds what the product needs
// besides: the remote (peer-HBM) reduce-scatter / all-gather kernels, the bf16 wire, the
// fused snapshot, bucket packing, the rank-pairing kernels and the one-launch round.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <algorithm>
#include <type_traits>

#include "esgd_internal.h"
#include "reduce_core.h"

namespace esgd {

// ---- all-gather of peer shards (data plane phase 2) ----
// Copies up to kMaxSeg segments (one per peer shard) in one launch; blockIdx.y picks
// the segment.  Sources are peer memory mapped over xGMI: loads carry system scope
// (sc0 sc1) so no stale line of a previous round can be served from this device's L2;
// stores are local and write-through (sc1).
constexpr int kMaxSeg = 16;
struct GatherSet {
    const void *src[kMaxSeg];
    void *dst[kMaxSeg];
    uint32_t nvec[kMaxSeg];
    uint32_t tail[kMaxSeg];   // bytes after the last full 16-B vector
};

template <int U>
__global__ __launch_bounds__(256) void k_gather(GatherSet g) {
    constexpr int B = 256;
    const int seg = blockIdx.y;
    const uint32_t nvec = g.nvec[seg];
    const int bytes = int(nvec * 16u);
    if (nvec) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(g.src[seg]), (short)0,
                                                                     bytes, 0x00020000);
        __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(g.dst[seg], (short)0, bytes, 0x00020000);
        const uint32_t step = gridDim.x * (B * U);
        for (uint32_t i = blockIdx.x * (B * U) + threadIdx.x; i < nvec; i += step) {
            raw16 r[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                r[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (i + u * B) * 16, 0, 19);
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_amdgcn_raw_buffer_store_b128(r[u], ws, (i + u * B) * 16, 0, 16);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < g.tail[seg]) {
        const uint8_t *src = static_cast<const uint8_t *>(g.src[seg]) + size_t(nvec) * 16;
        uint8_t *dst = static_cast<uint8_t *>(g.dst[seg]) + size_t(nvec) * 16;
        dst[threadIdx.x] = __hip_atomic_load(src + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- bf16 on the wire for fp32 buckets (ESGD_SCHED_WIRE_BF16) ----
// The bucket stays fp32 in HBM; what peers read over xGMI is a bf16 copy of it (half the
// bytes in both phases).  Convention (an extension, parity unpinned by the reference, which
// has no bf16: F/src/ff.h:21-32): every rank's contribution is rounded to bf16 once (RNE),
// the shard is folded in fp32 in the hypercube tree order and rounded to bf16 once, and every
// rank widens that same bf16 result back to fp32 -- so all ranks hold identical values, the
// oracle's bf16 tree of the rounded inputs (oracle/ffref.c ffref_tree_sum_bf16).
// 4 elements per lane and access: 16 B of fp32 <-> 8 B of bf16, so that every load and
// store instruction of a wave covers one contiguous span (16-B bf16 / 2 x 16-B fp32 per
// lane left every fp32 store instruction half-filling its cache lines: the wire phases
// ran at half the HBM rate in the shared-GPU rehearsal).
using raw8 = __attribute__((ext_vector_type(2))) unsigned int;

__device__ __forceinline__ raw8 narrow4(raw16 a) {
    raw8 h;
    h[0] = uint32_t(BF16::store(__uint_as_float(a[0]))) | (uint32_t(BF16::store(__uint_as_float(a[1]))) << 16);
    h[1] = uint32_t(BF16::store(__uint_as_float(a[2]))) | (uint32_t(BF16::store(__uint_as_float(a[3]))) << 16);
    return h;
}

__device__ __forceinline__ raw16 widen4(raw8 h) {
    raw16 a;
    a[0] = h[0] << 16; a[1] = h[0] & 0xffff0000u;
    a[2] = h[1] << 16; a[3] = h[1] & 0xffff0000u;
    return a;
}

// wire = bf16(src): local HBM, 6 B per element moved (4 read + 2 written).  The snapshot
// of a wire round: src is the send bucket (or rb in place) -- rb itself is not written
// before phase 1, which overwrites all of it.  ZERO: the wrapper's zero-after-use of the
// send bucket fused in (ESGD_SCHED_ZERO_SB), 4 B more written per element.
template <bool ZERO>
__global__ __launch_bounds__(256) void k_narrow_bf16(float *src, uint16_t *dst, uint64_t n) {
    constexpr int U = 4;
    const uint64_t nq = n / 4;
    raw16 *s = reinterpret_cast<raw16 *>(src);
    raw8 *d = reinterpret_cast<raw8 *>(dst);
    const raw16 z = {0u, 0u, 0u, 0u};
    const uint64_t stride = uint64_t(gridDim.x) * 256 * U;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 * U + threadIdx.x; i < nq; i += stride) {
        raw16 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < nq) r[u] = __builtin_nontemporal_load(s + i + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < nq) {
                d[i + u * 256] = narrow4(r[u]);
                if constexpr (ZERO) __builtin_nontemporal_store(z, s + i + u * 256);
            }
    }
    if (blockIdx.x == 0 && nq * 4 + threadIdx.x < n) {
        dst[nq * 4 + threadIdx.x] = BF16::store(src[nq * 4 + threadIdx.x]);
        if constexpr (ZERO) src[nq * 4 + threadIdx.x] = 0.0f;
    }
}

// Phase 1 over the wire: the K ranks' bf16 copies of this rank's shard (peer HBM, system-
// scope nt loads), folded in fp32 in tree order, rounded once; the bf16 result goes to this
// rank's wire shard (what peers gather) and its widening to the fp32 bucket.  The own input
// is the same wire shard: each lane reads its element before it stores it.
template <int K>
__global__ __launch_bounds__(256) void k_tree_sum_wire(InputSet in, uint16_t *outb, float *outf, uint32_t nq,
                                                       uint64_t count) {
    constexpr int U = 4, B = 256;
    const int bytes = int(nq * 8u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(in.p[j]), (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t wb = __builtin_amdgcn_make_buffer_rsrc(outb, (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t wf = __builtin_amdgcn_make_buffer_rsrc(outf, (short)0, 2 * bytes, 0x00020000);
    const uint32_t step = gridDim.x * (B * U);
    for (uint32_t i = blockIdx.x * (B * U) + threadIdx.x; i < nq; i += step) {
        raw8 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j)
                r[u][j] = __builtin_amdgcn_raw_buffer_load_b64(rs[j], (i + u * B) * 8, 0, 19);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            uint32_t h[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v[K];
#pragma unroll
                for (int j = 0; j < K; ++j) v[j] = __uint_as_float((e & 1) ? (r[u][j][e / 2] & 0xffff0000u)
                                                                            : (r[u][j][e / 2] << 16));
                tree_fold<BF16, K>(v);
                h[e] = BF16::store(v[0]);
            }
            raw8 hb;
            hb[0] = h[0] | (h[1] << 16);
            hb[1] = h[2] | (h[3] << 16);
            __builtin_amdgcn_raw_buffer_store_b64(hb, wb, (i + u * B) * 8, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b128(widen4(hb), wf, (i + u * B) * 16, 0, 16);
        }
    }
    const uint64_t e = uint64_t(nq) * 4 + threadIdx.x;
    if (blockIdx.x == 0 && e < count) {
        float v[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            v[j] = BF16::load(__hip_atomic_load(static_cast<const uint16_t *>(in.p[j]) + e, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM));
        tree_fold<BF16, K>(v);
        const uint16_t h = BF16::store(v[0]);
        outb[e] = h;
        outf[e] = BF16::load(h);
    }
}

// Phase 2 over the wire: every other rank's reduced bf16 shard (peer HBM), widened into the
// fp32 bucket.  blockIdx.y picks the segment; n = elements.
struct WidenSet {
    const uint16_t *src[kMaxSeg];
    float *dst[kMaxSeg];
    uint32_t n[kMaxSeg];
};

__global__ __launch_bounds__(256) void k_gather_widen(WidenSet g) {
    constexpr int B = 256, U = 8;
    const int seg = blockIdx.y;
    const uint32_t n = g.n[seg], nq = n / 4;
    if (nq) {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint16_t *>(g.src[seg]), (short)0,
                                                                     int(nq * 8u), 0x00020000);
        __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(g.dst[seg], (short)0, int(nq * 16u),
                                                                     0x00020000);
        const uint32_t step = gridDim.x * (B * U);
        for (uint32_t i = blockIdx.x * (B * U) + threadIdx.x; i < nq; i += step) {
            raw8 r[U];
#pragma unroll
            for (int u = 0; u < U; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b64(rs, (i + u * B) * 8, 0, 19);
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_amdgcn_raw_buffer_store_b128(widen4(r[u]), ws, (i + u * B) * 16, 0, 16);
        }
    }
    const uint32_t e = nq * 4 + threadIdx.x;
    if (blockIdx.x == 0 && e < n)
        g.dst[seg][e] = BF16::load(__hip_atomic_load(g.src[seg] + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// ---- the snapshot with the zero-after-use fused: dst = src, src = 0 ----
// The round's move (colls/ffallreduce.c:126-130) and the wrapper's zeroing of the send
// bucket after the wait (opt_esgd_solo_imagenet_imbalance.py:311-314) in one pass:
// 1 read + 2 writes instead of 2 reads + 2 writes (+ a memset launch).
__global__ __launch_bounds__(256) void k_move_zero(raw16 *dst, raw16 *src, uint64_t nvec, uint8_t *dtail,
                                                    uint8_t *stail, uint32_t ntail) {
    const uint64_t stride = uint64_t(gridDim.x) * 256 * 4;
    const raw16 z = {0u, 0u, 0u, 0u};
    for (uint64_t i = uint64_t(blockIdx.x) * 1024 + threadIdx.x; i < nvec; i += stride) {
        raw16 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < nvec) r[u] = __builtin_nontemporal_load(src + i + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * 256 < nvec) {
                dst[i + u * 256] = r[u];
                __builtin_nontemporal_store(z, src + i + u * 256);
            }
    }
    if (blockIdx.x == 0 && threadIdx.x < ntail) {
        dtail[threadIdx.x] = stail[threadIdx.x];
        stail[threadIdx.x] = 0;
    }
}

// unaligned buckets: byte by byte (never on the bench path: rb is 16-B aligned and the
// op's own buckets are allocation-aligned)
__global__ __launch_bounds__(256) void k_move_zero_bytes(uint8_t *dst, uint8_t *src, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
        dst[i] = src[i];
        src[i] = 0;
    }
}

// ---- bucket packing (fused rounds of many gradient tensors) ----
// One launch moves up to kPackSeg tensors; block b handles kPackTile consecutive elements of
// the tensor whose tile range holds b.  Tensor offsets inside a fused bucket are arbitrary (no
// vector alignment): such a tile moves 4-B elements, 16 per lane in flight, coalesced per
// wave; a tile whose two sides are both 16-B aligned (the op's own buckets, torch tensors)
// moves 16-B vectors.  Round 4's tiles of 1024 elements made a fused ResNet-50 pack 25 000
// workgroups of 4 KB each, and per-workgroup overhead held it near 1 TB/s (r05c:
// 211 us for 2 x 102 MB); 16 Ki elements per tile is ~1 700 workgroups.
constexpr int kPackSeg = 48;
constexpr uint32_t kPackTile = 16384;
struct PackSet {
    float *a[kPackSeg];          // pack: sources; unpack: destinations
    float *b[kPackSeg];          // tensor i's place in the bucket (or its own bucket: scatter)
    uint64_t n[kPackSeg];
    uint32_t tile0[kPackSeg + 1];
    int nseg;
};

using vf4 = __attribute__((ext_vector_type(4))) float;   // one 16-B access

template <bool DIV>
__device__ __forceinline__ float pack_value(float x, float divisor) {
    return DIV ? __fdiv_rn(x, divisor) : x;
}

template <bool PACK, bool DIV>
__global__ __launch_bounds__(256) void k_pack(PackSet p, float divisor) {
    const uint32_t b = blockIdx.x;
    int i = 0;
    while (i + 1 < p.nseg && p.tile0[i + 1] <= b) ++i;
    const uint64_t e0 = uint64_t(b - p.tile0[i]) * kPackTile;
    const float *src = PACK ? p.a[i] : p.b[i];
    float *dst = PACK ? p.b[i] : p.a[i];
    const uint64_t end = p.n[i] < e0 + kPackTile ? p.n[i] : e0 + kPackTile;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0) {
        // 16-B vectors: the tile's start is a multiple of 4 elements; a ragged end by element
        const uint64_t vend = e0 + (end - e0) / 4 * 4;
        for (uint64_t base = e0 + uint64_t(threadIdx.x) * 4; base < vend; base += 256 * 4 * 4) {
            vf4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t e = base + uint64_t(u) * 1024;
                if (e < vend) v[u] = __builtin_nontemporal_load(reinterpret_cast<const vf4 *>(src + e));
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t e = base + uint64_t(u) * 1024;
                if (e < vend) {
                    vf4 w;
#pragma unroll
                    for (int c = 0; c < 4; ++c) w[c] = pack_value<DIV>(v[u][c], divisor);
                    *reinterpret_cast<vf4 *>(dst + e) = w;
                }
            }
        }
        if (threadIdx.x < end - vend) dst[vend + threadIdx.x] = pack_value<DIV>(src[vend + threadIdx.x], divisor);
        return;
    }
    for (uint64_t base = e0 + threadIdx.x; base < end; base += 256 * 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint64_t e = base + uint64_t(u) * 256;
            if (e < end) v[u] = __builtin_nontemporal_load(src + e);
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint64_t e = base + uint64_t(u) * 256;
            if (e < end) dst[e] = pack_value<DIV>(v[u], divisor);
        }
    }
}

// ---- synthetic inputs (same generator as oracle/ffref.c) ----
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ float uniform_pm1(uint64_t base, uint64_t i) {
    const float u = float(splitmix64(base ^ i) >> 40) * (1.0f / 16777216.0f);
    return __fsub_rn(__fmul_rn(2.0f, u), 1.0f);
}

__global__ void k_fill_uniform_f32(uint64_t base, float *out, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = uniform_pm1(base, i);
}

__global__ void k_fill_uniform_bf16(uint64_t base, uint16_t *out, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = BF16::store(uniform_pm1(base, i));
}

template <class Tr, int K, bool SCALE>
static int dispatch_u(const InputSet &in, void *out, uint64_t count, float scale, bool aligned,
                      hipStream_t s, bool remote = false) {
    // bf16 folds 8 lanes per 16 B: two vectors per input keep it under 128 VGPRs
    constexpr int UD = sizeof(typename Tr::T) == 2 ? 2 : 4;
    if (remote) {
        // inputs live in peer HBM (IPC over xGMI): system-scope nt loads, local sc1 stores
        const bool fits32 = count / Tr::E * 16 + uint64_t(UD) * 256 * 16 < (1ull << 31);
        if (!aligned || !fits32) {
            set_error("remote reduce: shard must be 16-B aligned and < 2 GiB");
            return ESGD_INVALID_ARG;
        }
        return launch_buf<Tr, K, UD, 19, 16, SCALE>(in, out, count, scale, s);
    }
    if (!aligned) return launch_scalar<Tr, K, SCALE>(in, out, count, scale, s);
    // nt loads + sc1 stores, any size windowed into the buffer kernel
    return launch_windows<Tr, K, UD, 2, 16, SCALE>(in, out, count, scale, s);
}


template <class Tr, bool SCALE>
static int dispatch_k(int k, const InputSet &in, void *out, uint64_t count, float scale,
                      bool aligned, hipStream_t s, bool remote = false) {
    switch (k) {
    case 1: return dispatch_u<Tr, 1, SCALE>(in, out, count, scale, aligned, s, remote);
    case 2: return dispatch_u<Tr, 2, SCALE>(in, out, count, scale, aligned, s, remote);
    case 3: return dispatch_u<Tr, 3, SCALE>(in, out, count, scale, aligned, s, remote);
    case 4: return dispatch_u<Tr, 4, SCALE>(in, out, count, scale, aligned, s, remote);
    case 5: return dispatch_u<Tr, 5, SCALE>(in, out, count, scale, aligned, s, remote);
    case 6: return dispatch_u<Tr, 6, SCALE>(in, out, count, scale, aligned, s, remote);
    case 7: return dispatch_u<Tr, 7, SCALE>(in, out, count, scale, aligned, s, remote);
    case 8: return dispatch_u<Tr, 8, SCALE>(in, out, count, scale, aligned, s, remote);
    default: break;
    }
    set_error("esgd_reduce: fan-in %d outside [1, %d]", k, ESGD_MAX_FANIN);
    return ESGD_INVALID_ARG;
}

static int reduce_impl(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                       float scale, bool scaled, void *stream, bool remote = false) {
    ESGD_ARG(k >= 1 && k <= ESGD_MAX_FANIN, "esgd_reduce: fan-in %d outside [1, %d]", k,
             ESGD_MAX_FANIN);
    ESGD_ARG(inputs && out, "esgd_reduce: null inputs/out");
    if (count == 0) return ESGD_SUCCESS;
    if (int rc = require_device()) return rc;
    InputSet in;
    std::memset(&in, 0, sizeof(in));
    bool aligned = (reinterpret_cast<uintptr_t>(out) & 15) == 0;
    for (int j = 0; j < k; ++j) {
        ESGD_ARG(inputs[j], "esgd_reduce: input %d is null", j);
        in.p[j] = inputs[j];
        aligned = aligned && (reinterpret_cast<uintptr_t>(inputs[j]) & 15) == 0;
    }
    hipStream_t s = as_stream(stream);
    switch (dtype) {
    case ESGD_FLOAT:
        return scaled ? dispatch_k<F32, true>(k, in, out, count, scale, aligned, s, remote)
                      : dispatch_k<F32, false>(k, in, out, count, scale, aligned, s, remote);
    case ESGD_BF16:
        return scaled ? dispatch_k<BF16, true>(k, in, out, count, scale, aligned, s, remote)
                      : dispatch_k<BF16, false>(k, in, out, count, scale, aligned, s, remote);
    case ESGD_DOUBLE:
        ESGD_ARG(!scaled, "esgd_reduce_scaled: FLOAT/BF16 only");
        return dispatch_k<F64, false>(k, in, out, count, scale, aligned, s, remote);
    case ESGD_INT32:
        ESGD_ARG(!scaled, "esgd_reduce_scaled: FLOAT/BF16 only");
        return dispatch_k<I32, false>(k, in, out, count, scale, aligned, s, remote);
    case ESGD_INT64:
        ESGD_ARG(!scaled, "esgd_reduce_scaled: FLOAT/BF16 only");
        return dispatch_k<I64, false>(k, in, out, count, scale, aligned, s, remote);
    default: break;
    }
    set_error("esgd_reduce: unsupported dtype %d", dtype);
    return ESGD_INVALID_ARG;
}

// A round's completion word, stored by the GPU once everything queued before it on the
// stream is done (copy-outs included): the host polls it instead of an event, whose
// completion reaches the host several microseconds later.
__global__ void __launch_bounds__(64) k_store_fin(uint32_t *fin, uint32_t value) {
    if (threadIdx.x == 0) __hip_atomic_store(fin, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- internal entry points of the data plane (dataplane.cpp) ----
int store_fin(uint32_t *fin, uint32_t value, hipStream_t s) {
    hipLaunchKernelGGL(k_store_fin, dim3(1), dim3(64), 0, s, fin, value);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

int move_zero(void *dst, void *src, uint64_t bytes, hipStream_t s) {
    if (!bytes) return ESGD_SUCCESS;
    if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) == 0) {
        const uint64_t nvec = bytes / 16;
        const uint32_t ntail = uint32_t(bytes % 16);
        const unsigned grid = grid_for(1024, nvec ? nvec : 1, 4);
        hipLaunchKernelGGL(k_move_zero, dim3(grid), dim3(256), 0, s, static_cast<raw16 *>(dst),
                           static_cast<raw16 *>(src), nvec, static_cast<uint8_t *>(dst) + nvec * 16,
                           static_cast<uint8_t *>(src) + nvec * 16, ntail);
    } else {
        hipLaunchKernelGGL(k_move_zero_bytes, dim3(grid_for(256, bytes, 4)), dim3(256), 0, s,
                           static_cast<uint8_t *>(dst), static_cast<uint8_t *>(src), bytes);
    }
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// pack: tensors[i] (/ divisor) -> buckets[i]; unpack: buckets[i] -> tensors[i].  One
// launch per kPackSeg tensors.  `bucket` != nullptr: buckets[i] are consecutive places in
// that one bucket (esgd_pack_div / esgd_unpack); else `buckets` names each tensor's own.
static int pack_impl(bool pack, int n, float *const *tensors, const uint64_t *count, float *bucket,
                     float divisor, void *stream, float *const *buckets = nullptr) {
    ESGD_ARG(n >= 0 && n <= 4096, "esgd_pack: %d tensors outside [0, 4096]", n);
    ESGD_ARG(n == 0 || (tensors && count && (bucket || buckets)), "esgd_pack: null argument");
    ESGD_ARG(divisor == divisor && divisor != 0.0f, "esgd_pack: divisor must be a non-zero number");
    if (n == 0) return ESGD_SUCCESS;
    if (int rc = require_device()) return rc;
    hipStream_t s = as_stream(stream);
    uint64_t off = 0;
    for (int i0 = 0; i0 < n; i0 += kPackSeg) {
        PackSet p;
        std::memset(&p, 0, sizeof(p));
        p.nseg = std::min(kPackSeg, n - i0);
        uint64_t tiles = 0;
        for (int j = 0; j < p.nseg; ++j) {
            const uint64_t c = count[i0 + j];
            ESGD_ARG(c == 0 || tensors[i0 + j], "esgd_pack: tensor %d is null", i0 + j);
            p.a[j] = tensors[i0 + j];
            p.b[j] = bucket ? bucket + off : buckets[i0 + j];
            ESGD_ARG(c == 0 || p.b[j], "esgd_pack: bucket %d is null", i0 + j);
            p.n[j] = c;
            p.tile0[j] = uint32_t(tiles);
            tiles += (c + kPackTile - 1) / kPackTile;
            off += c;
        }
        ESGD_ARG(tiles < (1ull << 31), "esgd_pack: too many elements in one launch");
        p.tile0[p.nseg] = uint32_t(tiles);
        if (!tiles) continue;
        if (pack) {
            if (divisor == 1.0f) hipLaunchKernelGGL((k_pack<true, false>), dim3(unsigned(tiles)), dim3(256), 0, s, p, divisor);
            else hipLaunchKernelGGL((k_pack<true, true>), dim3(unsigned(tiles)), dim3(256), 0, s, p, divisor);
        } else {
            hipLaunchKernelGGL((k_pack<false, false>), dim3(unsigned(tiles)), dim3(256), 0, s, p, divisor);
        }
        ESGD_HIP(hipGetLastError());
    }
    return ESGD_SUCCESS;
}
// the deep500 op's group entry points: every op's copy-in (/ divisor) into its own send
// bucket, or every op's copy-out from its own receive bucket, in one launch per 48 ops
int pack_scatter(int n, const float *const *src, float *const *dst, const uint64_t *count, float divisor,
                 void *stream) {
    return pack_impl(true, n, const_cast<float *const *>(src), count, nullptr, divisor, stream, dst);
}

int unpack_gather(int n, float *const *dst, const float *const *src, const uint64_t *count, void *stream) {
    return pack_impl(false, n, dst, count, nullptr, 1.0f, stream, const_cast<float *const *>(src));
}

int reduce_remote(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                  float scale, hipStream_t s) {
    return reduce_impl(dtype, k, inputs, out, count, scale, scale != 1.0f, s, true);
}

int gather_remote(int n, const void *const *src, void *const *dst, const uint64_t *bytes,
                  hipStream_t s, unsigned max_blocks) {
    ESGD_ARG(n >= 0 && n <= kMaxSeg, "gather: %d segments", n);
    if (n == 0) return ESGD_SUCCESS;
    GatherSet g;
    std::memset(&g, 0, sizeof(g));
    uint64_t maxvec = 0;
    for (int i = 0; i < n; ++i) {
        ESGD_ARG(bytes[i] / 16 < (1ull << 27), "gather: segment of %llu bytes too large",
                 (unsigned long long)bytes[i]);
        ESGD_ARG(((reinterpret_cast<uintptr_t>(src[i]) | reinterpret_cast<uintptr_t>(dst[i])) & 15) == 0,
                 "gather: segment %d not 16-B aligned", i);
        g.src[i] = src[i]; g.dst[i] = dst[i];
        g.nvec[i] = uint32_t(bytes[i] / 16);
        g.tail[i] = uint32_t(bytes[i] % 16);
        maxvec = std::max<uint64_t>(maxvec, g.nvec[i]);
    }
    unsigned gx = grid_for(256 * 4, maxvec ? maxvec : 1, 8);
    unsigned per_seg = std::max(1u, (unsigned(cu_count()) * 4 + n - 1) / unsigned(n));
    if (gx > per_seg) gx = per_seg;
    if (max_blocks && gx > max_blocks) gx = max_blocks;
    hipLaunchKernelGGL((k_gather<4>), dim3(gx, n), dim3(256), 0, s, g);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// ---- bf16-wire entry points (dataplane.cpp, ESGD_SCHED_WIRE_BF16) ----
int narrow_bf16(float *src, uint16_t *dst, uint64_t n, bool zero_src, hipStream_t s) {
    if (!n) return ESGD_SUCCESS;
    ESGD_ARG(((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0,
             "wire: buckets must be 16-B aligned");
    const dim3 grid(grid_for(1024, n / 4 ? n / 4 : 1, 8));
    if (zero_src) hipLaunchKernelGGL(k_narrow_bf16<true>, grid, dim3(256), 0, s, src, dst, n);
    else hipLaunchKernelGGL(k_narrow_bf16<false>, grid, dim3(256), 0, s, src, dst, n);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

int reduce_wire(int k, const void *const *inputs, uint16_t *outb, float *outf, uint64_t count, hipStream_t s) {
    ESGD_ARG(k >= 1 && k <= ESGD_MAX_FANIN, "wire: fan-in %d", k);
    if (!count) return ESGD_SUCCESS;
    ESGD_ARG(count / 4 * 16 + 4 * 256 * 16 < (1ull << 31), "wire: shard piece of %llu elements too large",
             (unsigned long long)count);
    InputSet in;
    std::memset(&in, 0, sizeof(in));
    uintptr_t al = reinterpret_cast<uintptr_t>(outb) | reinterpret_cast<uintptr_t>(outf);
    for (int j = 0; j < k; ++j) { in.p[j] = inputs[j]; al |= reinterpret_cast<uintptr_t>(inputs[j]); }
    ESGD_ARG((al & 15) == 0, "wire: shards must be 16-B aligned");
    const uint32_t nq = uint32_t(count / 4);
    const unsigned grid = grid_for(1024, nq ? nq : 1, 4);
    switch (k) {
#define ESGD_WK(K) case K: hipLaunchKernelGGL((k_tree_sum_wire<K>), dim3(grid), dim3(256), 0, s, in, outb, outf, nq, count); break;
    ESGD_WK(1) ESGD_WK(2) ESGD_WK(3) ESGD_WK(4) ESGD_WK(5) ESGD_WK(6) ESGD_WK(7) ESGD_WK(8)
#undef ESGD_WK
    }
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

int gather_widen(int n, const void *const *src, void *const *dst, const uint64_t *count, hipStream_t s) {
    ESGD_ARG(n >= 0 && n <= kMaxSeg, "wire gather: %d segments", n);
    if (n == 0) return ESGD_SUCCESS;
    WidenSet g;
    std::memset(&g, 0, sizeof(g));
    uint64_t maxvec = 0;
    for (int i = 0; i < n; ++i) {
        ESGD_ARG(count[i] * 4 < (1ull << 31), "wire gather: segment of %llu elements too large",
                 (unsigned long long)count[i]);
        ESGD_ARG(((reinterpret_cast<uintptr_t>(src[i]) | reinterpret_cast<uintptr_t>(dst[i])) & 15) == 0,
                 "wire gather: segment %d not 16-B aligned", i);
        g.src[i] = static_cast<const uint16_t *>(src[i]);
        g.dst[i] = static_cast<float *>(dst[i]);
        g.n[i] = uint32_t(count[i]);
        maxvec = std::max<uint64_t>(maxvec, count[i] / 4);
    }
    unsigned gx = grid_for(256 * 8, maxvec ? maxvec : 1, 8);
    unsigned per_seg = std::max(1u, (unsigned(cu_count()) * 4 + n - 1) / unsigned(n));
    if (gx > per_seg) gx = per_seg;
    hipLaunchKernelGGL(k_gather_widen, dim3(gx, n), dim3(256), 0, s, g);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// ---- the arena chunk seal (arena.cpp, dataplane.cpp ipc_open) ----
// Written and read by one-wave kernels on the round stream, synchronously.
__global__ void k_seal_write(uint64_t *dst, uint64_t w0, uint64_t w1, uint64_t w2, uint64_t w3) {
    if (threadIdx.x == 0) {
        const uint64_t w[4] = {w0, w1, w2, w3};
        for (int i = 0; i < 4; ++i) __hip_atomic_store(&dst[i], w[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_seal_read(const uint64_t *src, uint64_t *dst) {
    if (threadIdx.x < 4)
        __hip_atomic_store(&dst[threadIdx.x],
                           __hip_atomic_load(const_cast<uint64_t *>(&src[threadIdx.x]), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The seal kernels run on a stream the process already has (seal_stream, dataplane.cpp):
// a stream of their own -- kept, or created per operation (the runtime pools its idle
// hardware queue) -- left one more hardware queue per process, and with it the peer rounds
// of two processes sharing a GPU ran 1.7x slower (round 4, r04m-r04o).
static std::mutex g_seal_mu;
static uint64_t *g_seal_host = nullptr, *g_seal_view = nullptr;   // pinned, mapped
static std::atomic<int> g_seal_busy{0};   // a seal kernel is queued and waited for (diagnostics)

const char *seal_io_busy() { return g_seal_busy.load(std::memory_order_relaxed) ? "yes" : nullptr; }

struct SealBusy {
    SealBusy() { g_seal_busy.fetch_add(1, std::memory_order_relaxed); }
    ~SealBusy() { g_seal_busy.fetch_sub(1, std::memory_order_relaxed); }
};

static int seal_io_begin(hipStream_t *s) {   // g_seal_mu held
    if (int rc = seal_stream(s)) return rc;
    if (!g_seal_host) {
        ESGD_HIP(hipHostMalloc(reinterpret_cast<void **>(&g_seal_host), 64, hipHostMallocMapped));
        ESGD_HIP(hipHostGetDevicePointer(reinterpret_cast<void **>(&g_seal_view), g_seal_host, 0));
    }
    return ESGD_SUCCESS;
}

// the 32-B seal into this process's chunk memory at dst, synchronously
int seal_write(void *dst, const uint64_t w[4]) {
    std::lock_guard<std::mutex> lk(g_seal_mu);
    hipStream_t s = nullptr;
    if (int rc = seal_io_begin(&s)) return rc;
    SealBusy busy;
    hipLaunchKernelGGL(k_seal_write, dim3(1), dim3(64), 0, s, static_cast<uint64_t *>(dst), w[0], w[1], w[2], w[3]);
    ESGD_HIP(hipGetLastError());
    ESGD_HIP(hipStreamSynchronize(s));
    return ESGD_SUCCESS;
}

// the 32 B at src (a peer's chunk, through this process's mapping), synchronously
int seal_read(const void *src, uint64_t w[4]) {
    std::lock_guard<std::mutex> lk(g_seal_mu);
    hipStream_t s = nullptr;
    if (int rc = seal_io_begin(&s)) return rc;
    SealBusy busy;
    for (int i = 0; i < 4; ++i) g_seal_host[i] = 0;
    hipLaunchKernelGGL(k_seal_read, dim3(1), dim3(64), 0, s, static_cast<const uint64_t *>(src), g_seal_view);
    ESGD_HIP(hipGetLastError());
    ESGD_HIP(hipStreamSynchronize(s));
    for (int i = 0; i < 4; ++i) w[i] = reinterpret_cast<volatile uint64_t *>(g_seal_host)[i];
    return ESGD_SUCCESS;
}

// Rank pairing inside a queued round: publish `value` in this rank's flag, then wait
// until every rank's flag has reached it.  The flags live in host memory shared by the
// ranks' processes (the registered node segment), written and read at system scope; one
// lane does it all.  The release fence makes this GPU's earlier writes (the previous
// kernel's shard) visible before the flag is.  A wait that outlives `timeout` ticks of
// the constant wall clock records the round in *err and returns, so a missing peer never
// leaves a wave spinning on the device.
// Every rank's flag at once: lane q polls flags[q] (relaxed, system scope) and the wave
// leaves when all of them reached `value` -- one host-memory round trip per sweep instead
// of one per rank (8 serial PCIe reads at P = 8).  Called by a whole wave; rounds compare
// modulo 2^32.  False on timeout -- or, every 16th sweep, when some rank's error word
// (errs[q], the node segment's per-rank words; nullptr: not checked) holds `errval`: a rank
// that failed this round publishes nothing more for it (the failure contract),
// so waiting for it could only end in the timeout.
__device__ __forceinline__ bool wave_wait_all(const uint32_t *flags, int world, uint32_t value, long long t0,
                                              long long timeout, const uint32_t *errs = nullptr,
                                              uint32_t errval = 0) {
    const int lane = int(threadIdx.x & 63u);
    unsigned sweep = 0;
    for (;;) {
        bool mine = true, bad = false;
        if (lane < world) {
            mine = int32_t(__hip_atomic_load(const_cast<uint32_t *>(&flags[lane]), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM) - value) >= 0;
            if (!mine && errs && (++sweep & 15u) == 0)
                bad = __hip_atomic_load(const_cast<uint32_t *>(&errs[lane]), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_SYSTEM) == errval;
        }
        if (__all(mine)) return true;
        if (__any(bad) || wall_clock64() - t0 > timeout) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

// Publication: release at system scope, drained (MI355X_MICROARCH.md: the explicit wait
// keeps the flag behind the write-back), then the value in every destination word -- one
// word in host memory, or this rank's word in every rank's device flag page.  Lane 0.
__device__ __forceinline__ void publish_flags(const PairFlags &f, uint32_t value) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int q = 0; q < f.ndst; ++q) __hip_atomic_store(f.dst[q], value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The same publication where every byte it announces was stored write-through at system
// scope (sc0 sc1) and drained: no L2 write-back, only the wait.  Lane 0.
__device__ __forceinline__ void publish_flags_drained(const PairFlags &f, uint32_t value) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int q = 0; q < f.ndst; ++q) __hip_atomic_store(f.dst[q], value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Peer buckets are coarse-grained memory of other processes (other GPUs on a node).  When
// the phase after a pairing reads peers, every XCD's L2 (and the L1 of every CU used) must
// first drop whatever lines of them it may still hold from an earlier round -- AFTER the
// pairing saw the peers' flags (on a shared GPU another rank's kernel may re-cache a peer's
// old lines until then).  k_drop_peer_lines, queued right behind the pairing on its stream,
// does it: one workgroup per CU (dealt round-robin over the XCDs), each a system-scope
// acquire (buffer_inv sc0 sc1), none waiting for anything.  The dispatch's own acquire scope
// is not relied on for this.  (Until round 6 these were workgroups of the pairing launch
// itself, spinning on a device gate while the pairing waited for its peers: 256 wave slots
// held per rank for as long as the slowest peer took -- on a GPU shared by 8 ranks, slots
// the peers' own kernels needed to reach the flags they were waiting for (DESIGN.md §5,
// r04zp, r06p).)
__global__ void __launch_bounds__(64) k_drop_peer_lines() {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// One lane pairs the ranks: publish this rank's flag, wait for every rank's.
// Failure contract: `errs` = every rank's error word (this rank's is errs[rank]); a failed
// pairing also records the round in `failw`, a device word of the schedule, and a pairing
// after the round's first (`after_fail`: reduced, done) publishes nothing when failw holds
// the round -- this rank's shard was folded from stale peer buckets, and a late peer must
// not take it for the round's (What's weak 1).  (failw, not the host error
// word: one HBM load instead of a PCIe round trip on every later pairing.)
__global__ void __launch_bounds__(64) k_round_sync(PairFlags f, int world, int rank,
                                                   uint32_t value, long long timeout,
                                                   uint32_t *errs, uint32_t errval, uint32_t *failw, int after_fail,
                                                   uint64_t *ts, uint32_t *fin) {
    const bool lead = threadIdx.x == 0;
    uint32_t *err = errs + rank;
    __shared__ int failed;
    if (lead) {
        failed = after_fail && __hip_atomic_load(failw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == errval;
        if (ts) ts[0] = uint64_t(wall_clock64());
        if (!failed) publish_flags(f, value);
    }
    __syncthreads();
    if (failed) return;   // nothing published, nothing waited for
    const long long t0 = wall_clock64();
    const bool ok = wave_wait_all(f.mine, world, value, t0, timeout, errs, errval);
    if (!lead) return;
    if (!ok) {
        __hip_atomic_store(failw, errval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(err, errval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (ok && ts) __hip_atomic_store(&ts[1], uint64_t(wall_clock64()), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // the round's last kernel reports completion itself (the host polls fin, not an event)
    if (ok && fin) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(fin, errval, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ts (optional): wall-clock stamps of entry and exit (tracing, ESGD_GPU_TRACE=1);
// errval: what a timed-out wait records in *err (the round, also when `value` numbers
// a chunk of it); drop_peer_lines: the next phase reads peer memory (k_drop_peer_lines after)
int round_sync(const PairFlags &f, int world, int rank, uint32_t value, long long timeout_ticks,
               uint32_t *errs, uint32_t errval, uint32_t *failw, bool after_fail, uint64_t *ts, bool drop_peer_lines,
               uint32_t *fin, hipStream_t s) {
    ESGD_ARG(f.mine && errs && failw && world >= 1 && world <= kPairMax && rank >= 0 && rank < world &&
                 f.ndst >= 1 && f.ndst <= kPairMax,
             "round_sync: bad arguments");
    hipLaunchKernelGGL(k_round_sync, dim3(1), dim3(64), 0, s, f, world, rank, value, timeout_ticks, errs, errval,
                       failw, after_fail ? 1 : 0, ts, fin);
    ESGD_HIP(hipGetLastError());
    if (drop_peer_lines) {
        hipLaunchKernelGGL(k_drop_peer_lines, dim3(unsigned(cu_count())), dim3(64), 0, s);
        ESGD_HIP(hipGetLastError());
    }
    return ESGD_SUCCESS;
}

// ---- a whole small round in ONE launch ----
// For small buckets the round is latency-bound: five launches (three pairings, the
// reduce-scatter, the all-gather) cost ~15 us of host time and ~4 us of GPU time per
// kernel boundary (tools/lat.sh).  k_round_small does the same steps inside one kernel of
// at most kSmallBlocks workgroups:
//   publish ready -> wait for every rank's ready -> reduce-scatter (tree order) into rb
//   and the published shard -> grid count; the last workgroup publishes reduced -> wait
//   for every rank's reduced -> all-gather from the peers' published shards -> grid
//   count; the last workgroup writes `fin` (the host polls it instead of an event).
// Hand-offs: every payload store is system-scope write-through (sc0 sc1) and drained
// (s_waitcnt vmcnt(0)) before the workgroup counts itself; peer payload is read with
// system-scope loads after a system-scope acquire.  The grid is far below one workgroup
// per CU, so every workgroup is resident while others wait on it (several ranks sharing
// one GPU included); every wait is bounded by the wall-clock timeout, and a timed-out
// workgroup records the round in *err and leaves.
constexpr int kSmallBlocks = 64;

struct SmallRoundArgs {
    const void *src[kMaxSeg];   // phase 1 inputs: shard `rank` of every rank's rb, rank order
    void *out;                  // phase 1 output: shard `rank` of the local rb ...
    void *pub;                  // ... and of this rank's published shard (peers gather it)
    uint64_t n;                 // elements of the local shard
    const void *gsrc[kMaxSeg];  // phase 2: every other rank's published shard (peer memory) ...
    void *gdst[kMaxSeg];        // ... and where it lands in the local rb
    uint32_t gvec[kMaxSeg];     // 16-B vectors per segment
    uint32_t gtail[kMaxSeg];    // bytes after the last full vector
    int nseg;
    PairFlags ready, reduced;
    uint32_t *fin, *err;
    uint64_t *ts;               // optional GPU trace stamps (6)
    uint32_t *counter;          // device words: [0], [1] arrivals (zero between rounds),
                                // [2], [3] gates raised to the round by the polling lane
    int rank, world;
    uint32_t value;
    long long timeout;
    // ESGD_STRICT_HANDOFFS / esgd_set_config("strict_handoffs"): round 2's hand-offs --
    // acq_rel arrival counts, an agent-scope release on the gates and an L2 write-back
    // before the reduced flag -- instead of the relaxed ones below (a cross-GPU A/B)
    int strict;
};

// err (optional): a word that holds `value` once the round failed elsewhere in this kernel
// (the leader's peer wait), checked every 64th poll -- a wait that can no longer succeed
// ends then, not at the timeout
__device__ __forceinline__ bool spin_all(uint32_t *flags, int world, uint32_t value, long long t0,
                                         long long timeout, const uint32_t *err = nullptr) {
    unsigned polls = 0;
    for (int q = 0; q < world; ++q) {
        while (int32_t(__hip_atomic_load(&flags[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - value) < 0) {
            if (wall_clock64() - t0 > timeout) return false;
            if (err && (++polls & 63u) == 0 &&
                __hip_atomic_load(const_cast<uint32_t *>(err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == value)
                return false;
            __builtin_amdgcn_s_sleep(1);
        }
    }
    return true;
}

// Only ONE lane of the grid polls the ranks' flags in host memory (`leader`): it then
// raises `gate` (a device word) to the round, and every workgroup's lane 0 polls that
// instead -- 64 workgroups polling host memory over PCIe slowed every hand-off ~5x
// (tools/lat.sh).  The workgroup then acquires at system scope.
__device__ __forceinline__ bool block_wait(const SmallRoundArgs &a, const uint32_t *flags, uint32_t *gate,
                                           bool leader, long long t0, int *ok) {
    if (threadIdx.x < 64) {   // the first wave
        bool good = true;
        if (leader) {         // every rank's flag at once, one lane per rank
            good = wave_wait_all(flags, a.world, a.value, t0, a.timeout, a.err - a.rank, a.value);
            // relaxed: the gate carries no data of this workgroup's -- every waiter runs
            // its own system-scope acquire after seeing it (an agent release here was a
            // buffer_wbl2 sc1, ~1.7 us, on every pairing's critical path)
            if (good && threadIdx.x == 0) {
                if (a.strict) __hip_atomic_store(gate, a.value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                else __hip_atomic_store(gate, a.value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else if (threadIdx.x == 0) {
            // the leader records a failed wait in this rank's error word and raises no gate
            good = spin_all(gate, 1, a.value, t0, a.timeout, a.err);
        }
        if (threadIdx.x == 0) {
            if (good) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            else __hip_atomic_store(a.err, a.value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            *ok = good;
        }
    }
    __syncthreads();
    return *ok != 0;
}

// every workgroup drains its stores and counts itself; true in the last one to arrive.
// The count is a relaxed agent-scope add: every payload store of this kernel is
// system-scope write-through (sc0 sc1) and every wave has drained its stores (vmcnt(0))
// before the barrier that precedes the add, so the bytes are in memory before the add
// is issued (MI355X_MICROARCH.md, hand-off table row 1), and the last workgroup reads
// none of them itself.  An acq_rel add lowered to buffer_wbl2 sc1 + buffer_inv sc1 in
// EVERY workgroup, ~3.5 us, twice per round.
// strict: an acq_rel add (round 2's hand-off, ESGD_STRICT_HANDOFFS).
__device__ __forceinline__ bool block_count(uint32_t *ctr, int *last, int strict) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t old = strict ? __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                                    : __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *last = old + 1 == gridDim.x;
        if (*last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return *last != 0;
}

template <class Tr, int K>
__global__ __launch_bounds__(256) void k_round_small(SmallRoundArgs a) {
    using T = typename Tr::T;
    using A = typename Tr::A;
    __shared__ int ok, last;
    const long long t0 = wall_clock64();
    const bool lead = threadIdx.x == 0;
    const bool stamp = a.ts != nullptr && lead;
    if (lead && blockIdx.x == 0) {   // the snapshot queued before this launch has landed
        if (stamp) a.ts[0] = uint64_t(t0);
        // same protocol as k_round_sync: release at system scope, drained, then the flag
        publish_flags(a.ready, a.value);
    }
    if (!block_wait(a, a.ready.mine, &a.counter[2], blockIdx.x == 0, t0, &ok)) return;
    if (stamp && blockIdx.x == 0) a.ts[1] = uint64_t(wall_clock64());

    // phase 1: the local shard, folded in tree order from every rank's rb
    const uint32_t nvec = uint32_t(a.n / Tr::E);
    const int bytes = int(nvec * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.src[j]), (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(a.out, (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t wp = __builtin_amdgcn_make_buffer_rsrc(a.pub, (short)0, bytes, 0x00020000);
    // U vectors per input per lane in flight (the range check drops the ragged end)
    constexpr int U = sizeof(T) == 2 ? 2 : 4;
    for (uint32_t i = blockIdx.x * (256 * U) + threadIdx.x; i < nvec; i += gridDim.x * (256 * U)) {
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j)
                r[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs[j], (i + u * 256) * 16, 0, 17);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const raw16 o = fold16<Tr, K, false>(r[u], 1.0f);
            __builtin_amdgcn_raw_buffer_store_b128(o, ws, (i + u * 256) * 16, 0, 17);
            __builtin_amdgcn_raw_buffer_store_b128(o, wp, (i + u * 256) * 16, 0, 17);
        }
    }
    if (blockIdx.x == 0 && uint64_t(nvec) * Tr::E + threadIdx.x < a.n) {
        const uint64_t e = uint64_t(nvec) * Tr::E + threadIdx.x;
        A v[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            v[j] = Tr::load(__hip_atomic_load(static_cast<const T *>(a.src[j]) + e, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_SYSTEM));
        tree_fold<Tr, K>(v);
        __hip_atomic_store(static_cast<T *>(a.out) + e, Tr::store(v[0]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(static_cast<T *>(a.pub) + e, Tr::store(v[0]), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    const bool last1 = block_count(&a.counter[0], &last, a.strict);
    if (last1 && lead) {
        if (stamp) a.ts[2] = uint64_t(wall_clock64());
        // phase 1 wrote only sc0 sc1 (write-through) stores, drained by every workgroup
        // before its count: no L2 write-back is needed before the flag (strict: one anyway)
        if (a.strict) publish_flags(a.reduced, a.value);
        else publish_flags_drained(a.reduced, a.value);
    }
    if (!block_wait(a, a.reduced.mine, &a.counter[3], last1, t0, &ok)) return;
    // the all-gather span is stamped by ONE workgroup (the last to finish): the wall
    // clocks of different XCDs are not aligned to the microsecond
    const uint64_t t_gather = stamp ? uint64_t(wall_clock64()) : 0;

    // phase 2: every other rank's reduced shard into the local rb.
    // The segments' 1024-vector chunks are dealt over the grid as ONE list, so every
    // workgroup has work whatever the segment sizes (segment by segment, only
    // gvec / 1024 workgroups were busy at a time -- half the grid at P = 2).
    {
        uint32_t total = 0;
        for (int sg = 0; sg < a.nseg; ++sg) total += (a.gvec[sg] + 1023u) / 1024u;
        int sg = 0;
        uint32_t base = 0;   // first chunk index of segment sg
        for (uint32_t c = blockIdx.x; c < total; c += gridDim.x) {
            while (c >= base + (a.gvec[sg] + 1023u) / 1024u) base += (a.gvec[sg++] + 1023u) / 1024u;
            const uint32_t gv = a.gvec[sg];
            __amdgpu_buffer_rsrc_t gs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.gsrc[sg]), (short)0,
                                                                         int(gv * 16u), 0x00020000);
            __amdgpu_buffer_rsrc_t gd = __builtin_amdgcn_make_buffer_rsrc(a.gdst[sg], (short)0, int(gv * 16u),
                                                                         0x00020000);
            const uint32_t i = (c - base) * 1024u + threadIdx.x;
            raw16 r[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(gs, (i + u * 256) * 16, 0, 17);
#pragma unroll
            for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], gd, (i + u * 256) * 16, 0, 17);
        }
    }
    for (int sg = 0; sg < a.nseg; ++sg) {   // ragged tails (bytes after the last vector)
        const uint32_t gv = a.gvec[sg];
        if (blockIdx.x == 0 && threadIdx.x < a.gtail[sg]) {
            const uint8_t *src = static_cast<const uint8_t *>(a.gsrc[sg]) + size_t(gv) * 16;
            uint8_t *dst = static_cast<uint8_t *>(a.gdst[sg]) + size_t(gv) * 16;
            __hip_atomic_store(dst + threadIdx.x,
                               __hip_atomic_load(src + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    // No third pairing: peers gather from `pub`, which this rank rewrites only in the
    // next round's phase 1 -- after that round's ready pairing, i.e. after every peer's
    // kernel of this round has finished -- and rb itself is read by peers only in phase 1.
    if (!block_count(&a.counter[1], &last, a.strict) || !lead) return;
    if (stamp) {
        a.ts[3] = t_gather;
        a.ts[4] = a.ts[5] = uint64_t(wall_clock64());
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the stamps land before fin
    // no fin when a copy-out follows on the stream (its own finish reports the round)
    if (a.fin) __hip_atomic_store(a.fin, a.value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class Tr>
static int launch_small_t(const SmallRoundArgs &a, unsigned grid, hipStream_t s) {
    switch (a.world) {
#define ESGD_SMALL_K(KK) \
    case KK: hipLaunchKernelGGL((k_round_small<Tr, KK>), dim3(grid), dim3(256), 0, s, a); break;
    ESGD_SMALL_K(2) ESGD_SMALL_K(3) ESGD_SMALL_K(4) ESGD_SMALL_K(5) ESGD_SMALL_K(6) ESGD_SMALL_K(7)
    ESGD_SMALL_K(8)
#undef ESGD_SMALL_K
    default:
        set_error("small round: %d ranks outside [2, %d]", a.world, ESGD_MAX_FANIN);
        return ESGD_INVALID_ARG;
    }
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// Entry point of the data plane (dataplane.cpp).  The shard layout keeps every shard
// 1 KiB aligned; segments are checked here.
int round_small(int dtype, const void *const *src, void *out, void *pub, uint64_t n, int nseg,
                const void *const *gsrc, void *const *gdst, const uint64_t *gbytes,
                const PairFlags &ready, const PairFlags &reduced, uint32_t *fin, uint32_t *err,
                uint64_t *ts, uint32_t *counter, int rank, int world, uint32_t value,
                long long timeout_ticks, int strict, hipStream_t s) {
    ESGD_ARG(world >= 2 && world <= ESGD_MAX_FANIN && nseg >= 0 && nseg < kMaxSeg,
             "small round: world %d, %d segments", world, nseg);
    const size_t es = esgd_dtype_size(dtype);
    ESGD_ARG(es > 0, "small round: dtype %d", dtype);
    SmallRoundArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int j = 0; j < world; ++j) a.src[j] = src[j];
    // an empty shard may start anywhere (count 1 at P = 2: shard 1 at element 1)
    ESGD_ARG(n == 0 || ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(pub)) & 15) == 0,
             "small round: shard not 16-B aligned");
    a.out = out;
    a.pub = pub;
    a.n = n;
    uint64_t maxv = n * es / 16;
    for (int i = 0; i < nseg; ++i) {
        ESGD_ARG(((reinterpret_cast<uintptr_t>(gsrc[i]) | reinterpret_cast<uintptr_t>(gdst[i])) & 15) == 0,
                 "small round: segment %d not 16-B aligned", i);
        a.gsrc[i] = gsrc[i];
        a.gdst[i] = gdst[i];
        a.gvec[i] = uint32_t(gbytes[i] / 16);
        a.gtail[i] = uint32_t(gbytes[i] % 16);
        maxv = std::max<uint64_t>(maxv, a.gvec[i]);
    }
    a.nseg = nseg;
    a.ready = ready; a.reduced = reduced; a.fin = fin; a.err = err;
    a.ts = ts;
    a.counter = counter;
    a.rank = rank; a.world = world; a.value = value; a.timeout = timeout_ticks;
    a.strict = strict;
    // at most kSmallBlocks workgroups: every one must be resident
    constexpr uint64_t cap = kSmallBlocks;
    const unsigned grid = unsigned(std::min<uint64_t>(cap, std::max<uint64_t>(1, (maxv + 1023) / 1024)));
    switch (dtype) {
    case ESGD_FLOAT: return launch_small_t<F32>(a, grid, s);
    case ESGD_BF16: return launch_small_t<BF16>(a, grid, s);
    case ESGD_DOUBLE: return launch_small_t<F64>(a, grid, s);
    case ESGD_INT32: return launch_small_t<I32>(a, grid, s);
    case ESGD_INT64: return launch_small_t<I64>(a, grid, s);
    default: break;
    }
    set_error("small round: unsupported dtype %d", dtype);
    return ESGD_INVALID_ARG;
}

}  // namespace esgd

using namespace esgd;

extern "C" {

int esgd_reduce(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                void *stream) {
    return reduce_impl(dtype, k, inputs, out, count, 1.0f, false, stream);
}

int esgd_reduce_scaled(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                       float scale, void *stream) {
    if (scale == 1.0f) return reduce_impl(dtype, k, inputs, out, count, 1.0f, false, stream);
    return reduce_impl(dtype, k, inputs, out, count, scale, true, stream);
}

int esgd_vsum(int dtype, const void *a, const void *b, void *c, uint64_t count, void *stream) {
    // tree order for k=2 is x1 + x0; with x0 = b (rb) and x1 = a (tmp) this is exactly
    // the reference's c = a + b (ffop_gcomp_operator.c:13).
    const void *in[2] = {b, a};
    return reduce_impl(dtype, 2, in, c, count, 1.0f, false, stream);
}

int esgd_pack_div(int n, const float *const *src, const uint64_t *count, float *dst, float divisor,
                  void *stream) {
    return pack_impl(true, n, const_cast<float *const *>(src), count, dst, divisor, stream);
}

int esgd_unpack(int n, float *const *dst, const uint64_t *count, const float *src, void *stream) {
    return pack_impl(false, n, dst, count, const_cast<float *>(src), 1.0f, stream);
}

int esgd_fill_uniform_f32(uint64_t seed, int rank, float *out, uint64_t n, void *stream) {
    ESGD_ARG(out || n == 0, "esgd_fill_uniform_f32: null output");
    if (!n) return ESGD_SUCCESS;
    if (int rc = require_device()) return rc;
    const uint64_t base = seed ^ (uint64_t(uint32_t(rank)) << 40);
    hipLaunchKernelGGL(k_fill_uniform_f32, dim3(grid_for(256, n)), dim3(256), 0, as_stream(stream),
                       base, out, n);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

int esgd_fill_uniform_bf16(uint64_t seed, int rank, uint16_t *out, uint64_t n, void *stream) {
    ESGD_ARG(out || n == 0, "esgd_fill_uniform_bf16: null output");
    if (!n) return ESGD_SUCCESS;
    if (int rc = require_device()) return rc;
    const uint64_t base = seed ^ (uint64_t(uint32_t(rank)) << 40);
    hipLaunchKernelGGL(k_fill_uniform_bf16, dim3(grid_for(256, n)), dim3(256), 0,
                       as_stream(stream), base, out, n);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}
}  // extern "C"
