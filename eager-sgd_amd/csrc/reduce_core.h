// reduce_core.h — the tree-order bucket reduction kernel and its launch sizing, shared by
// libesgd.so (reduce_kernels.hip) and the tools-only sweep library
// (tools/sweeps/reduce_sweeps.hip, `make sweeps`).  Device templates and header-only
// launch helpers; nothing here is exported.
//
// Reference behaviour (fflib2, /root/reference/eager-SGD-modules/fflib2):
//   * FFSUM on a pair of buffers, c = a + b, is a scalar C loop strip-mined in 1024s
//     on the progress pthread (src/components/gcomp/ffop_gcomp_operator.c:8-25, 33-58).
//   * ffallreduce applies it log2(P) times in recursive-doubling order
//     (src/colls/ffallreduce.c:138-171), so every rank ends with the hypercube tree
//     ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7)).
// Here the whole tree is one pass: each lane loads 16 B from each of the k inputs,
// folds them in exactly that tree order in registers and stores 16 B once.  The
// result is bit-identical to the reference for fp32/fp64/int32/int64 (no FMA, no
// reassociation, denormals kept — hipcc's default f32 denorm mode).
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "esgd_internal.h"

namespace esgd {

using raw16 = __attribute__((ext_vector_type(4))) unsigned int;  // one 16-B access

struct InputSet {
    const void *p[ESGD_MAX_FANIN];
};

// ---- element traits: T = storage, A = accumulator, E = elements per 16 B ----
struct F32 {
    using T = float; using A = float; static constexpr int E = 4;
    __device__ static A load(T x) { return x; }
    __device__ static T store(A a) { return a; }
};
struct F64 {
    using T = double; using A = double; static constexpr int E = 2;
    __device__ static A load(T x) { return x; }
    __device__ static T store(A a) { return a; }
};
struct I32 {  // wrapping two's-complement add, like the reference's int32 SUM
    using T = uint32_t; using A = uint32_t; static constexpr int E = 4;
    __device__ static A load(T x) { return x; }
    __device__ static T store(A a) { return a; }
};
struct I64 {
    using T = uint64_t; using A = uint64_t; static constexpr int E = 2;
    __device__ static A load(T x) { return x; }
    __device__ static T store(A a) { return a; }
};
struct BF16 {  // extension: fp32 accumulate, one round-to-nearest-even at the end
    using T = uint16_t; using A = float; static constexpr int E = 8;
    __device__ static A load(T x) { return __uint_as_float(uint32_t(x) << 16); }
    __device__ static T store(A a) {
        uint32_t u = __float_as_uint(a);
        if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu))
            return uint16_t((u >> 16) | 0x0040u);            // NaN stays a (quiet) NaN
        u += 0x7fffu + ((u >> 16) & 1u);
        return uint16_t(u >> 16);
    }
};

// The hypercube tree of ffallreduce.c:138-171 as rank 0 evaluates it: at distance s
// the partner's partial (operand a, `tmp`) is added to the local one (operand b, `rb`).
template <class Tr, int K>
__device__ __forceinline__ void tree_fold(typename Tr::A (&v)[K]) {
#pragma unroll
    for (int s = 1; s < K; s <<= 1) {
#pragma unroll
        for (int j = 0; j + s < K; j += 2 * s) v[j] = v[j + s] + v[j];
    }
}

// fold one 16-B column of K inputs
template <class Tr, int K, bool SCALE>
__device__ __forceinline__ raw16 fold16(const raw16 (&r)[K], float scale) {
    using T = typename Tr::T;
    using A = typename Tr::A;
    constexpr int E = Tr::E;
    T out[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
        A v[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            T x;
            __builtin_memcpy(&x, reinterpret_cast<const char *>(&r[j]) + e * sizeof(T), sizeof(T));
            v[j] = Tr::load(x);
        }
        tree_fold<Tr, K>(v);
        if constexpr (SCALE) v[0] = v[0] * scale;
        out[e] = Tr::store(v[0]);
    }
    raw16 o;
    __builtin_memcpy(&o, out, 16);
    return o;
}

// ragged tail (< E elements after the last 16-B column): block 0, one element per lane
template <class Tr, int K, bool SCALE>
__device__ __forceinline__ void fold_tail(const InputSet &in, void *out, uint64_t tail0, uint64_t count,
                                          float scale) {
    using T = typename Tr::T;
    using A = typename Tr::A;
    if (blockIdx.x == 0 && tail0 + threadIdx.x < count) {
        const uint64_t e = tail0 + threadIdx.x;
        A v[K];
#pragma unroll
        for (int j = 0; j < K; ++j) v[j] = Tr::load(static_cast<const T *>(in.p[j])[e]);
        tree_fold<Tr, K>(v);
        if constexpr (SCALE) v[0] = v[0] * scale;
        static_cast<T *>(out)[e] = Tr::store(v[0]);
    }
}

// Production body: buffer-descriptor loads/stores (`buffer_load_dwordx4 ... offen`) with
// explicit cache-policy bits (aux: 1 = sc0, 2 = nt, 16 = sc1).  Measured on MI355X
// (profiles/r01/sweep_policy.md): nt loads + sc1 (write-through, not retained in L2)
// stores move 6.5 TB/s at k = 8 x 256 MiB against 5.9 TB/s for plain global
// loads/stores — the once-read inputs and the once-written output stop competing for
// L2 / Infinity Cache.  The descriptor's range check (num_records = bytes of the vector
// body) turns the ragged last iteration into zero-fill loads and dropped stores, so the
// loop has no per-element branch (cdna_hip_programming.md §5 item 4c).
// MI355X mapping: pure HBM streaming (k reads + 1 write per element, ~0.2 FLOP/B),
// so the design goal is bytes in flight: 64-wide waves, 16-B loads per lane
// (1 KiB per wave-instruction), U independent vectors per input per lane, a
// grid-stride loop over what is resident at once.  No LDS: there is no reuse to stage,
// and a round trip through it only adds instructions (cdna_hip_programming.md Appendix B
// "Element-wise"; the LDS-DMA ring variants measured slower: profiles/r02).
template <class Tr, int K, int U, int LAUX, int SAUX, bool SCALE, int B = 256>
__global__ __launch_bounds__(B) void k_tree_sum_buf(InputSet in, void *out, uint32_t nvec,
                                                     uint64_t count, float scale) {
    const int bytes = int(nvec * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(in.p[j]), (short)0, bytes,
                                                  0x00020000);
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, bytes, 0x00020000);
    const uint32_t step = gridDim.x * (B * U);
    for (uint32_t i = blockIdx.x * (B * U) + threadIdx.x; i < nvec; i += step) {
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j)
                r[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs[j], (i + u * B) * 16, 0, LAUX);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(fold16<Tr, K, SCALE>(r[u], scale), ws,
                                                   (i + u * B) * 16, 0, SAUX);
    }
    fold_tail<Tr, K, SCALE>(in, out, uint64_t(nvec) * Tr::E, count, scale);
}

// Fallback for pointers that are not 16-B aligned: one element per lane.
template <class Tr, int K, bool SCALE>
__global__ __launch_bounds__(256) void k_tree_sum_scalar(InputSet in, void *out, uint64_t count,
                                                          float scale) {
    using T = typename Tr::T;
    using A = typename Tr::A;
    const uint64_t stride = uint64_t(gridDim.x) * 256;
    for (uint64_t e = uint64_t(blockIdx.x) * 256 + threadIdx.x; e < count; e += stride) {
        A v[K];
#pragma unroll
        for (int j = 0; j < K; ++j) v[j] = Tr::load(static_cast<const T *>(in.p[j])[e]);
        tree_fold<Tr, K>(v);
        if constexpr (SCALE) v[0] = v[0] * scale;
        static_cast<T *>(out)[e] = Tr::store(v[0]);
    }
}

// ---- launch sizing ----
inline int cu_count() {
    static int cus[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        hipDeviceProp_t p;
        cus[dev] = (hipGetDeviceProperties(&p, dev) == hipSuccess && p.multiProcessorCount > 0)
                       ? p.multiProcessorCount : 256;
    }
    return cus[dev];
}

// Grid-stride launches are sized to what is resident at once (CUs x blocks per CU that
// the kernel's registers admit): a second, queued wave of blocks only adds a tail
// (profiles/r01/sweep_grid.md: 1024 blocks = 4/CU beat 2048 at 98 VGPRs).
// `fixed` > 0 (sweeps only) replaces the computed grid.
inline unsigned grid_for(uint64_t items_per_block_pass, uint64_t items, int blocks_per_cu = 8,
                         unsigned fixed = 0) {
    if (fixed > 0) return fixed;
    uint64_t need = (items + items_per_block_pass - 1) / items_per_block_pass;
    uint64_t cap = uint64_t(cu_count()) * uint64_t(blocks_per_cu > 0 ? blocks_per_cu : 1);
    if (need < 1) need = 1;
    return unsigned(need < cap ? need : cap);
}

template <typename KernelT>
int resident_blocks(KernelT kernel, int block = 256) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, block, 0) != hipSuccess || nb <= 0)
        nb = 4;
    return nb < 8 ? nb : 8;
}

template <class Tr, int K, int U, int LA, int SA, bool SCALE, int B = 256>
int launch_buf(const InputSet &in, void *out, uint64_t count, float scale, hipStream_t s,
               unsigned fixed_grid = 0) {
    const uint64_t nvec = count / Tr::E;
    static const int per_cu = resident_blocks(k_tree_sum_buf<Tr, K, U, LA, SA, SCALE, B>, B);
    unsigned grid = grid_for(uint64_t(B) * U, nvec ? nvec : 1, per_cu, fixed_grid);
    hipLaunchKernelGGL((k_tree_sum_buf<Tr, K, U, LA, SA, SCALE, B>), dim3(grid), dim3(B), 0, s, in,
                       out, uint32_t(nvec), count, scale);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// Buckets larger than a window run as consecutive launches over window-sized slices of
// every input (same kernel, same per-element work).  Measured at 8 inputs
// (profiles/r02/sweeps_windowed.jsonl): one launch over 8 x 256 MiB reached 77.6-78.1 %
// of 8 TB/s, 64 MiB windows 80.1 %; 8 x 1 GiB 67.8 % -> 74.8 %; at 128 MiB 79.5 -> 81.2 %.
// Each launch starts its occupancy-sized grid together at the window's start, where one
// long grid-stride launch lets its workgroups drift apart over the whole footprint.
// Every window also fits the buffer descriptors' 32-bit range, whatever the bucket size.
constexpr uint64_t kWindowBytes = uint64_t(64) << 20;

template <class Tr, int K, int U, int LA, int SA, bool SCALE>
int launch_windows(const InputSet &in, void *out, uint64_t count, float scale, hipStream_t s,
                   uint64_t window_bytes = kWindowBytes, unsigned fixed_grid = 0) {
    using T = typename Tr::T;
    const uint64_t w = window_bytes / sizeof(T);
    if (count <= w + w / 2) return launch_buf<Tr, K, U, LA, SA, SCALE>(in, out, count, scale, s, fixed_grid);
    for (uint64_t o = 0; o < count; o += w) {
        InputSet sl = in;
        for (int j = 0; j < K; ++j) sl.p[j] = static_cast<const T *>(in.p[j]) + o;
        if (int rc = launch_buf<Tr, K, U, LA, SA, SCALE>(sl, static_cast<T *>(out) + o, std::min(w, count - o),
                                                         scale, s, fixed_grid))
            return rc;
    }
    return ESGD_SUCCESS;
}

template <class Tr, int K, bool SCALE>
int launch_scalar(const InputSet &in, void *out, uint64_t count, float scale, hipStream_t s) {
    unsigned grid = grid_for(256, count);
    hipLaunchKernelGGL((k_tree_sum_scalar<Tr, K, SCALE>), dim3(grid), dim3(256), 0, s, in, out,
                       count, scale);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

}  // namespace esgd
