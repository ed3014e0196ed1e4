// reduce_sweeps.hip — measurement-only variants of the tree reduction (NOT the product).
//
// `make sweeps` builds tools/bin/libesgd_sweeps.so from this file; tools/sweep_reduce.py
// loads it with ctypes next to libesgd.so (which provides memory and streams).  Every
// variant here was measured against the production kernel (reduce_core.h,
// k_tree_sum_buf with nt loads + sc1 stores, 64 MiB windows) and lost; they are kept so
// the sweeps behind profiles/r01 and profiles/r02 stay reproducible:
//   policy 0        flat-address global loads/stores (nt = non-temporal both ways)
//   policy 1..8     other {load aux, store aux} cache-policy pairs of the buffer kernel
//   policy 9..13    block shapes (unroll 3; 512 / 128 / 1024-thread blocks)
//   policy 14..16   store policies (nt only, plain, sc0+sc1)
//   policy 17..20   LDS-DMA ring (buffer_load ... lds), (waves per block, ring depth)
//   policy 21..23   window sizes 32 / 64 / 96 MiB; 24 one launch over the whole bucket
//   policy 25..27   64 MiB windows dealt round-robin over 2 / 3 / 4 streams (forked from and
//                   joined back to the caller's stream by events): a window's launch can
//                   start while the previous one's last workgroups drain; 28 / 29 the same
//                   with 32 / 16 MiB windows over 2 streams
//   policy 30 / 33  ONE launch that walks the 64 / 32 MiB windows itself, a grid-wide barrier
//                   between windows (the grid is what is resident, so every block is there):
//                   the windows' compact footprint without their launch boundaries
//   policy 31 / 32  ONE launch over the whole bucket, each block at most 1 / 2 grid-stride
//                   iterations ahead of the slowest (a shared progress counter): bounded drift
//   policy 34..36   XCD-aware block placement (k_tree_sum_xcd: remapped grid stride, contiguous
//                   range per remapped block, contiguous range per block)
//   policy 37 / 38  window sizes 128 / 48 MiB
//   policy -1       the production launch (the baseline every variant is timed against)
// fp32, fan-in 8 only.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "reduce_core.h"

namespace esgd {

// this library's own error plumbing (libesgd.so keeps its internals local)
static thread_local char g_err[256] = "";
void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
int hip_fail(hipError_t e, const char *what, const char *file, int line) {
    set_error("%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    return ESGD_ERROR;
}

template <bool NT>
__device__ __forceinline__ raw16 ld16(const void *base, uint64_t i) {
    const raw16 *p = static_cast<const raw16 *>(base) + i;
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <bool NT>
__device__ __forceinline__ void st16(void *base, uint64_t i, raw16 v) {
    raw16 *p = static_cast<raw16 *>(base) + i;
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// flat-address body: `nvec` 16-B columns, ragged tail by block 0
template <class Tr, int K, int U, bool NT>
__global__ __launch_bounds__(256) void k_tree_sum_flat(InputSet in, void *out, uint64_t nvec, uint64_t count) {
    constexpr int B = 256;
    const uint64_t stride = uint64_t(gridDim.x) * B * U;
    uint64_t i = uint64_t(blockIdx.x) * B * U + threadIdx.x;
    for (; i + uint64_t(U - 1) * B < nvec; i += stride) {
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) r[u][j] = ld16<NT>(in.p[j], i + u * B);
#pragma unroll
        for (int u = 0; u < U; ++u) st16<NT>(out, i + u * B, fold16<Tr, K, false>(r[u], 1.0f));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t c = i + u * B;
        if (c < nvec) {
            raw16 r[K];
#pragma unroll
            for (int j = 0; j < K; ++j) r[j] = ld16<NT>(in.p[j], c);
            st16<NT>(out, c, fold16<Tr, K, false>(r, 1.0f));
        }
    }
    fold_tail<Tr, K, false>(in, out, nvec * Tr::E, count, 1.0f);
}

// LDS-DMA body: every wave streams chunks of 64 16-B columns; the K inputs of a chunk
// arrive by `buffer_load_dwordx4 ... lds` straight into the wave's own LDS ring, NB - 1
// chunks ahead, and are folded from LDS.  Each wave only reads what it loaded itself, so
// a counted vmcnt is the only synchronisation.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    // gfx9 encoding: vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt[5:4] << 14
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

typedef __attribute__((address_space(3))) char lds_char;

template <int K, int LAUX>
__device__ __forceinline__ void lds_issue(__amdgpu_buffer_rsrc_t (&rs)[K], lds_char *stage, uint32_t col) {
#if defined(__HIP_DEVICE_COMPILE__)   // the LDS-DMA builtin exists for the device target only
#pragma unroll
    for (int j = 0; j < K; ++j)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs[j], (__attribute__((address_space(3))) void *)(stage + j * 1024),
                                                 16, col * 16, 0, 0, LAUX);
#endif
}

template <class Tr, int K, int W, int NB, int LAUX>
__global__ __launch_bounds__(W * 64) void k_tree_sum_lds(InputSet in, void *out, uint32_t nvec, uint64_t count) {
    __shared__ raw16 ring[W][NB][K][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int bytes = int(nvec * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(in.p[j]), (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, bytes, 0x00020000);
    const uint32_t nchunk = (nvec + 63) / 64;
    const uint32_t c0 = blockIdx.x * W + w, step = gridDim.x * W;
    lds_char *mine = (lds_char *)(&ring[w][0][0][0]);
#pragma unroll
    for (int p = 0; p < NB - 1; ++p) lds_issue<K, LAUX>(rs, mine + p * K * 1024, (c0 + p * step) * 64 + lane);
    int st = 0;
    for (uint32_t c = c0; c < nchunk; c += step) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the stage refilled next was read
        lds_issue<K, LAUX>(rs, mine + ((st + NB - 1) % NB) * K * 1024, (c + (NB - 1) * step) * 64 + lane);
        wait_vmcnt<K * (NB - 1)>();                            // chunk c has landed
        raw16 r[K];
#pragma unroll
        for (int j = 0; j < K; ++j) r[j] = ring[w][st][j][lane];
        __builtin_amdgcn_raw_buffer_store_b128(fold16<Tr, K, false>(r, 1.0f), ws, (c * 64 + lane) * 16, 0, 16);
        st = (st + 1) % NB;
    }
    fold_tail<Tr, K, false>(in, out, uint64_t(nvec) * Tr::E, count, 1.0f);
}

template <int U, bool NT>
static int launch_flat(const InputSet &in, void *out, uint64_t count, hipStream_t s, unsigned grid) {
    const uint64_t nvec = count / F32::E;
    const unsigned g = grid_for(uint64_t(256) * U, nvec ? nvec : 1, 8, grid);
    hipLaunchKernelGGL((k_tree_sum_flat<F32, 8, U, NT>), dim3(g), dim3(256), 0, s, in, out, nvec, count);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

template <int W, int NB, int LA>
static int launch_lds(const InputSet &in, void *out, uint64_t count, hipStream_t s, unsigned grid) {
    const uint64_t nvec = count / F32::E;
    static const int per_cu = resident_blocks(k_tree_sum_lds<F32, 8, W, NB, LA>, W * 64);
    const unsigned g = grid_for(uint64_t(W) * 64, (nvec + 63) / 64 * 64 ? (nvec + 63) / 64 * 64 : 1, per_cu, grid);
    hipLaunchKernelGGL((k_tree_sum_lds<F32, 8, W, NB, LA>), dim3(g), dim3(W * 64), 0, s, in, out,
                       uint32_t(nvec), count);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// ---- pacing variants (policies 30-33) ----
// bar[0]: arrivals (barrier) / finished iterations (drift), bar[1]: barrier generation,
// bar[2]: blocks done.  The last block out resets bar[0] and bar[2], so consecutive launches
// on one stream start from zero.  Every wait gives up after ~1 s of polling (a block that is
// not resident can never arrive; the kernel then finishes unpaced instead of hanging).
// Every counter access is relaxed: the windows share no data, only pacing, and an acquire
// or release at agent scope costs an L2 invalidate / write-back per block on gfx950 (the
// first version, with acq_rel, ran 1.5-4x slower than production).
constexpr uint32_t kSpinLimit = 1u << 20;

__device__ __forceinline__ void grid_barrier(uint32_t *bar) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t gen = __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&bar[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            for (uint32_t n = 0; n < kSpinLimit &&
                                 __hip_atomic_load(&bar[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen; ++n)
                __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
}

__device__ __forceinline__ void block_exit(uint32_t *bar) {
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(&bar[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
        __hip_atomic_store(&bar[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bar[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the production loop body over one window [v0, v0 + nv) of 16-B columns
template <int U>
__device__ __forceinline__ void window_body(const InputSet &in, void *out, uint64_t v0, uint32_t nv) {
    constexpr int B = 256, K = 8;
    const int bytes = int(nv * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(static_cast<const char *>(in.p[j])) + v0 * 16,
                                                  (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(static_cast<char *>(out) + v0 * 16, (short)0,
                                                                  bytes, 0x00020000);
    const uint32_t step = gridDim.x * (B * U);
    for (uint32_t i = blockIdx.x * (B * U) + threadIdx.x; i < nv; i += step) {
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) r[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs[j], (i + u * B) * 16, 0, 2);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(fold16<F32, K, false>(r[u], 1.0f), ws, (i + u * B) * 16, 0, 16);
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_tree_sum_paced_windows(InputSet in, void *out, uint64_t count,
                                                                 uint32_t win_vec, uint32_t *bar) {
    const uint64_t nvec = count / 4;
    for (uint64_t v0 = 0; v0 < nvec; v0 += win_vec) {
        if (v0) grid_barrier(bar);
        window_body<U>(in, out, v0, uint32_t(nvec - v0 < win_vec ? nvec - v0 : win_vec));
    }
    fold_tail<F32, 8, false>(in, out, nvec * 4, count, 1.0f);
    block_exit(bar);
}

template <int U, int D>
__global__ __launch_bounds__(256) void k_tree_sum_bounded_drift(InputSet in, void *out, uint32_t nvec,
                                                                 uint64_t count, uint32_t *bar) {
    constexpr int B = 256, K = 8;
    const int bytes = int(nvec * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(in.p[j]), (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, bytes, 0x00020000);
    const uint32_t step = gridDim.x * (B * U);
    uint32_t k = 0;
    for (uint32_t i = blockIdx.x * (B * U) + threadIdx.x; __builtin_amdgcn_readfirstlane(i - threadIdx.x) < nvec;
         i += step, ++k) {
        if (k > D) {   // iteration k may start once every block has finished iteration k - D - 1
            if (threadIdx.x == 0) {
                const uint32_t need = (k - D) * gridDim.x;
                for (uint32_t n = 0; n < kSpinLimit &&
                                     __hip_atomic_load(&bar[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need; ++n)
                    __builtin_amdgcn_s_sleep(2);
            }
            __syncthreads();
        }
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) r[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs[j], (i + u * B) * 16, 0, 2);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(fold16<F32, K, false>(r[u], 1.0f), ws, (i + u * B) * 16, 0, 16);
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(&bar[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // blocks with fewer iterations still count the ones they skip, so `need` is reachable
    const uint32_t iters = (nvec + step - 1) / step;
    if (threadIdx.x == 0 && k < iters)
        __hip_atomic_fetch_add(&bar[0], iters - k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fold_tail<F32, 8, false>(in, out, uint64_t(nvec) * 4, count, 1.0f);
    block_exit(bar);
}

// XCD-aware block placement.  Workgroups are dealt round-robin over the 8 XCDs (block b on
// XCD b % 8), so in the production grid-stride order neighbouring 16 KiB slices of every
// input stream through eight different L2s.  MODE 0: the grid-stride loop over a remapped
// block index (XCD x owns logical blocks x*G/8 .. (x+1)*G/8-1, a contiguous eighth of
// every pass); MODE 1: every logical (remapped) block walks one contiguous range of the
// bucket, so each XCD streams one contiguous eighth of it; MODE 2: contiguous ranges per
// block without the remap.
template <int U, int MODE>
__global__ __launch_bounds__(256) void k_tree_sum_xcd(InputSet in, void *out, uint32_t nvec, uint64_t count) {
    constexpr int B = 256, K = 8;
    const int bytes = int(nvec * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(in.p[j]), (short)0, bytes, 0x00020000);
    __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, bytes, 0x00020000);
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint32_t lb = (MODE == 2) ? b : (b % 8u) * (G / 8u) + b / 8u;
    uint32_t first, last, step;
    if constexpr (MODE == 0) {
        first = lb * (B * U);
        last = nvec;
        step = G * (B * U);
    } else {
        const uint32_t chunk = B * U;
        const uint32_t per = ((nvec + G - 1) / G + chunk - 1) / chunk * chunk;
        first = lb * per;
        last = first + per < nvec ? first + per : nvec;
        step = chunk;
    }
    for (uint32_t i = first + threadIdx.x; i - threadIdx.x < last; i += step) {
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j) r[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs[j], (i + u * B) * 16, 0, 2);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(fold16<F32, K, false>(r[u], 1.0f), ws, (i + u * B) * 16, 0, 16);
    }
    fold_tail<F32, 8, false>(in, out, uint64_t(nvec) * 4, count, 1.0f);
}

template <int MODE>
static int launch_xcd(const InputSet &in, void *out, uint64_t count, hipStream_t s, unsigned fixed) {
    const uint64_t nvec = count / 4;
    if (nvec >= (uint64_t(1) << 27)) {
        set_error("xcd policies take one descriptor range (< 2 GiB)");
        return ESGD_INVALID_ARG;
    }
    static const int per_cu = resident_blocks(k_tree_sum_xcd<4, MODE>, 256);
    unsigned grid = grid_for(uint64_t(256) * 4, nvec ? nvec : 1, per_cu, fixed);
    if (MODE != 2) grid = grid < 8 ? 8 : grid / 8 * 8;   // the remap needs G % 8 == 0
    hipLaunchKernelGGL((k_tree_sum_xcd<4, MODE>), dim3(grid), dim3(256), 0, s, in, out, uint32_t(nvec), count);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

static uint32_t *g_bar = nullptr;

static int pace_bar(uint32_t **out) {
    if (!g_bar) {
        ESGD_HIP(hipMalloc(reinterpret_cast<void **>(&g_bar), 64));
        ESGD_HIP(hipMemset(g_bar, 0, 64));
        ESGD_HIP(hipDeviceSynchronize());
    }
    *out = g_bar;
    return ESGD_SUCCESS;
}

static int launch_paced_windows(const InputSet &in, void *out, uint64_t count, hipStream_t s, uint64_t window_bytes) {
    uint32_t *bar = nullptr;
    if (int rc = pace_bar(&bar)) return rc;
    static const int per_cu = resident_blocks(k_tree_sum_paced_windows<4>, 256);
    const uint64_t win_vec = window_bytes / 16;
    const unsigned grid = grid_for(uint64_t(256) * 4, std::min<uint64_t>(win_vec, count / 4 ? count / 4 : 1), per_cu);
    hipLaunchKernelGGL((k_tree_sum_paced_windows<4>), dim3(grid), dim3(256), 0, s, in, out, count,
                       uint32_t(win_vec), bar);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

template <int D>
static int launch_bounded_drift(const InputSet &in, void *out, uint64_t count, hipStream_t s) {
    uint32_t *bar = nullptr;
    if (int rc = pace_bar(&bar)) return rc;
    static const int per_cu = resident_blocks(k_tree_sum_bounded_drift<4, D>, 256);
    const uint64_t nvec = count / 4;
    const unsigned grid = grid_for(uint64_t(256) * 4, nvec ? nvec : 1, per_cu);
    hipLaunchKernelGGL((k_tree_sum_bounded_drift<4, D>), dim3(grid), dim3(256), 0, s, in, out, uint32_t(nvec),
                       count, bar);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// windows over NS streams: stream 0 is the caller's, the others fork from it and join back
static hipStream_t g_aux[4] = {};
static hipEvent_t g_fork = nullptr, g_join[4] = {};

static int launch_windows_streams(const InputSet &in, void *out, uint64_t count, hipStream_t s, int ns,
                                  unsigned grid, uint64_t window_bytes = kWindowBytes) {
    const uint64_t w = window_bytes / 4;
    if (count <= w + w / 2) return launch_buf<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, grid);
    if (!g_fork) {
        ESGD_HIP(hipEventCreateWithFlags(&g_fork, hipEventDisableTiming));
        for (int i = 1; i < 4; ++i) {
            ESGD_HIP(hipStreamCreateWithFlags(&g_aux[i], hipStreamNonBlocking));
            ESGD_HIP(hipEventCreateWithFlags(&g_join[i], hipEventDisableTiming));
        }
    }
    ESGD_HIP(hipEventRecord(g_fork, s));
    for (int i = 1; i < ns; ++i) ESGD_HIP(hipStreamWaitEvent(g_aux[i], g_fork, 0));
    int idx = 0;
    for (uint64_t o = 0; o < count; o += w, ++idx) {
        InputSet sl = in;
        for (int j = 0; j < 8; ++j) sl.p[j] = static_cast<const float *>(in.p[j]) + o;
        hipStream_t st = (idx % ns) == 0 ? s : g_aux[idx % ns];
        if (int rc = launch_buf<F32, 8, 4, 2, 16, false>(sl, static_cast<float *>(out) + o, std::min(w, count - o),
                                                         1.0f, st, grid))
            return rc;
    }
    for (int i = 1; i < ns; ++i) {
        ESGD_HIP(hipEventRecord(g_join[i], g_aux[i]));
        ESGD_HIP(hipStreamWaitEvent(s, g_join[i], 0));
    }
    return ESGD_SUCCESS;
}

// A stand-in for a concurrent persistent kernel (an RCCL kernel, a long kernel on another
// stream of the training loop): workgroups of 1024 threads (16 waves: two fill a CU's 32
// wave slots) that stay resident for `ticks` of the constant wall clock, then leave.
__global__ __launch_bounds__(1024) void k_occupy(long long ticks) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

}  // namespace esgd

using namespace esgd;

extern "C" {

// `blocks` k_occupy workgroups on `stream` for `usec` microseconds each (the residency test
// of batched rounds, tests/test_dataplane_gpu.py: 2 x CUs - 2k blocks leave k CUs' worth of
// wave slots free); returns at once
int esgd_sweep_occupy(int blocks, uint64_t usec, void *stream) {
    if (blocks <= 0) { set_error("occupy: %d blocks", blocks); return ESGD_INVALID_ARG; }
    int dev = 0, khz = 0;
    ESGD_HIP(hipGetDevice(&dev));
    ESGD_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    const long long ticks = (long long)usec * khz / 1000;
    hipLaunchKernelGGL(k_occupy, dim3(unsigned(blocks)), dim3(1024), 0, static_cast<hipStream_t>(stream), ticks);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

// the device's compute units (sizing the occupying grid)
int esgd_sweep_cu_count(void) { return cu_count(); }

const char *esgd_sweep_last_error(void) { return g_err; }

// One fp32 fan-in-8 reduction with variant `policy` (see the table at the top); unroll
// (2 or 4) and nt apply to policy 0; grid > 0 fixes the grid of the buffer / flat / LDS
// kernels.  Same bits as esgd_reduce for every variant (tools/sweep_reduce.py checks).
int esgd_sweep_reduce(int policy, int unroll, int nt, int grid, const void *const *inputs, void *out,
                      uint64_t count, void *stream) {
    if (!inputs || !out) { set_error("null argument"); return ESGD_INVALID_ARG; }
    InputSet in;
    std::memset(&in, 0, sizeof(in));
    for (int j = 0; j < 8; ++j) in.p[j] = inputs[j];
    hipStream_t s = static_cast<hipStream_t>(stream);
    const unsigned g = grid > 0 ? unsigned(grid) : 0u;
    const bool fits32 = count / 4 * 16 + uint64_t(4) * 256 * 16 < (1ull << 31);
    if (policy != -1 && policy != 0 && !fits32) {
        set_error("policy %d needs the bucket inside one 32-bit descriptor range", policy);
        return ESGD_INVALID_ARG;
    }
    switch (policy) {
    case -1: return launch_windows<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, kWindowBytes, g);
    case 0:
        if (unroll == 4) return nt ? launch_flat<4, true>(in, out, count, s, g) : launch_flat<4, false>(in, out, count, s, g);
        return nt ? launch_flat<2, true>(in, out, count, s, g) : launch_flat<2, false>(in, out, count, s, g);
#define ESGD_POL(ID, LA, SA) case ID: return launch_buf<F32, 8, 4, LA, SA, false>(in, out, count, 1.0f, s, g);
    ESGD_POL(1, 2, 16) ESGD_POL(2, 2, 17) ESGD_POL(3, 2, 18) ESGD_POL(4, 2, 19)
    ESGD_POL(5, 0, 16) ESGD_POL(6, 3, 16) ESGD_POL(7, 18, 16) ESGD_POL(8, 16, 16)
#undef ESGD_POL
    case 9: return launch_buf<F32, 8, 3, 2, 16, false>(in, out, count, 1.0f, s, g);
    case 10: return launch_buf<F32, 8, 2, 2, 16, false, 512>(in, out, count, 1.0f, s, g);
    case 11: return launch_buf<F32, 8, 4, 2, 16, false, 512>(in, out, count, 1.0f, s, g);
    case 12: return launch_buf<F32, 8, 4, 2, 16, false, 128>(in, out, count, 1.0f, s, g);
    case 13: return launch_buf<F32, 8, 2, 2, 16, false, 1024>(in, out, count, 1.0f, s, g);
    case 14: return launch_buf<F32, 8, 4, 2, 2, false>(in, out, count, 1.0f, s, g);
    case 15: return launch_buf<F32, 8, 4, 2, 0, false>(in, out, count, 1.0f, s, g);
    case 16: return launch_buf<F32, 8, 4, 2, 3, false>(in, out, count, 1.0f, s, g);
    case 17: return launch_lds<4, 2, 2>(in, out, count, s, g);
    case 18: return launch_lds<2, 4, 2>(in, out, count, s, g);
    case 19: return launch_lds<1, 8, 2>(in, out, count, s, g);
    case 20: return launch_lds<2, 3, 2>(in, out, count, s, g);
    case 21: return launch_windows<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, uint64_t(32) << 20, g);
    case 22: return launch_windows<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, uint64_t(64) << 20, g);
    case 23: return launch_windows<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, uint64_t(96) << 20, g);
    case 24: return launch_buf<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, g);
    case 25: return launch_windows_streams(in, out, count, s, 2, g);
    case 26: return launch_windows_streams(in, out, count, s, 3, g);
    case 27: return launch_windows_streams(in, out, count, s, 4, g);
    case 28: return launch_windows_streams(in, out, count, s, 2, g, uint64_t(32) << 20);
    case 29: return launch_windows_streams(in, out, count, s, 2, g, uint64_t(16) << 20);
    case 30: return launch_paced_windows(in, out, count, s, uint64_t(64) << 20);
    case 31: return launch_bounded_drift<1>(in, out, count, s);
    case 32: return launch_bounded_drift<2>(in, out, count, s);
    case 37: return launch_windows<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, uint64_t(128) << 20, g);
    case 38: return launch_windows<F32, 8, 4, 2, 16, false>(in, out, count, 1.0f, s, uint64_t(48) << 20, g);
    case 34: return launch_xcd<0>(in, out, count, s, g);
    case 35: return launch_xcd<1>(in, out, count, s, g);
    case 36: return launch_xcd<2>(in, out, count, s, g);
    case 33: return launch_paced_windows(in, out, count, s, uint64_t(32) << 20);
    default: break;
    }
    set_error("unknown policy %d", policy);
    return ESGD_INVALID_ARG;
}

}  // extern "C"
