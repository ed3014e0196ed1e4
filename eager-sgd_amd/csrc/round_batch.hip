// round_batch.hip — k_round_batch: the one-launch rounds due in issue order, in one kernel.
//
// Grid: ONE agent workgroup (block 0, dispatched first) plus `workers` workgroups of 256
// threads.  Residency contract: the agent and at least ONE worker must be resident; the
// other workers may be kept out by concurrent kernels (a torch stream, an RCCL kernel,
// other ranks sharing the GPU).  Workers take tiles from a per-process counter in list
// order (BatchArgs::dynamic), so every tile a resident worker spins on depends only on
// tiles already taken -- by workers that are running -- and on peers' flags of entries no
// later in the ring.  (Static assignment, tile g on worker 1 + g % workers, needed every
// worker resident at once: one not dispatched while the others spun on gates its own tiles
// would open deadlocked the launch -- round 4, 8 ranks on one GPU.)  The host still sizes
// the grid to what the ranks sharing this GPU leave free (round_batch_capacity), for speed.
//
// Agent (wave 0 of block 0; lane e owns entry e):
//   * publishes `ready` of every entry at once -- everything the entries' snapshots
//     wrote was queued on the stream before this launch -- behind one system-scope
//     release (L2 write-back) and a drain; an entry whose snapshot the workers do in this
//     launch (phase 0) publishes once all its snapshot tiles have counted themselves;
//   * polls every rank's ready / reduced flag of its entry (one system-scope load per rank,
//     all lanes' loads in flight together) and raises the entry's device gates.
// Workers walk a global tile list in ring order -- every entry's snapshot tiles, then its
// phase-1 tiles, then its phase-2 tiles -- taking the next tile from the counter:
//   * phase 0 (snapshot, ESGD_SNAPSHOT_IN_BATCH): 1024 vectors of rb = sb, rb = 0 or, for a
//     round posted with its own send data (esgd_schedule_post_io), rb = src / divisor --
//     write-through, drained, counted -- no gate: every snapshot tile is taken before any
//     gated tile;
//   * phase 1 (reduce-scatter): wait for the entry's ready gate; fold one tile (tv1 16-B
//     vectors) of shard `rank` of every rank's rb in the reference's tree order
//     (ffallreduce.c:138-171 via tree_fold) into the local rb (or the round's own output)
//     and the published shard; the last tile of an entry to arrive publishes the entry's
//     `reduced` flag;
//   * phase 2 (all-gather): wait for the entry's reduced gate; copy one tile of a peer's
//     published shard into the local rb (or the round's own output); the last tile to
//     arrive stores the round in the entry's fin word (the host polls it).
// The agent never waits for one entry before serving another, and a worker's tiles come
// in ring order, so a flag of entry i depends only on flags of entries <= i on every rank:
// ranks that cut the issue ring into launches differently cannot deadlock.
//
// Hand-offs (relaxed, as in k_round_small; strict with BatchDesc::strict): payload stores
// are system-scope write-through (sc0 sc1) and drained by every wave before its workgroup
// counts itself; peer memory is read with system-scope loads, and each worker drops stale
// peer lines from its CU's L1 and its XCD's L2 once, at the start of the launch (every
// read of peer memory in this launch follows its gate, and no entry's buffers are touched
// by an earlier launch's reads after that point).
#include <atomic>

#include "reduce_core.h"
#include "round_batch.h"

namespace esgd {

namespace {

__device__ __forceinline__ bool reached(uint32_t v, uint32_t want) { return int32_t(v - want) >= 0; }

__device__ __forceinline__ uint32_t load_sys(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void store_sys(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void store_gate(uint32_t *p, uint32_t v, bool strict) {
    if (strict) __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one entry's flag words in every destination (host memory: one word; device flag pages:
// this rank's word in every rank's page)
__device__ __forceinline__ void put_flags(const PairFlags &f, uint32_t v) {
    for (int q = 0; q < f.ndst; ++q) store_sys(f.dst[q], v);
}

// A timed-out wait: the host fails the round (err) and no worker is left waiting (both
// gates open).  err is released at system scope before the gates: a worker's fin can only
// follow an open gate, and the host reads fin before err (dataplane.cpp base_query).
__device__ __forceinline__ void fail_entry(const BatchDesc *d, uint32_t v) {
    store_sys(d->err, v);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_gate(d->ctr + 2, v, false);
    store_gate(d->ctr + 3, v, false);
}

template <int K>
__device__ void agent(const BatchArgs &a, long long t0) {
    const int lane = int(threadIdx.x);
    const bool act = lane < int(a.nent);
    const BatchDesc *d = act ? &a.table[a.sid[lane]] : nullptr;
    const uint32_t v = act ? a.value[lane] : 0u;
    // entries whose snapshot the workers do first wait for it (-1) before their ready
    const uint32_t snaps = act && a.snap[lane] ? a.tile0[lane + 1] - a.tile0[lane] : 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // system scope: what the snapshots wrote
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (act && !snaps) put_flags(d->ready, v);
    int st = act ? (snaps ? -1 : 0) : 2;   // 0: waiting for every ready, 1: for every reduced, 2: done
    for (;;) {
        bool pub = false;   // this entry's snapshot has just landed
        if (st == -1) {
            // the snapshot tiles stored write-through and drained before counting: once all
            // are counted the bucket is in memory, and the ready below follows a release
            const uint32_t n = __hip_atomic_load(d->ctr + 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (n >= snaps) {
                __hip_atomic_store(d->ctr + 4, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                st = 0;
                pub = true;
            } else if (wall_clock64() - t0 > a.timeout) {
                fail_entry(d, v);
                st = 2;
            }
        }
        if (__any(pub)) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (pub) put_flags(d->ready, v);
        if (st >= 0 && st < 2) {
            const uint32_t *f = st == 0 ? d->ready.mine : d->reduced.mine;
            uint32_t got[K];
#pragma unroll
            for (int q = 0; q < K; ++q) got[q] = load_sys(&f[q]);   // all in flight at once
            bool all = true;
#pragma unroll
            for (int q = 0; q < K; ++q) all = all && reached(got[q], v);
            if (all) {
                store_gate(d->ctr + 2 + st, v, d->strict != 0);
                ++st;
            } else if (wall_clock64() - t0 > a.timeout) {
                fail_entry(d, v);
                st = 2;
            }
        }
        if (__all(st == 2)) return;
        __builtin_amdgcn_s_sleep(1);
    }
}

// phase 1, tile `local` of an entry: fold the shard's vectors [local * tv1, +tv1) into
// `out` (the shard in rb, or in the round's own output) and the published shard
// own: this rank's operand read from the snapshot's source instead of rb (nullptr: rb),
// divided by div (fp32 kind 3; 1: as it is) -- the value the snapshot would have stored
template <class Tr, int K>
__device__ __forceinline__ void tile_reduce(const BatchDesc &d, uint32_t local, void *out, const void *own,
                                            float div) {
    using T = typename Tr::T;
    using A = typename Tr::A;
    const uint32_t nvec = uint32_t(d.n / Tr::E);
    const int bytes = int(nvec * 16u);
    __amdgpu_buffer_rsrc_t rs[K];
#pragma unroll
    for (int j = 0; j < K; ++j)
        rs[j] = __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(own && j == int(d.rank) ? own : d.src[j]),
                                                  (short)0, bytes, 0x00020000);
    constexpr bool kF32 = sizeof(T) == 4 && Tr::E == 4 && __is_same(T, float);
    const bool divide = kF32 && own && div != 1.0f;
    const __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(out, (short)0, bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wp = __builtin_amdgcn_make_buffer_rsrc(d.pub, (short)0, bytes, 0x00020000);
    constexpr int U = sizeof(T) == 2 ? 2 : 4;   // vectors per input per lane in flight
    const uint32_t v0 = local * d.tv1;
    for (uint32_t base = v0; base < v0 + d.tv1 && base < nvec; base += 256u * U) {
        const uint32_t i = base + threadIdx.x;
        raw16 r[U][K];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < K; ++j)
                r[u][j] = __builtin_amdgcn_raw_buffer_load_b128(rs[j], (i + u * 256) * 16, 0, 17);
        if (divide) {   // the own operand as the snapshot's kind 3 stores it (__fdiv_rn)
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int j = 0; j < K; ++j)
                    if (j == int(d.rank))
#pragma unroll
                        for (int c = 0; c < 4; ++c)
                            r[u][j][c] = __float_as_uint(__fdiv_rn(__uint_as_float(r[u][j][c]), div));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const raw16 o = fold16<Tr, K, false>(r[u], 1.0f);
            __builtin_amdgcn_raw_buffer_store_b128(o, ws, (i + u * 256) * 16, 0, 17);
            __builtin_amdgcn_raw_buffer_store_b128(o, wp, (i + u * 256) * 16, 0, 17);
        }
    }
    // the ragged tail (elements after the last 16-B vector): tile 0, one element per lane
    if (local == 0 && uint64_t(nvec) * Tr::E + threadIdx.x < d.n) {
        const uint64_t e = uint64_t(nvec) * Tr::E + threadIdx.x;
        A v[K];
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const bool mine = own && j == int(d.rank);
            T x = __hip_atomic_load(static_cast<const T *>(mine ? own : d.src[j]) + e, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_SYSTEM);
            if constexpr (kF32) {
                if (mine && divide) x = __fdiv_rn(x, div);
            }
            v[j] = Tr::load(x);
        }
        tree_fold<Tr, K>(v);
        __hip_atomic_store(static_cast<T *>(out) + e, Tr::store(v[0]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(static_cast<T *>(d.pub) + e, Tr::store(v[0]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// phase 0, tile `local` of an entry's snapshot: 1024 16-B vectors of rb = src (kind 1),
// rb = 0 (kind 2) or rb = src / div (kind 3, fp32: the deep500 op's copy-in with the
// wrapper's division, opt_esgd_solo_imagenet_imbalance.py:40, correctly rounded like
// k_pack<DIV>), write-through; src = the round's own send data or the send bucket; the
// ragged tail in tile 0 (bytes, or 4-B elements for kind 3)
__device__ __forceinline__ void tile_snapshot(const BatchDesc &d, uint32_t local, uint8_t kind, const void *isrc,
                                              float div) {
    const uint32_t nv = d.svec, v0 = local * 1024u;
    const void *src = isrc ? isrc : d.ssrc;
    const __amdgpu_buffer_rsrc_t wd = __builtin_amdgcn_make_buffer_rsrc(d.sdst, (short)0, int(nv * 16u), 0x00020000);
    // a sourced snapshot leaves this rank's own shard out: phase 1 reads src there itself
    const bool skip_own = kind != 2 && src;
    raw16 r[4];
    bool mine[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint32_t vi = v0 + u * 256 + threadIdx.x;
        mine[u] = skip_own && vi >= d.own_v0 && vi < d.own_v1;
    }
    if (kind == 2) {
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = raw16{0u, 0u, 0u, 0u};
    } else {
        const __amdgpu_buffer_rsrc_t rd =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(src), (short)0, int(nv * 16u), 0x00020000);
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (!mine[u]) r[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, (v0 + u * 256 + threadIdx.x) * 16, 0, 2);
        if (kind == 3) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int c = 0; c < 4; ++c) r[u][c] = __float_as_uint(__fdiv_rn(__uint_as_float(r[u][c]), div));
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (!mine[u]) __builtin_amdgcn_raw_buffer_store_b128(r[u], wd, (v0 + u * 256 + threadIdx.x) * 16, 0, 17);
    if (local == 0 && threadIdx.x < d.stail && !(skip_own && d.own_tail)) {
        if (kind == 3) {   // fp32: the tail holds whole elements
            if (threadIdx.x < d.stail / 4) {
                const float x = static_cast<const float *>(src)[size_t(nv) * 4 + threadIdx.x];
                __hip_atomic_store(static_cast<float *>(d.sdst) + size_t(nv) * 4 + threadIdx.x, __fdiv_rn(x, div),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
            uint8_t *dst = static_cast<uint8_t *>(d.sdst) + size_t(nv) * 16;
            const uint8_t b = kind == 1 ? static_cast<const uint8_t *>(src)[size_t(nv) * 16 + threadIdx.x] : uint8_t(0);
            __hip_atomic_store(dst + threadIdx.x, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// phase 2, tile `local` of an entry: tvg[sg] vectors of one peer's published shard, into
// rb or (shift != 0) the same place of the round's own output
__device__ __forceinline__ void tile_gather(const BatchDesc &d, uint32_t local, ptrdiff_t shift) {
    uint32_t sg = 0;
    while (sg < d.nseg && local >= d.t2pre[sg + 1]) ++sg;
    if (sg >= d.nseg) return;   // an entry with nothing to gather (its one dummy tile)
    const uint32_t gv = d.gvec[sg], tv = d.tvg[sg], first = (local - d.t2pre[sg]) * tv;
    const __amdgpu_buffer_rsrc_t gs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(d.gsrc[sg]), (short)0, int(gv * 16u), 0x00020000);
    char *gdst = static_cast<char *>(d.gdst[sg]) + shift;
    const __amdgpu_buffer_rsrc_t gd = __builtin_amdgcn_make_buffer_rsrc(gdst, (short)0, int(gv * 16u), 0x00020000);
    for (uint32_t base = first; base < first + tv && base < gv; base += 1024u) {
        const uint32_t i = base + threadIdx.x;
        raw16 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(gs, (i + u * 256) * 16, 0, 17);
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], gd, (i + u * 256) * 16, 0, 17);
    }
    if (first == 0 && threadIdx.x < d.gtail[sg]) {   // bytes after the last full vector
        const uint8_t *src = static_cast<const uint8_t *>(d.gsrc[sg]) + size_t(gv) * 16;
        uint8_t *dst = reinterpret_cast<uint8_t *>(gdst) + size_t(gv) * 16;
        __hip_atomic_store(dst + threadIdx.x,
                           __hip_atomic_load(src + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

template <class Tr, int K>
__global__ __launch_bounds__(256) void k_round_batch(BatchArgs a) {
    const long long t0 = wall_clock64();
    if (blockIdx.x == 0) {   // dispatched first: the agent never waits for a free slot
        if (threadIdx.x < 64) agent<K>(a, t0);
        return;
    }
    // stale peer lines of earlier launches out of this CU's L1 and this XCD's L2 (a worker
    // that starts late still does this before its first tile)
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const uint32_t workers = gridDim.x - 1;
    // the tile list: every entry's snapshot tiles (phase 0), its phase-1 tiles, its phase-2
    // tiles, each in ring order; a worker meets no gate before its snapshot tiles are done
    const uint32_t T0 = a.tile0[a.nent], T1 = T0 + a.tile1[a.nent], T = T0 + a.tile1[a.nent] + a.tile2[a.nent];
    __shared__ uint32_t s_next;
    uint32_t e = 0;
    int phase = 0;
    for (uint32_t g = blockIdx.x - 1;; g += workers) {
        if (a.dynamic) {   // the next tile of the list, whichever worker is free (BatchArgs)
            if (threadIdx.x == 0)
                s_next = __hip_atomic_fetch_add(a.queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a.qbase;
            __syncthreads();
            g = s_next;   // read by every thread before the next write (a barrier follows in each path)
        }
        if (g >= T) break;
        const int ph = g < T0 ? 0 : g < T1 ? 1 : 2;
        if (ph != phase) { phase = ph; e = 0; }
        const uint32_t t = ph == 0 ? g : ph == 1 ? g - T0 : g - T1;
        const uint32_t *pre = ph == 0 ? a.tile0 : ph == 1 ? a.tile1 : a.tile2;
        while (t >= pre[e + 1]) ++e;
        const BatchDesc &d = a.table[a.sid[e]];
        const uint32_t v = a.value[e];
        if (ph == 0) {
            tile_snapshot(d, t - pre[e], a.snap[e], a.isrc[e], a.idiv[e]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are in memory
            __syncthreads();
            if (threadIdx.x == 0) {
                if (d.strict) __hip_atomic_fetch_add(d.ctr + 4, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
                else __hip_atomic_fetch_add(d.ctr + 4, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            continue;
        }
        const bool gather = ph == 2;
        if (threadIdx.x == 0) {
            const uint32_t *gate = d.ctr + (gather ? 3 : 2);
            while (!reached(__hip_atomic_load(const_cast<uint32_t *>(gate), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                            v)) {
                if (wall_clock64() - t0 > 2 * a.timeout) break;   // the agent's timeout comes first
                __builtin_amdgcn_s_sleep(1);
            }
            if (d.strict) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        }
        __syncthreads();
        const uint32_t local = t - pre[e];
        // a round with its own output (esgd_schedule_post_io) lands there, at rb's offsets
        const ptrdiff_t shift = a.iout[e] ? static_cast<char *>(a.iout[e]) - static_cast<char *>(d.rbase) : 0;
        // a sourced in-launch snapshot skipped the own shard: its operand comes from the source
        const uint8_t kind = a.snap[e];
        const void *ssrc = a.isrc[e] ? a.isrc[e] : d.ssrc;
        const void *own = (kind == 1 || kind == 3) && ssrc ? static_cast<const char *>(ssrc) + d.own_off : nullptr;
        if (!gather) tile_reduce<Tr, K>(d, local, static_cast<char *>(d.out) + shift, own, kind == 3 ? a.idiv[e] : 1.0f);
        else tile_gather(d, local, shift);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores are in memory
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t *cnt = d.ctr + (gather ? 1 : 0);
            const uint32_t need = pre[e + 1] - pre[e];
            const uint32_t old = d.strict ? __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                                          : __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old + 1 == need) {   // the entry's last tile of this phase
                __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (!gather) {
                    // every tile of the entry was stored write-through and drained before
                    // its count: no L2 write-back before the flag (strict: one anyway)
                    if (d.strict) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    put_flags(d.reduced, v);
                } else {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    store_sys(d.fin, v);
                }
            }
        }
        __syncthreads();
    }
}

// workgroups of k_round_batch<Tr, K> resident on the whole GPU at once
template <class Tr>
static int capacity_t(int world) {
    int nb = 0;
    hipError_t e = hipErrorInvalidValue;
    switch (world) {
#define ESGD_BATCH_OCC(KK) \
    case KK: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_round_batch<Tr, KK>, 256, 0); break;
    ESGD_BATCH_OCC(2) ESGD_BATCH_OCC(3) ESGD_BATCH_OCC(4) ESGD_BATCH_OCC(5) ESGD_BATCH_OCC(6) ESGD_BATCH_OCC(7)
    ESGD_BATCH_OCC(8)
#undef ESGD_BATCH_OCC
    default: break;
    }
    if (e != hipSuccess || nb <= 0) {
        (void)hipGetLastError();
        nb = 1;
    }
    return nb * cu_count();
}

// cached per (dtype, world); 0 for a dtype or world the kernel does not take (the caller
// fails the flush: a silent single worker once made every bf16 round 10-20x slower)
int round_batch_capacity(int dtype, int world) {
    static std::atomic<int> cache[5][ESGD_MAX_FANIN + 1] = {};
    if (world < 2 || world > ESGD_MAX_FANIN) return 0;
    int slot = -1;
    switch (dtype) {   // dtype codes are not dense (ESGD_BF16 = 16)
    case ESGD_FLOAT: slot = 0; break;
    case ESGD_BF16: slot = 1; break;
    case ESGD_DOUBLE: slot = 2; break;
    case ESGD_INT32: slot = 3; break;
    case ESGD_INT64: slot = 4; break;
    default: return 0;
    }
    int c = cache[slot][world].load(std::memory_order_relaxed);
    if (!c) {
        switch (slot) {
        case 0: c = capacity_t<F32>(world); break;
        case 1: c = capacity_t<BF16>(world); break;
        case 2: c = capacity_t<F64>(world); break;
        case 3: c = capacity_t<I32>(world); break;
        default: c = capacity_t<I64>(world); break;
        }
        cache[slot][world].store(c, std::memory_order_relaxed);
    }
    return c;
}

// The shared launch's snapshots: tile g (1024 16-B vectors of one segment) on block
// g mod grid; nt loads, write-through stores (peers read these buckets over xGMI once
// the kernel boundary and the agent's ready have passed); ragged tails byte by byte.
__global__ __launch_bounds__(256) void k_copy_many(CopySet c) {
    const uint32_t total = c.tile0[c.nseg];
    int i = 0;
    for (uint32_t g = blockIdx.x; g < total; g += gridDim.x) {
        while (g >= c.tile0[i + 1]) ++i;
        const uint32_t nv = c.nvec[i];
        const uint32_t v0 = (g - c.tile0[i]) * 1024u;
        const __amdgpu_buffer_rsrc_t wd = __builtin_amdgcn_make_buffer_rsrc(c.dst[i], (short)0, int(nv * 16u), 0x00020000);
        raw16 r[4];
        if (c.src[i]) {
            const __amdgpu_buffer_rsrc_t rd =
                __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(c.src[i]), (short)0, int(nv * 16u), 0x00020000);
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = __builtin_amdgcn_raw_buffer_load_b128(rd, (v0 + u * 256 + threadIdx.x) * 16, 0, 2);
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) r[u] = raw16{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) __builtin_amdgcn_raw_buffer_store_b128(r[u], wd, (v0 + u * 256 + threadIdx.x) * 16, 0, 17);
        if (v0 == 0 && threadIdx.x < c.tail[i]) {
            uint8_t *d = static_cast<uint8_t *>(c.dst[i]) + size_t(nv) * 16;
            const uint8_t *src = static_cast<const uint8_t *>(c.src[i]);
            d[threadIdx.x] = src ? src[size_t(nv) * 16 + threadIdx.x] : uint8_t(0);
        }
    }
}

int copy_many(const CopySet &c, hipStream_t s) {
    ESGD_ARG(c.nseg >= 1 && c.nseg <= kBatchMax, "copy_many: %d segments", c.nseg);
    const uint32_t total = c.tile0[c.nseg];
    if (!total) return ESGD_SUCCESS;
    const unsigned grid = std::min<unsigned>(total, unsigned(cu_count()) * 4u);
    hipLaunchKernelGGL(k_copy_many, dim3(grid), dim3(256), 0, s, c);
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

template <class Tr>
static int launch_batch_t(int world, const BatchArgs &a, unsigned grid, hipStream_t s) {
    switch (world) {
#define ESGD_BATCH_K(KK) \
    case KK: hipLaunchKernelGGL((k_round_batch<Tr, KK>), dim3(grid), dim3(256), 0, s, a); break;
    ESGD_BATCH_K(2) ESGD_BATCH_K(3) ESGD_BATCH_K(4) ESGD_BATCH_K(5) ESGD_BATCH_K(6) ESGD_BATCH_K(7)
    ESGD_BATCH_K(8)
#undef ESGD_BATCH_K
    default:
        set_error("batched rounds: %d ranks outside [2, %d]", world, ESGD_MAX_FANIN);
        return ESGD_INVALID_ARG;
    }
    ESGD_HIP(hipGetLastError());
    return ESGD_SUCCESS;
}

int round_batch(int dtype, int world, const BatchArgs &a, unsigned workers, hipStream_t s) {
    ESGD_ARG(a.nent >= 1 && a.nent <= uint32_t(kBatchMax) && a.table && workers >= 1 && workers <= kBatchWorkersMax,
             "batched rounds: %u entries, %u workers", a.nent, workers);
    const unsigned grid = workers + 1;
    switch (dtype) {
    case ESGD_FLOAT: return launch_batch_t<F32>(world, a, grid, s);
    case ESGD_BF16: return launch_batch_t<BF16>(world, a, grid, s);
    case ESGD_DOUBLE: return launch_batch_t<F64>(world, a, grid, s);
    case ESGD_INT32: return launch_batch_t<I32>(world, a, grid, s);
    case ESGD_INT64: return launch_batch_t<I64>(world, a, grid, s);
    default: break;
    }
    set_error("batched rounds: unsupported dtype %d", dtype);
    return ESGD_INVALID_ARG;
}

}  // namespace esgd
