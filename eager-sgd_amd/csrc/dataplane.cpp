// dataplane.cpp — how a round's bytes move between the ranks of one node.
//
// IpcTransport (the GPU data plane).  fflib2 sends the whole receive buffer to one
// partner per round, log2(P) rounds (src/colls/ffallreduce.c:138-171).  On an MI355X
// node every GPU pair has its own xGMI link, so instead every rank owns one shard of
// the bucket and, in two launches,
//   phase 1 (reduce-scatter): reads its shard from all P ranks' rb (peer HBM mapped
//            through IPC) and folds it with the tree kernel in exactly the reference's
//            hypercube order -> writes the shard into its own rb;
//   phase 2 (all-gather):    reads every other rank's reduced shard into its own rb.
// Each rank only ever WRITES its own HBM; remote bytes are only READ, with system-scope
// loads.  That keeps every device's L2 coherent without relying on remote writes
// invalidating lines (they do not on gfx950).  Per link and direction each phase moves
// S/P bytes: the 2S/(P * link) lower bound of SURVEY.md §8d.
//
// NullTransport: moves nothing.  It exists only so that the control plane (activation,
// limiter, majority draw, round protocol) can be exercised by multi-process CPU tests;
// it is reachable only through ESGD_BUF_NONE and computes nothing.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "esgd_internal.h"
#include "esgd.h"
#include "round_batch.h"

namespace esgd {

int reduce_remote(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                  float scale, hipStream_t s);
// max_blocks (0: sized for HBM): a cap for copies that run beside the round's kernels
int gather_remote(int n, const void *const *src, void *const *dst, const uint64_t *bytes,
                  hipStream_t s, unsigned max_blocks = 0);
int move_zero(void *dst, void *src, uint64_t bytes, hipStream_t s);

int narrow_bf16(float *src, uint16_t *dst, uint64_t n, bool zero_src, hipStream_t s);
int reduce_wire(int k, const void *const *inputs, uint16_t *outb, float *outf, uint64_t count, hipStream_t s);
int gather_widen(int n, const void *const *src, void *const *dst, const uint64_t *count, hipStream_t s);
int store_fin(uint32_t *fin, uint32_t value, hipStream_t s);

int round_small(int dtype, const void *const *src, void *out, void *pub, uint64_t n, int nseg,
                const void *const *gsrc, void *const *gdst, const uint64_t *gbytes,
                const PairFlags &ready, const PairFlags &reduced, uint32_t *fin, uint32_t *err,
                uint64_t *ts, uint32_t *counter, int rank, int world, uint32_t value,
                long long timeout_ticks, int strict, hipStream_t s);

constexpr int kMaxSegs = 16;                      // segments per gather launch (kMaxSeg)

// Bytes per input / segment of one remote launch: 64 MiB, the local tree kernel's window
// (reduce_kernels.hip kWindowBytes; in the shared-GPU rehearsal 64 MiB pieces took C5's
// 256 MiB - 1 GiB rounds 2-7 % faster than 1 GiB ones), at most 1 GiB (the kernels
// address a shard through 32-bit buffer offsets).  The tests drive the piecewise path with
// small pieces (ESGD_TEST piece_bytes, a multiple of 1 KiB).
static uint64_t piece_bytes() {
    static const uint64_t v = [] {
        const uint64_t b = uint64_t(std::max<int64_t>(0, test_knob("piece_bytes", int64_t(64) << 20)));
        return std::max<uint64_t>(1024, std::min<uint64_t>(b, uint64_t(1) << 30) / 1024 * 1024);
    }();
    return v;
}

// Buckets up to this many bytes run as one launch per round (k_round_small);
// ESGD_SMALL_ROUND_BYTES overrides (0 = never).
static uint64_t small_round_bytes() {
    static const uint64_t v = [] {
        const char *e = getenv("ESGD_SMALL_ROUND_BYTES");
        return (e && *e) ? uint64_t(strtoull(e, nullptr, 10)) : (uint64_t(4) << 20);
    }();
    return v;
}

// ESGD_STRICT_HANDOFFS=1: one-launch rounds use acq_rel arrival counts, agent-scope
// release gates and an L2 write-back before the reduced flag (round 2's hand-offs) instead
// of the relaxed ones (memory ordering); a cross-GPU A/B.
static int strict_env() {
    static const int v = getenv("ESGD_STRICT_HANDOFFS") && *getenv("ESGD_STRICT_HANDOFFS") == '1' ? 1 : 0;
    return v;
}

// Where the rank-pairing flags live (dataplane.cpp, "device pairing flags"): 0 host
// memory (default), 1 uncached HBM, 2 fine-grained HBM; ESGD_DEVICE_FLAGS overrides.
static int device_flags_env() {
    static const int m = getenv("ESGD_DEVICE_FLAGS") ? atoi(getenv("ESGD_DEVICE_FLAGS")) : 0;
    return m;
}

// esgd_set_config: what schedules created afterwards capture (-1 = the env default).
// All ranks must set the same values before the same creations (the creation signature
// checks it), so a benchmark can A/B them inside one job.
static std::atomic<int64_t> g_cfg_small{-1}, g_cfg_flags{-1}, g_cfg_strict{-1}, g_cfg_batch{-1};
// "batch_hold" (diagnostics / tests): 1 = the end of a pump never sends the pending shared
// launch; only an explicit flush (another launch on the round stream, schedule deletion,
// finalize) does -- so a test can finalize with rounds held
static std::atomic<int64_t> g_cfg_hold{0};
// "batch_workers_max" (ESGD_BATCH_WORKERS, default 64): a shared launch's worker cap, and the
// phase tiles per entry of schedules whose first batched round comes after the setting
static std::atomic<int64_t> g_cfg_workers{-1};
// "snapshot_workers_max" (ESGD_SNAPSHOT_WORKERS, default kSnapshotWorkers = 256; 0 = as
// batch_workers_max): the worker cap of a shared launch that holds phase-0 snapshot tiles
// (rounds posted with their own data, separate send buckets).  A snapshot is a plain copy: it
// wants waves, where the gated phases want few spinning workgroups (r05ac, ranks sharing one
// GPU: the optimizer's per-tensor step 1.44 -> 1.35 ms at P = 2, 2.20 -> 1.93 at P = 4, with
// 256 against 64); process-local, read at each flush
static std::atomic<int64_t> g_cfg_snapw{-1};

// One-launch rounds due together in issue order share one launch of at most this many
// rounds (k_round_batch, round_batch.hip; default kBatchMax); 0 or 1 = one k_round_small
// launch per round (esgd_set_config("batch_rounds")).  A process-local setting, not part of
// the creation signature: ranks may cut the issue ring into launches differently anyway.
static int64_t batch_rounds() {
    const int64_t v = g_cfg_batch.load();
    return std::min<int64_t>(kBatchMax, v >= 0 ? v : int64_t(kBatchMax));
}

bool config_strict_handoffs() {
    const int64_t v = g_cfg_strict.load();
    return v >= 0 ? v != 0 : strict_env() != 0;
}

// round kernels launched by this process (k_round_small and k_round_batch launches, and
// five-launch rounds' first pairing): esgd_get_config("launches"), for the bench's
// per-step breakdown
static std::atomic<uint64_t> g_launches{0};
// worker workgroups of the last shared launch: esgd_get_config("batch_workers"), so a test
// can see that the grid is sized by the residency figure and not a fallback
static std::atomic<int64_t> g_batch_workers{0};

uint64_t config_small_round_bytes() {
    const int64_t v = g_cfg_small.load();
    return v >= 0 ? uint64_t(v) : small_round_bytes();
}

int config_device_flags() {
    const int64_t v = g_cfg_flags.load();
    const int m = v >= 0 ? int(v) : device_flags_env();
    return (m >= 0 && m <= 2) ? m : 0;
}

int config_set(const char *key, int64_t value) {
    ESGD_ARG(key, "esgd_set_config: null key");
    if (!std::strcmp(key, "small_round_bytes")) {
        ESGD_ARG(value >= -1, "small_round_bytes: >= 0 (or -1: the default)");
        g_cfg_small.store(value);
    } else if (!std::strcmp(key, "device_flags")) {
        ESGD_ARG(value >= -1 && value <= 2, "device_flags: 0 host, 1 uncached HBM, 2 fine-grained HBM (-1: the default)");
        g_cfg_flags.store(value);
    } else if (!std::strcmp(key, "strict_handoffs")) {
        ESGD_ARG(value >= -1 && value <= 1, "strict_handoffs: 0 relaxed, 1 strict (-1: the default)");
        g_cfg_strict.store(value);
    } else if (!std::strcmp(key, "batch_rounds")) {
        ESGD_ARG(value >= -1 && value <= kBatchMax, "batch_rounds: 0..%d rounds per launch (-1: the default)",
                 kBatchMax);
        g_cfg_batch.store(value);
    } else if (!std::strcmp(key, "batch_hold")) {
        ESGD_ARG(value >= -1 && value <= 1, "batch_hold: 0 or 1 (-1: the default, 0)");
        g_cfg_hold.store(value < 0 ? 0 : value);
    } else if (!std::strcmp(key, "batch_workers_max")) {
        ESGD_ARG(value == -1 || (value >= 1 && value <= int64_t(kBatchWorkersMax)),
                 "batch_workers_max: 1..%u (-1: the default)", kBatchWorkersMax);
        g_cfg_workers.store(value);
    } else if (!std::strcmp(key, "snapshot_workers_max")) {
        ESGD_ARG(value >= -1 && value <= int64_t(kBatchWorkersMax),
                 "snapshot_workers_max: 0..%u (0: batch_workers_max; -1: the default)", kBatchWorkersMax);
        g_cfg_snapw.store(value);
    } else {
        set_error("esgd_set_config: unknown key '%s' (small_round_bytes, device_flags, strict_handoffs, "
                  "batch_rounds, batch_hold, batch_workers_max, snapshot_workers_max)", key);
        return ESGD_INVALID_ARG;
    }
    return ESGD_SUCCESS;
}

static uint32_t snapshot_workers_max();

int config_get(const char *key, int64_t *value) {
    ESGD_ARG(key && value, "esgd_get_config: null argument");
    if (!std::strcmp(key, "small_round_bytes")) *value = int64_t(config_small_round_bytes());
    else if (!std::strcmp(key, "device_flags")) *value = config_device_flags();
    else if (!std::strcmp(key, "strict_handoffs")) *value = config_strict_handoffs() ? 1 : 0;
    else if (!std::strcmp(key, "batch_rounds")) *value = batch_rounds();
    else if (!std::strcmp(key, "launches")) *value = int64_t(g_launches.load());
    else if (!std::strcmp(key, "batch_workers")) *value = g_batch_workers.load();
    else if (!std::strcmp(key, "batch_hold")) *value = g_cfg_hold.load();
    else if (!std::strcmp(key, "batch_workers_max")) *value = int64_t(batch_workers_max());
    else if (!std::strcmp(key, "snapshot_workers_max")) *value = int64_t(snapshot_workers_max());
    else {
        set_error("esgd_get_config: unknown key '%s' (small_round_bytes, device_flags, strict_handoffs, "
                  "batch_rounds, launches, batch_workers, batch_hold, batch_workers_max, snapshot_workers_max)", key);
        return ESGD_INVALID_ARG;
    }
    return ESGD_SUCCESS;
}

// ---- IPC mapping cache: one hipIpcOpenMemHandle per (peer, arena chunk) ----
// Every exported bucket lives in an arena chunk that is never freed while the process
// runs (arena.cpp), so handle bytes never repeat and a mapping, once open, stays valid:
// mappings are kept until the data plane shuts down, whatever schedules come and go.
// (Closing mappings and letting exporters free and re-export the memory was the source
// of round 1's illegal accesses and of wrong sums at 8 ranks; arena.cpp.)
struct IpcKey {
    int peer;
    uint8_t h[64];
    bool operator<(const IpcKey &o) const {
        if (peer != o.peer) return peer < o.peer;
        return std::memcmp(h, o.h, 64) < 0;
    }
};
static std::mutex g_ipc_mu;
static std::map<IpcKey, void *> g_ipc;
// set by ipc_open when a fresh mapping's seal did not match (the caller asks the exporter to
// move: SchedShm::remap); per thread, read right after the call
static thread_local bool t_seal_mismatch = false;

// ESGD_TEST fail_maps=N: this process's first N sealed mappings are treated as showing
// other memory, so the re-publish-and-remap retry of schedule creation runs anywhere
static bool simulated_map_failure() {
    static std::atomic<int> left{int(std::max<int64_t>(0, test_knob("fail_maps", 0)))};
    int n = left.load();
    while (n > 0 && !left.compare_exchange_weak(n, n - 1)) {
    }
    return n > 0;
}

// Map a peer's exported chunk (once per (peer, chunk)).  `slot` (may be null: flag pages)
// carries the chunk's seal: a fresh mapping is only kept if the seal read through it is
// the exporter's -- a mapping that shows other memory fails the creation loudly instead
// of feeding another process's bytes into the sums.
static int ipc_open(int peer, const uint8_t *h, void **base, const IpcSlot *slot = nullptr) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    t_seal_mismatch = false;
    IpcKey k;
    k.peer = peer;
    std::memcpy(k.h, h, 64);
    auto it = g_ipc.find(k);
    if (it != g_ipc.end()) {
        *base = it->second;
        return ESGD_SUCCESS;
    }
    hipIpcMemHandle_t hh;
    std::memcpy(&hh, h, sizeof(hh));
    void *p = nullptr;
    ESGD_HIP(hipIpcOpenMemHandle(&p, hh, hipIpcMemLazyEnablePeerAccess));
    if (slot && slot->seal_nonce) {
        ChunkSeal got;
        uint64_t w[4];
        if (int rc = seal_read(static_cast<char *>(p) + slot->chunk_bytes, w)) return rc;
        std::memcpy(&got, w, sizeof(got));
        const bool simulated = simulated_map_failure();
        if (simulated)
            std::fprintf(stderr, "esgd: pid %d: mapping of rank %d's chunk %#llx treated as showing other memory "
                         "(ESGD_TEST fail_maps)\n", int(getpid()), peer, (unsigned long long)slot->chunk_base);
        if (simulated || got.magic != kSealMagic || got.nonce != slot->seal_nonce || got.base != slot->chunk_base) {
            t_seal_mismatch = true;
            if (!simulated)
                std::fprintf(stderr, "esgd: pid %d: rank %d's chunk %#llx (%llu B) mapped at %p shows other memory: seal "
                         "magic %#llx base %#llx nonce %#llx pid %u, expected base %#llx nonce %#llx\n", int(getpid()),
                         peer, (unsigned long long)slot->chunk_base, (unsigned long long)slot->chunk_bytes, p,
                         (unsigned long long)got.magic, (unsigned long long)got.base, (unsigned long long)got.nonce,
                         got.pid, (unsigned long long)slot->chunk_base, (unsigned long long)slot->seal_nonce);
            set_error("the runtime mapped rank %d's exported chunk to other memory (its seal does not match; "
                      "DESIGN.md §5)", peer);
            return ESGD_ERROR;   // not cached; the mapping is left open (closing is unsafe)
        }
    }
    g_ipc[k] = p;
    *base = p;
    return ESGD_SUCCESS;
}

// every mapping, at data-plane shutdown (after the last round has drained).  Once a
// mapping has been closed, this process must not start another multi-process job: its
// peers' arena chunks keep their handles, and re-opening handle bytes that were opened
// and closed before is the illegal-access trigger of DESIGN.md §5 (engine_init refuses).
static bool g_mappings_closed = false;

static void ipc_close_all() {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto &kv : g_ipc) {
        hip_ignore(hipIpcCloseMemHandle(kv.second));
    }
    if (!g_ipc.empty()) g_mappings_closed = true;
    g_ipc.clear();
}

// ESGD_TEST arena_bypass=2 (diagnostics only): besides the arena bypass (arena.cpp), a
// schedule's teardown closes the peer mappings it opened -- round 2's pre-arena lifetime,
// where deletion was local and every rank closed its peers' buckets.
static bool close_on_delete() {
    static const bool b = test_knob("arena_bypass", 0) == 2;
    return b;
}

static void ipc_close_one(int peer, const uint8_t *h) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    IpcKey k;
    k.peer = peer;
    std::memcpy(k.h, h, 64);
    auto it = g_ipc.find(k);
    if (it == g_ipc.end()) return;
    hip_ignore(hipIpcCloseMemHandle(it->second));
    g_ipc.erase(it);
}

bool dataplane_mappings_closed() {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    return g_mappings_closed;
}

// ---- process-wide data-plane resources -----------------------------------------------
// One round stream per process: every round of every schedule is queued on it in the
// node's issue order (engine.cpp), so no GPU-side wait of one round can sit in front of
// a round a peer needs first.  The node segment is registered with the GPU once: the
// rounds' pairing flags live in it (SchedShm::ready/reduced/done/gpu_err).
static std::mutex g_dp_mu;
static hipStream_t g_rs = nullptr;
static Segment *g_seg_reg = nullptr;
static char *g_seg_dev = nullptr;
static long long g_ticks_per_s = 0;

static int round_stream(hipStream_t *out) {
    std::lock_guard<std::mutex> lk(g_dp_mu);
    if (!g_rs) ESGD_HIP(hipStreamCreateWithFlags(&g_rs, hipStreamNonBlocking));
    *out = g_rs;
    return ESGD_SUCCESS;
}

// The arena seal's kernels (reduce_kernels.hip) run on the round stream, synchronously, at
// an export or a first mapping -- never on a stream of their own (one more hardware queue
// per process slowed shared-GPU rounds 1.7x).  Waiting for the round stream
// cannot deadlock: every rank launches rounds in the node's one issue order, so the
// earliest round in flight anywhere has been launched by every rank and completes.
int seal_stream(hipStream_t *out) { return round_stream(out); }


// Copy streams of the chunked host-bucket rounds (one per direction, so a chunk's D2H
// runs while the next chunk's H2D does: PCIe is full duplex).  Created on first use.
static hipStream_t g_h2d = nullptr, g_d2h = nullptr;

static int copy_streams(hipStream_t *h2d, hipStream_t *d2h) {
    std::lock_guard<std::mutex> lk(g_dp_mu);
    if (!g_h2d) ESGD_HIP(hipStreamCreateWithFlags(&g_h2d, hipStreamNonBlocking));
    if (!g_d2h) ESGD_HIP(hipStreamCreateWithFlags(&g_d2h, hipStreamNonBlocking));
    *h2d = g_h2d;
    *d2h = g_d2h;
    return ESGD_SUCCESS;
}

// Host buckets of at least two chunks of this many bytes run chunked rounds (16 MiB; the
// tests drive it with small chunks: ESGD_TEST host_chunk_bytes, 0 = never).
static uint64_t host_chunk_bytes() {
    static const uint64_t v = [] {
        const uint64_t b = uint64_t(std::max<int64_t>(0, test_knob("host_chunk_bytes", int64_t(16) << 20)));
        return b ? std::max<uint64_t>(16384, b / 1024 * 1024) : 0;
    }();
    return v;
}

static int register_segment() {
    std::lock_guard<std::mutex> lk(g_dp_mu);
    Segment *seg = engine_segment();
    if (g_seg_reg == seg) return ESGD_SUCCESS;
    ESGD_HIP(hipHostRegister(seg, sizeof(Segment), hipHostRegisterMapped));
    void *d = nullptr;
    ESGD_HIP(hipHostGetDevicePointer(&d, seg, 0));
    int dev = 0, khz = 0;
    ESGD_HIP(hipGetDevice(&dev));
    ESGD_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    g_ticks_per_s = (long long)khz * 1000;
    g_seg_reg = seg;
    g_seg_dev = static_cast<char *>(d);
    return ESGD_SUCCESS;
}

template <class T>
static uint32_t *dev_flag(T *host) {
    return reinterpret_cast<uint32_t *>(g_seg_dev + (reinterpret_cast<char *>(host) -
                                                     reinterpret_cast<char *>(g_seg_reg)));
}

// the device address of pinned host memory (nullptr: not mapped, use DMA copies)
static void *host_view(void *host) {
    void *d = nullptr;
    if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return d;
}

// errs: every rank's error word (the node segment); after_fail: a pairing after the round's
// first publishes nothing once this rank's error word holds the round (failure contract)
int round_sync(const PairFlags &f, int world, int rank, uint32_t value, long long timeout_ticks,
               uint32_t *errs, uint32_t errval, uint32_t *failw, bool after_fail, uint64_t *ts, bool drop_peer_lines,
               uint32_t *fin, hipStream_t s);

// ---- device pairing flags (schedules with flag_mode 1 or 2, opt-in) ----
// Each rank owns a page of HBM per mode -- uncached (hipDeviceMallocUncached: loads and
// stores go to memory, no cache holds a flag) or fine-grained -- with one word per
// (schedule, pairing, peer); a rank publishes a round by storing it in its word of EVERY
// rank's page (peers' pages are IPC-mapped, stores cross xGMI) and polls its own page --
// no PCIe round trip to host memory.  Opt-in: cross-GPU visibility of these stores has
// only been exercised with the ranks sharing one GPU.  A page, like every
// exported buffer, is never freed while the process runs; it is zeroed for every new job.
constexpr size_t kPageWords = size_t(kMaxSched) * 3 * kMaxRanks;
struct FlagPages {
    uint32_t *page = nullptr;                 // this rank's page
    Segment *seg = nullptr;                   // the job it was published for
    uint32_t *peer[kMaxRanks] = {};           // every rank's page (own included)
    bool mapped = false;
};
static FlagPages g_pages[3];                  // [mode]; [0] unused (host flags)

static int flags_publish(int rank, int mode) {
    std::lock_guard<std::mutex> lk(g_dp_mu);
    FlagPages &fp = g_pages[mode];
    Segment *seg = engine_segment();
    if (fp.seg == seg) return ESGD_SUCCESS;
    if (!fp.page)
        ESGD_HIP(hipExtMallocWithFlags(reinterpret_cast<void **>(&fp.page), kPageWords * sizeof(uint32_t),
                                       mode == 2 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
    // the null stream: rounds run on non-blocking streams, nothing in flight is waited for
    ESGD_HIP(hipMemsetAsync(fp.page, 0, kPageWords * sizeof(uint32_t), nullptr));
    ESGD_HIP(hipStreamSynchronize(nullptr));
    hipIpcMemHandle_t h;
    ESGD_HIP(hipIpcGetMemHandle(&h, fp.page));
    IpcSlot &mine = seg->flagpage[mode - 1][rank];
    std::memcpy(mine.handle, &h, 64);
    mine.seal_nonce = 0;   // not arena memory: no seal
    mine.offset = 0;
    mine.bytes = kPageWords * sizeof(uint32_t);
    mine.gen.store(1, std::memory_order_release);
    fp.seg = seg;
    fp.mapped = false;
    return ESGD_SUCCESS;
}

// after the creation vote: every peer has published its page
static int flags_connect(int rank, int world, int mode) {
    std::lock_guard<std::mutex> lk(g_dp_mu);
    FlagPages &fp = g_pages[mode];
    if (fp.mapped) return ESGD_SUCCESS;
    Segment *seg = engine_segment();
    for (int q = 0; q < world; ++q) {
        if (q == rank) { fp.peer[q] = fp.page; continue; }
        if (seg->flagpage[mode - 1][q].gen.load(std::memory_order_acquire) != 1) {
            set_error("device flags: rank %d did not publish its mode-%d flag page (every rank must create "
                      "the schedule with the same device_flags setting)", q, mode);
            return ESGD_ERROR;
        }
        void *p = nullptr;
        if (int rc = ipc_open(q, seg->flagpage[mode - 1][q].handle, &p)) return rc;
        fp.peer[q] = static_cast<uint32_t *>(p);
    }
    fp.mapped = true;
    return ESGD_SUCCESS;
}

// the flags of pairing `which` (0 ready, 1 reduced, 2 done) of schedule s
static PairFlags pair_flags(Sched &s, std::atomic<uint32_t> *host, int which) {
    PairFlags f{};
    if (s.flag_mode > 0) {
        const FlagPages &fp = g_pages[s.flag_mode];
        const size_t base = (size_t(s.id) * 3 + size_t(which)) * kMaxRanks;
        f.mine = fp.page + base;
        for (int q = 0; q < s.world; ++q) f.dst[q] = fp.peer[q] + base + s.rank;
        f.ndst = s.world;
    } else {
        f.mine = dev_flag(host);
        f.dst[0] = dev_flag(&host[s.rank]);
        f.ndst = 1;
    }
    return f;
}

static bool gpu_trace_on() {
    static const bool on = getenv("ESGD_GPU_TRACE") && *getenv("ESGD_GPU_TRACE") == '1';
    return on;
}

static int ctr_words(int sched_id, hipStream_t cs, uint32_t **out);

// which = 0 ready, 1 reduced, 2 done; `value` is the round, or the chunk number of a
// chunked round (a timeout still records the round)
// fin: the pairing is the round's last kernel and stores the round there when it is done
static int pair_ranks(Sched &s, std::atomic<uint32_t> *flags, int which, uint32_t round, hipStream_t cs,
                      uint32_t value = 0, std::atomic<uint32_t> *fin = nullptr) {
    const long long ticks = (long long)(engine_timeout() * double(g_ticks_per_s));
    uint64_t *ts = gpu_trace_on() ? reinterpret_cast<uint64_t *>(dev_flag(&s.sh->gpu_ts[s.rank][2 * which]))
                                  : nullptr;
    // the ready and reduced pairings are followed by a phase that reads peer buckets: a
    // kernel behind each drops stale peer lines from every XCD's caches
    uint32_t *ctr = nullptr;
    if (int rc = ctr_words(s.id, cs, &ctr)) return rc;
    // word 12: the round whose pairing failed here (the later pairings then publish nothing)
    return round_sync(pair_flags(s, flags, which), s.world, s.rank, value ? value : round, ticks,
                      dev_flag(&s.sh->gpu_err[0]), round, ctr + 12, which > 0, ts, which < 2,
                      fin ? dev_flag(fin) : nullptr, cs);
}

// ns between the GPU stamps of the last round (ESGD_GPU_TRACE=1), for the timeline
void gpu_trace_read(Sched &s, uint64_t out[6]) {
    for (int k = 0; k < 6; ++k) out[k] = 0;
    if (!gpu_trace_on() || !g_ticks_per_s || s.world < 2) return;
    volatile uint64_t *t = s.sh->gpu_ts[s.rank];
    const double ns = 1e9 / double(g_ticks_per_s);
    // sync1 wait, RS, sync2 wait, AG, sync3 wait, total
    out[0] = uint64_t(double(t[1] - t[0]) * ns);
    out[1] = uint64_t(double(t[2] - t[1]) * ns);
    out[2] = uint64_t(double(t[3] - t[2]) * ns);
    out[3] = uint64_t(double(t[4] - t[3]) * ns);
    out[4] = uint64_t(double(t[5] - t[4]) * ns);
    out[5] = uint64_t(double(t[5] - t[0]) * ns);
}

void rccl_shutdown();

// Per-schedule device words -- k_round_small's two arrival counters and two gates
// ([0..3]), two unused ([4], [5]: the five-launch round's cache-maintenance gates until
// round 6), the batched rounds' words ([6..11], BatchDesc::ctr) and the five-launch
// round's failed round ([12]) -- one
// allocation for the process: a hipMalloc per schedule, on the round path, is avoided
// (host-side memory operations were seen to slow later peer-reading kernels).
static uint32_t *g_ctr_pool = nullptr;
constexpr int kCtrWords = 16;   // per schedule (64 B)

static int ctr_words(int sched_id, hipStream_t cs, uint32_t **out) {
    std::lock_guard<std::mutex> lk(g_dp_mu);
    if (!g_ctr_pool) {
        const size_t bytes = size_t(kMaxSched) * kCtrWords * sizeof(uint32_t);
        ESGD_HIP(hipMalloc(reinterpret_cast<void **>(&g_ctr_pool), bytes));
        ESGD_HIP(hipMemsetAsync(g_ctr_pool, 0, bytes, cs));
    }
    *out = g_ctr_pool + size_t(sched_id) * kCtrWords;
    return ESGD_SUCCESS;
}

static void batch_shutdown();

void dataplane_shutdown() {
    batch_shutdown();
    rccl_shutdown();
    std::lock_guard<std::mutex> lk(g_dp_mu);
    if (g_rs) { hip_ignore(hipStreamSynchronize(g_rs)); hip_ignore(hipStreamDestroy(g_rs)); g_rs = nullptr; }
    for (hipStream_t *c : {&g_h2d, &g_d2h})
        if (*c) { hip_ignore(hipStreamSynchronize(*c)); hip_ignore(hipStreamDestroy(*c)); *c = nullptr; }
    if (g_ctr_pool) { hip_ignore(hipFree(g_ctr_pool)); g_ctr_pool = nullptr; }
    ipc_close_all();
    for (FlagPages &fp : g_pages) {   // the pages themselves stay (exported memory)
        for (auto &p : fp.peer) p = nullptr;
        fp.mapped = false;
        fp.seg = nullptr;
    }
    arena_trim();
    if (g_seg_reg) { hip_ignore(hipHostUnregister(g_seg_reg)); g_seg_reg = nullptr; g_seg_dev = nullptr; }
}

// State every GPU transport keeps per schedule: the round stream, the completion
// event, the device receive bucket (the caller's, or an HBM copy of a host bucket), the
// shard layout and the producer events of posted rounds.
struct BaseState {
    hipStream_t stream = nullptr;     // the process's round stream (not owned)
    hipEvent_t ev = nullptr;
    // a round that went out in a shared launch (k_round_batch) reports faults through
    // that launch's event
    std::shared_ptr<hipEvent_t> batch_ev;
    char *rb_dev = nullptr;
    size_t cap = 0;                   // bytes of rb_dev (owned buckets may grow)
    uint64_t laid_count = ~0ull;      // count the shard layout was computed for
    bool owns_rb = false, reg_sb = false, reg_rb = false;
    // device buckets the IPC runtime cannot export (carved out of a cached allocation)
    // are shadowed by an owned bucket: copied in at the snapshot, out at the finish
    bool shadow = false;
    // host buckets that could not be pinned (FFCOLL_BUFFERS move every round) go
    // through this pinned staging buffer: host memcpy + DMA, never an async copy into
    // pageable memory whose completion an event would not cover
    char *pin = nullptr;
    // device views of the pinned host buffers (registered caller buckets, the staging
    // buffer): small host rounds move through them by kernel (host_move)
    char *view_sb = nullptr, *view_rb = nullptr, *view_pin = nullptr;
    size_t pin_cap = 0;
    bool copyout_pending = false;
    bool fin_mode = false;            // the round in flight reports through SchedShm::fin
    int batch_rc = 0;                 // the shared launch of this round failed (its status)
    bool in_batch = false;            // the round in flight went into a shared launch
    std::atomic<uint32_t> flushed{0}; // the last round whose shared launch went out
    uint64_t batch_seq = 0;           // that launch's number (g_batch_seq; g_batch_mu)
    std::vector<char *> retired;      // grown-out buckets: peers may still map them
    uint64_t off[kMaxRanks] = {}, len[kMaxRanks] = {};   // elements
    // events from the process-wide pool (pooled_event); one recording may be shared by a
    // group of posts / releases (esgd_schedule_post_group / _release_group)
    std::map<uint32_t, std::shared_ptr<hipEvent_t>> producer;
    // hold mode: the caller's last reads of rb / writes of sb (esgd_schedule_release)
    std::shared_ptr<hipEvent_t> consumer;
    bool consumer_pending = false;
    // rounds posted with their own data (esgd_schedule_post_io), by round; io_on: the
    // launched round takes cur_io (it was joined fresh, i.e. at or after that post)
    std::map<uint32_t, RoundIO> io;
    RoundIO cur_io{nullptr, nullptr, 1.0f};
    bool io_on = false;
    virtual ~BaseState() {}
};

// A mapped peer publication (IpcSlot): where it is in this process and which version.
struct PeerMap {
    char *ptr = nullptr;
    void *base = nullptr;
    uint32_t ver = 0;
    uint8_t handle[64] = {};
};

struct IpcState : BaseState {
    uint32_t *ctr = nullptr;          // device: k_round_small's counters and gates (pool)
    std::vector<hipEvent_t> cev;      // chunked host rounds: per chunk H2D / reduced / D2H
    bool chunked_before = false;
    // this rank's published shard (one-launch rounds): phase 1 writes the reduced shard
    // here as well as into rb, peers all-gather from it.  rb is then read by peers only in
    // phase 1, and pub is rewritten only after the next round's ready pairing, so the
    // round needs no third ("done") pairing.  Arena memory, L elements (the largest
    // shard).  k_round_small's last workgroup ends the round with SchedShm::fin = round;
    // teardown returns pub to the arena only once every peer's fin has reached pub_round
    // (deletion is local).  Five-launch rounds keep the done pairing and gather from rb:
    // the second store of the shard costs more there (+15-28 % at 256 MiB - 1 GiB,
    // profiles/r02/README.md) than the pairing's few microseconds.
    char *pub = nullptr;
    size_t pub_cap = 0;
    uint32_t pub_round = 0;
    char *peer[kMaxRanks] = {};       // every rank's rb (own included); its wire copy in wire mode
    // ESGD_SCHED_WIRE_BF16: this rank's bf16 copy of rb (arena, exported instead of rb;
    // count x 2 bytes).  Peers read only this: rb itself is never mapped by a peer.
    char *wire = nullptr;
    size_t wire_cap = 0;
    PeerMap rbmap[kMaxRanks], pubmap[kMaxRanks];
    // batched one-launch rounds: this schedule's BatchDesc is in the device table
    bool desc_built = false;
    // the round's snapshot, done by the shared launch's own workers (phase 0): 1 rb = sb,
    // 2 rb = 0, 3 rb = src / divisor (0: queued before the launch, or none)
    uint8_t snap_kind = 0;
    uint32_t t1 = 0, t2 = 0;          // its phase-1 / phase-2 tiles
};

// shard j = [off_j, off_j + len_j): equal shards rounded up to 1 KiB so every shard
// (and the 16-B vectors the kernels move) starts aligned; the last one is ragged.
static void layout(Sched &s, BaseState &st) {
    st.laid_count = s.count;
    const uint64_t align = 1024 / s.esize;
    uint64_t per = (s.count + uint64_t(s.world) - 1) / uint64_t(s.world);
    per = (per + align - 1) / align * align;
    for (int j = 0; j < s.world; ++j) {
        const uint64_t o = std::min<uint64_t>(s.count, per * uint64_t(j));
        st.off[j] = o;
        st.len[j] = std::min<uint64_t>(per, s.count - o);
    }
}

// Buckets the library owns come from the IPC arena (exportable, never freed under a peer).
static int alloc_bucket(size_t bytes, char **out, size_t *cap) {
    if (int rc = arena_alloc(std::max<size_t>(bytes, 1), reinterpret_cast<void **>(out))) return rc;
    *cap = std::max<size_t>(bytes, 1);
    return ESGD_SUCCESS;
}

static void free_bucket(char *p) {
    if (p && !arena_free(p)) hip_ignore(hipFree(p));
}

static int base_setup(Sched &s, BaseState &st) {
    if (s.esize == 0) { set_error("schedule: unsupported dtype %d", s.dtype); return ESGD_INVALID_ARG; }
    if (int rc = require_device()) return rc;
    const size_t bytes = s.count * s.esize;
    if (int rc = round_stream(&st.stream)) return rc;
    ESGD_HIP(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
    if (s.host_mode) {
        // FFCOLL_BUFFERS buckets change size: start with head room
        if (int rc = alloc_bucket(s.resolve ? std::max<size_t>(bytes, size_t(4) << 20) : bytes,
                                  &st.rb_dev, &st.cap))
            return rc;
        st.owns_rb = true;
        // pin (and map) the caller's persistent host buckets so the move / copy-out go
        // straight between them and HBM: DMA, or by kernel through the device view for
        // small buckets (host_move); not for FFCOLL_BUFFERS, whose buffers move every round
        if (!s.resolve && bytes && s.rb && hipHostRegister(s.rb, bytes, hipHostRegisterMapped) == hipSuccess) {
            st.reg_rb = true;
            st.view_rb = static_cast<char *>(host_view(s.rb));
        }
        if (!s.resolve && bytes && s.sb && s.sb != s.rb &&
            hipHostRegister(s.sb, bytes, hipHostRegisterMapped) == hipSuccess) {
            st.reg_sb = true;
            st.view_sb = static_cast<char *>(host_view(s.sb));
        }
        (void)hipGetLastError();   // "already registered" is fine
    } else {
        if (!s.rb) { set_error("schedule: null receive buffer"); return ESGD_INVALID_ARG; }
        if (reinterpret_cast<uintptr_t>(s.rb) & 15) {
            set_error("schedule: device receive buffer must be 16-B aligned");
            return ESGD_INVALID_ARG;
        }
        st.rb_dev = static_cast<char *>(s.rb);
    }
    layout(s, st);
    return ESGD_SUCCESS;
}

static std::mutex g_evfree_mu;
static std::vector<hipEvent_t> g_evfree;   // pooled events no round refers to any more

// ---- events: a process-wide pool, and recordings shared by a group of schedules ----
// A producer (consumer) event marks where the caller's stream stands at a post (release).
// esgd_schedule_post_group / _release_group record ONE event for all the schedules they
// name (dataplane_group_begin/end: this thread's posts / releases on that stream use it),
// and the round stream waits for a recording once however many rounds refer to it.
static std::shared_ptr<hipEvent_t> pooled_event() {
    hipEvent_t e = nullptr;
    {
        std::lock_guard<std::mutex> lk(g_evfree_mu);
        if (!g_evfree.empty()) { e = g_evfree.back(); g_evfree.pop_back(); }
    }
    if (!e && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
        (void)hip_fail(hipGetLastError(), "hipEventCreateWithFlags", __FILE__, __LINE__);
        return nullptr;
    }
    return std::shared_ptr<hipEvent_t>(new hipEvent_t(e), [](hipEvent_t *p) {
        std::lock_guard<std::mutex> lk(g_evfree_mu);
        g_evfree.push_back(*p);
        delete p;
    });
}

static hipStream_t user_stream(void *stream) {   // ESGD_STREAM_NULL names the legacy default stream
    return stream == ESGD_STREAM_NULL ? nullptr : static_cast<hipStream_t>(stream);
}

struct GroupEvent {   // this thread's open group: [0] posts, [1] releases
    bool open = false;
    void *stream = nullptr;
    std::shared_ptr<hipEvent_t> ev;
};
static thread_local GroupEvent g_group[2];

int dataplane_group_begin(int which, void *stream) {
    GroupEvent &g = g_group[which];
    g.open = true;
    g.stream = stream;
    g.ev.reset();   // recorded by the group's first schedule that needs it
    return ESGD_SUCCESS;
}

void dataplane_group_end(int which) {
    g_group[which].open = false;
    g_group[which].ev.reset();
}

// the event of a post (which 0) or release (1) on `stream`: the open group's recording,
// or a new one
static int note_event(int which, void *stream, std::shared_ptr<hipEvent_t> *out) {
    GroupEvent &g = g_group[which];
    const bool same = g.open && g.stream == stream;
    if (same && g.ev) {
        *out = g.ev;
        return ESGD_SUCCESS;
    }
    std::shared_ptr<hipEvent_t> ev = pooled_event();
    if (!ev) return ESGD_ERROR;
    ESGD_HIP(hipEventRecord(*ev, user_stream(stream)));
    if (g.open && g.stream == stream) g.ev = ev;
    *out = ev;
    return ESGD_SUCCESS;
}

// cs waits for ev -- once per recording: a later wait on the same recording is implied
// by stream order (the progress thread queues every wait on the round / copy streams)
static struct {
    hipStream_t s;
    std::shared_ptr<hipEvent_t> ev;
} g_waited[4];

static int stream_wait(hipStream_t cs, const std::shared_ptr<hipEvent_t> &ev) {
    int slot = -1;
    for (int i = 0; i < 4; ++i) {
        if (g_waited[i].s == cs) {
            if (g_waited[i].ev == ev) return ESGD_SUCCESS;
            slot = i;
            break;
        }
        if (!g_waited[i].s && slot < 0) slot = i;
    }
    ESGD_HIP(hipStreamWaitEvent(cs, *ev, 0));
    if (slot >= 0) {
        g_waited[slot].s = cs;
        g_waited[slot].ev = ev;
    }
    return ESGD_SUCCESS;
}

static int base_note_producer(BaseState &st, uint32_t round, void *stream) {
    std::shared_ptr<hipEvent_t> ev;
    if (int rc = note_event(0, stream, &ev)) return rc;
    st.producer[round] = std::move(ev);
    return ESGD_SUCCESS;
}

static int base_note_consumer(BaseState &st, void *stream) {
    std::shared_ptr<hipEvent_t> ev;
    if (int rc = note_event(1, stream, &ev)) return rc;
    st.consumer = std::move(ev);
    st.consumer_pending = true;
    return ESGD_SUCCESS;
}

int Transport::note_io(Sched &, uint32_t, const RoundIO &) {
    set_error("this transport does not take a round's own data (esgd_schedule_post_io)");
    return ESGD_INVALID_ARG;
}

// esgd_schedule_post_io: checked at the post, used by the round it posts if that round
// is joined fresh (take_io)
static int base_note_io(Sched &s, BaseState &st, uint32_t round, const RoundIO &io) {
    ESGD_ARG(!s.host_mode && !s.resolve && !s.wire_bf16,
             "schedule %d: a round's own data needs a device schedule without FFCOLL_BUFFERS or WIRE_BF16", s.id);
    if (io.segs) {   // post_iov: fp32 pieces, any alignment (the pack kernels take it)
        ESGD_ARG(s.dtype == ESGD_FLOAT, "schedule %d: post_iov needs FLOAT buckets", s.id);
        ESGD_ARG(io.div == io.div && io.div != 0.0f, "schedule %d: post_iov: bad divisor", s.id);
        uint64_t total = 0;
        for (size_t i = 0; i < io.segs->count.size(); ++i) {
            ESGD_ARG(io.segs->count[i] == 0 || (io.segs->src[i] && io.segs->dst[i]),
                     "schedule %d: post_iov: piece %zu has a null pointer", s.id, i);
            total += io.segs->count[i];
        }
        ESGD_ARG(total == s.count, "schedule %d: post_iov: %llu elements in the pieces for a %llu-element schedule",
                 s.id, (unsigned long long)total, (unsigned long long)s.count);
        st.io[round] = io;
        return ESGD_SUCCESS;
    }
    ESGD_ARG(s.count == 0 || (io.src && io.dst), "schedule %d: post_io: null src or dst", s.id);
    ESGD_ARG(((reinterpret_cast<uintptr_t>(io.src) | reinterpret_cast<uintptr_t>(io.dst)) & 15) == 0,
             "schedule %d: post_io: src and dst must be 16-B aligned", s.id);
    ESGD_ARG(io.div == io.div && io.div != 0.0f, "schedule %d: post_io: bad divisor", s.id);
    ESGD_ARG(io.div == 1.0f || s.dtype == ESGD_FLOAT, "schedule %d: post_io: a divisor needs FLOAT buckets", s.id);
    st.io[round] = io;
    return ESGD_SUCCESS;
}

// at launch: the round's own data, if it was posted with some and joined fresh; entries
// of this and earlier rounds are dropped (a round carried through before its post ran
// with the send bucket)
static void take_io(BaseState &st, uint32_t round, bool fresh) {
    st.io_on = false;
    for (auto it = st.io.begin(); it != st.io.end() && it->first <= round;) {
        if (it->first == round && fresh) {
            st.cur_io = it->second;
            st.io_on = true;
        }
        it = st.io.erase(it);
    }
}

// rb's place of each piece of a post_iov round, in order
static std::vector<float *> io_pieces_in_rb(const BaseState &st, const RoundIOSegs &g) {
    std::vector<float *> at(g.count.size());
    float *p = reinterpret_cast<float *>(st.rb_dev);
    for (size_t i = 0; i < at.size(); ++i) {
        at[i] = p;
        p += g.count[i];
    }
    return at;
}

// the copy-in of a round with its own data, queued on the round stream: rb = src / div
static int io_copy_in(Sched &s, BaseState &st, hipStream_t cs) {
    const size_t bytes = s.count * s.esize;
    if (!bytes) return ESGD_SUCCESS;
    if (const RoundIOSegs *g = st.cur_io.segs.get()) {   // the pieces packed into rb (/ div)
        const std::vector<float *> at = io_pieces_in_rb(st, *g);
        return pack_scatter(int(at.size()), g->src.data(), at.data(), g->count.data(), st.cur_io.div, cs);
    }
    if (st.cur_io.div == 1.0f) {
        ESGD_HIP(hipMemcpyAsync(st.rb_dev, st.cur_io.src, bytes, hipMemcpyDeviceToDevice, cs));
        return ESGD_SUCCESS;
    }
    const float *src = static_cast<const float *>(st.cur_io.src);
    float *dst = reinterpret_cast<float *>(st.rb_dev);
    const uint64_t n = s.count;
    return pack_scatter(1, &src, &dst, &n, st.cur_io.div, cs);
}

// queued at launch, before anything touches the buckets: the caller's copy-out of the
// previous round (and its zeroing of sb) has finished -- fresh round or not
static int consumer_wait(BaseState &st, hipStream_t cs) {
    if (st.consumer_pending) {
        if (int rc = stream_wait(cs, st.consumer)) return rc;
        st.consumer_pending = false;
    }
    return ESGD_SUCCESS;
}

// FFCOLL_BUFFERS rounds may change the count: re-lay the shards and grow the owned
// device bucket (ffallreduce_post resizes its temporaries the same way, :42-48).
// Returns 1 when the device bucket moved (peers must re-map it).
static int base_refit(Sched &s, BaseState &st) {
    if (st.laid_count == s.count) return 0;
    const size_t bytes = s.count * s.esize;
    int moved = 0;
    if (bytes > st.cap) {
        if (!st.owns_rb) { set_error("schedule %d: device bucket cannot grow", s.id); return ESGD_INVALID_ARG; }
        // grow geometrically; the old bucket goes back to the arena at teardown
        st.retired.push_back(st.rb_dev);
        if (int rc = alloc_bucket(std::max(bytes, 2 * st.cap), &st.rb_dev, &st.cap)) return rc;
        moved = 1;
    }
    layout(s, st);
    return moved;
}

static bool debug_on() {
    static const bool on = getenv("ESGD_DEBUG") && *getenv("ESGD_DEBUG") == '1';
    return on;
}
#define ESGD_TRACE(...)                                                   \
    do {                                                                  \
        if (debug_on()) { fprintf(stderr, "[esgd] " __VA_ARGS__); fflush(stderr); } \
    } while (0)

// Host buckets up to this many bytes move between host memory and HBM by kernel: the
// round's stream reads / writes the pinned bucket directly over PCIe (16-B system-scope
// loads, all in flight at once) instead of a DMA copy, whose fixed cost dominates small
// buckets (C1, 1 MiB: DESIGN.md §7).
constexpr uint64_t kHostKernelCopyBytes = uint64_t(4) << 20;

// dst <- src, one of them pinned host memory with device view `view` (or nullptr)
static int host_move(void *dst, const void *src, const void *view, bool h2d, size_t bytes, hipStream_t cs) {
    const void *ks = h2d ? view : src;
    void *kd = h2d ? dst : const_cast<void *>(view);
    if (view && bytes <= kHostKernelCopyBytes &&
        ((reinterpret_cast<uintptr_t>(ks) | reinterpret_cast<uintptr_t>(kd)) & 15) == 0) {
        const uint64_t b = bytes;
        return gather_remote(1, &ks, &kd, &b, cs);
    }
    ESGD_HIP(hipMemcpyAsync(dst, src, bytes, h2d ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, cs));
    return ESGD_SUCCESS;
}

static bool staged(Sched &s, BaseState &st) {
    return s.host_mode && (s.resolve || !st.reg_rb || (s.sb && s.sb != s.rb && !st.reg_sb));
}

static int ensure_pin(BaseState &st, size_t bytes) {
    if (bytes <= st.pin_cap) return ESGD_SUCCESS;
    if (st.pin) ESGD_HIP(hipHostFree(st.pin));
    st.pin = nullptr;
    ESGD_HIP(hipHostMalloc(reinterpret_cast<void **>(&st.pin), bytes, hipHostMallocMapped));
    st.pin_cap = bytes;
    st.view_pin = static_cast<char *>(host_view(st.pin));
    return ESGD_SUCCESS;
}

// Join-time host work: the move of an unpinned host bucket into the pinned staging
// buffer happens now, when the rank joins (the reference's move reads sb at activation,
// colls/ffallreduce.c:126-130).  The previous round has completed, so the buffer is free.
static int base_prepare(Sched &s, BaseState &st, bool fresh) {
    const size_t bytes = s.count * s.esize;
    if (bytes && staged(s, st) && !(s.fresh_only && !fresh)) {   // FRESH_ONLY: not read
        if (int rc = ensure_pin(st, bytes)) return rc;
        std::memcpy(st.pin, s.sb ? s.sb : s.rb, bytes);
    }
    return ESGD_SUCCESS;
}

// queued at launch: the producer of this round (posted before the join) must have
// finished, then the move sb -> rb (host -> HBM for host buckets)
static int producer_wait(BaseState &st, uint32_t round, bool fresh, hipStream_t cs) {
    for (auto it = st.producer.begin(); it != st.producer.end();) {
        if (it->first == round && fresh)
            if (int rc = stream_wait(cs, it->second)) return rc;
        if (it->first <= round) it = st.producer.erase(it);
        else ++it;
    }
    return ESGD_SUCCESS;
}

static int base_copy_in(Sched &s, BaseState &st, uint32_t round, bool fresh, hipStream_t cs) {
    if (int rc = consumer_wait(st, cs)) return rc;
    if (int rc = producer_wait(st, round, fresh, cs)) return rc;
    const size_t bytes = s.count * s.esize;
    if (!bytes) return ESGD_SUCCESS;
    if (st.io_on) return io_copy_in(s, st, cs);   // the round's own data (post_io)
    if (s.fresh_only && !fresh) {
        // carried through a round it had not posted: this rank contributes zeros, and its
        // send bucket -- which the caller may be writing right now -- is not read
        ESGD_HIP(hipMemsetAsync(st.rb_dev, 0, bytes, cs));
        return ESGD_SUCCESS;
    }
    if (s.host_mode) {
        const bool stg = staged(s, st);
        const void *src = stg ? st.pin : (s.sb ? s.sb : s.rb);
        const void *view = stg ? st.view_pin : (s.sb ? st.view_sb : st.view_rb);
        if (int rc = host_move(st.rb_dev, src, view, true, bytes, cs)) return rc;
    } else if (s.zero_sb) {
        // the move and the wrapper's zero-after-use in one pass: rb = sb, sb = 0
        if (int rc = move_zero(st.rb_dev, s.sb, bytes, cs)) return rc;
    } else if (!s.in_place || st.shadow) {
        const void *src = s.in_place ? s.rb : s.sb;
        ESGD_HIP(hipMemcpyAsync(st.rb_dev, src, bytes, hipMemcpyDeviceToDevice, cs));
    }
    return ESGD_SUCCESS;
}

// queued at launch, last: the copy-out and the round's completion event
// The end of every queued round: a one-lane kernel stores the round in the rank's fin
// word (polled by the progress thread) behind everything queued before it; the event
// after it only reports faults.  Without the registered node segment (a world of one
// that never needed it) completion is the event's.
static int finish_round(Sched &s, BaseState &st, hipStream_t cs) {
    st.fin_mode = g_seg_reg != nullptr && g_seg_reg == engine_segment();
    if (st.fin_mode)
        if (int rc = store_fin(dev_flag(&s.sh->fin[s.rank]), s.cur, cs)) return rc;
    ESGD_HIP(hipEventRecord(st.ev, cs));
    return ESGD_SUCCESS;
}

static int base_copy_out(Sched &s, BaseState &st, hipStream_t cs) {
    const size_t bytes = s.count * s.esize;
    if (st.io_on && bytes && st.cur_io.segs) {   // post_iov: rb unpacked into the pieces
        const RoundIOSegs &g = *st.cur_io.segs;
        const std::vector<float *> at = io_pieces_in_rb(st, g);
        std::vector<const float *> from(at.begin(), at.end());
        if (int rc = unpack_gather(int(at.size()), g.dst.data(), from.data(), g.count.data(), cs)) return rc;
    } else if (st.io_on && bytes) {   // the round's own output (post_io); rb is not the caller's then
        ESGD_HIP(hipMemcpyAsync(st.cur_io.dst, st.rb_dev, bytes, hipMemcpyDeviceToDevice, cs));
    } else if (s.host_mode && bytes) {
        if (staged(s, st)) {
            if (int rc = ensure_pin(st, bytes)) return rc;
            if (int rc = host_move(st.pin, st.rb_dev, st.view_pin, false, bytes, cs)) return rc;
            st.copyout_pending = true;
        } else {
            if (int rc = host_move(s.rb, st.rb_dev, st.view_rb, false, bytes, cs)) return rc;
        }
    } else if (st.shadow && bytes) {
        ESGD_HIP(hipMemcpyAsync(s.rb, st.rb_dev, bytes, hipMemcpyDeviceToDevice, cs));
    }
    return finish_round(s, st, cs);
}

static int base_complete(Sched &s, BaseState &st) {
    if (st.copyout_pending) {
        std::memcpy(s.rb, st.pin, s.count * s.esize);
        st.copyout_pending = false;
    }
    return ESGD_SUCCESS;
}

// Why a round has not finished: every rank's flag words of this schedule (ready / reduced /
// done / fin, the GPU error word, the last round it joined) and how this rank's round went
// out (one launch of its own, a shared launch, shadowed).
static std::string base_diagnose(Sched &s) {
    std::string m = "(per rank ready/reduced/done/fin/err/joined:";
    char buf[96];
    for (int q = 0; q < s.world; ++q) {
        snprintf(buf, sizeof(buf), " r%d %u/%u/%u/%u/%u/%u", q, s.sh->ready[q].load(), s.sh->reduced[q].load(),
                 s.sh->done[q].load(), s.sh->fin[q].load(), s.sh->gpu_err[q].load(), s.sh->joined[q].load());
        m += buf;
    }
    if (s.flag_mode > 0) m += "; pairing flags in device memory, mode " + std::to_string(s.flag_mode) + " (not shown)";
    if (auto *st = static_cast<BaseState *>(s.tstate)) {
        snprintf(buf, sizeof(buf), "; this rank: %s%s%s", st->batch_ev ? "shared launch" : "own launch",
                 st->shadow ? ", shadowed bucket" : "", st->fin_mode ? ", fin-polled" : ", event-polled");
        m += buf;
    }
    return m + ")";
}

// The failure contract: a round that failed on ANY rank -- a GPU flag wait
// that timed out, or that found a peer's error word holding the round -- fails here too.
// The GPU side already keeps a failed rank from publishing reduced / fin for the round, so
// a late peer cannot complete it from that rank's stale shard; this check also fails a
// round this rank completed while a peer gave up on it.
static int round_failed(Sched &s) {
    if (s.world < 2) return 0;
    for (int q = 0; q < s.world; ++q) {
        if (s.sh->gpu_err[q].load(std::memory_order_acquire) != s.cur) continue;
        if (q == s.rank)
            set_error("this rank's GPU waited more than %.0f s for its peers in round %u %s", engine_timeout(), s.cur,
                      base_diagnose(s).c_str());
        else
            set_error("rank %d failed round %u (its GPU flag wait timed out or saw a failure), so this rank fails "
                      "it too %s",
                      q, s.cur, base_diagnose(s).c_str());
        return ESGD_ERROR;
    }
    return 0;
}

static int base_query(Sched &s, BaseState &st) {
    if (st.batch_rc) return st.batch_rc;   // error message set by the failed launch
    if (st.fin_mode) {   // the round's last kernel writes fin (finish_round, k_round_small, done pairing)
        // a timed-out flag wait of a batched round still lets its workers finish (and
        // write fin): fin is loaded first, then the error word -- the GPU stores the error
        // (and releases it) before it opens the gates that let any worker write fin, so a
        // fin seen here comes with the error of that round, if there was one (a timed-out
        // k_round_small leaves without fin: the error alone fails the round then)
        const bool finished = int32_t(s.sh->fin[s.rank].load(std::memory_order_acquire) - s.cur) >= 0;
        if (int rc = round_failed(s)) return rc;
        if (finished) {
            // the kernel may still be retiring (not ready is fine); a fault is reported
            // against this round, not a later one
            const hipError_t e = hipEventQuery(st.batch_ev ? *st.batch_ev : st.ev);
            if (e != hipSuccess && e != hipErrorNotReady) {
                (void)hip_fail(e, "one-launch round", __FILE__, __LINE__);
                std::string m = esgd_last_error();
                set_error("%s (schedule %d, %llu elements of dtype %d)", m.c_str(), s.id,
                          (unsigned long long)s.count, s.dtype);
                return ESGD_ERROR;
            }
            return 1;
        }
        return 0;
    }
    hipError_t e = hipEventQuery(st.ev);
    if (e == hipErrorNotReady) return 0;
    if (e != hipSuccess) {
        (void)hip_fail(e, "hipEventQuery", __FILE__, __LINE__);
        std::string m = esgd_last_error();
        set_error("%s (schedule %d, %llu elements of dtype %d)", m.c_str(), s.id,
                  (unsigned long long)s.count, s.dtype);
        return ESGD_ERROR;
    }
    if (int rc = round_failed(s)) return rc;
    return 1;
}

static void base_teardown(Sched &s, BaseState &st) {
    if (st.stream) hip_ignore(hipStreamSynchronize(st.stream));
    if (st.owns_rb) free_bucket(st.rb_dev);
    if (st.reg_rb) hip_ignore(hipHostUnregister(s.rb));
    if (st.reg_sb) hip_ignore(hipHostUnregister(s.sb));
    st.producer.clear();   // pooled events go back to the pool
    st.consumer.reset();
    if (st.pin) hip_ignore(hipHostFree(st.pin));
    for (char *p : st.retired) free_bucket(p);
    if (st.ev) hip_ignore(hipEventDestroy(st.ev));
}

// ---- batched one-launch rounds (round_batch.hip) ---------------------------------------
// Device rounds of one-launch size that come due together in issue order go out in ONE
// k_round_batch launch: IpcTransport::launch queues each round's snapshot on the round
// stream and appends the round here; the engine flushes at the end of every pump of the
// issue ring, and every other launch on the round stream flushes first, so the stream
// still holds the rounds in ring order (the deadlock argument of DESIGN.md §5).
static std::mutex g_batch_mu;
static BatchDesc *g_desc_dev = nullptr, *g_desc_host = nullptr;   // [kMaxSched], by schedule id
struct BatchEntry {
    Sched *s;
    IpcState *st;
    uint32_t round;
    uint8_t snap;   // the snapshot the launch's workers do (0: none, or queued before it)
    RoundIO io;     // the round's own data (src nullptr: none; dst nullptr: results in rb)
};

// the whole-bucket snapshot (rb = src) fits the kernel's 32-bit buffer ranges and 16-B
// vectors (src nullptr: rb alone)
static bool snap_eligible(const Sched &s, const IpcState &st, const void *src) {
    const size_t bytes = s.count * s.esize;
    const uintptr_t al = reinterpret_cast<uintptr_t>(st.rb_dev) | reinterpret_cast<uintptr_t>(src);
    return bytes && bytes < (size_t(1) << 31) && (al & 15) == 0;
}
static std::vector<BatchEntry> g_pend;
static uint64_t g_batch_seq = 0;   // shared launches sent so far (g_batch_mu)
// the shared launches' tile bookkeeping (BatchArgs::slots: kLaunchSlots x kSlotWords device
// words behind the descriptor table); launch n uses slot n % kLaunchSlots, and each launch
// zeroes the others on the GPU, so no host count has to track the device's
static uint32_t *g_slots = nullptr;
static uint32_t g_slot_seq = 0;

uint32_t batch_workers_max() {
    static const uint32_t env = [] {
        const char *e = getenv("ESGD_BATCH_WORKERS");
        const long n = (e && *e) ? atol(e) : long(kBatchWorkers);
        return uint32_t(std::max<long>(1, std::min<long>(long(kBatchWorkersMax), n)));
    }();
    const int64_t v = g_cfg_workers.load(std::memory_order_relaxed);
    return v > 0 ? uint32_t(v) : env;
}

static uint32_t snapshot_workers_max() {
    static const uint32_t env = [] {
        const char *e = getenv("ESGD_SNAPSHOT_WORKERS");
        const long n = (e && *e) ? atol(e) : long(kSnapshotWorkers);
        return uint32_t(std::max<long>(0, std::min<long>(long(kBatchWorkersMax), n)));
    }();
    const int64_t v = g_cfg_snapw.load(std::memory_order_relaxed);
    const uint32_t w = v >= 0 ? uint32_t(v) : env;
    return w ? std::max(w, batch_workers_max()) : batch_workers_max();
}

// shared launches queued and not yet seen complete, oldest first (their events)
static std::deque<std::shared_ptr<hipEvent_t>> g_outstanding;

// At the end of a pump the pending launch goes out only while no shared launch is queued
// and unfinished; rounds that come due meanwhile join the next launch instead of each pump
// making its own (round 4, ranks sharing one GPU, interleaved A/B: the 161-bucket pipelined
// step 0.75-0.83 -> 0.66-0.71 ms at P = 2, 1.26-1.52 -> 0.97-0.99 ms at P = 4 against a
// flush at every pump; holding more launches back slowed P = 4).
constexpr size_t kBatchDepth = 1;

// this schedule's BatchDesc: built at its first batched round and uploaded on the round
// stream (ahead of the launch that reads it); its buckets, peers' mappings and flags never
// move afterwards (FFCOLL_BUFFERS schedules are not batched).  g_batch_mu held.
static int batch_desc(Sched &s, IpcState &st, hipStream_t cs) {
    if (st.desc_built) return ESGD_SUCCESS;
    if (!g_desc_dev) {
        const size_t slot_bytes = size_t(kLaunchSlots) * kSlotWords * sizeof(uint32_t);
        ESGD_HIP(hipMalloc(reinterpret_cast<void **>(&g_desc_dev), sizeof(BatchDesc) * kMaxSched + slot_bytes));
        ESGD_HIP(hipHostMalloc(reinterpret_cast<void **>(&g_desc_host), sizeof(BatchDesc) * kMaxSched,
                               hipHostMallocDefault));
        g_slots = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(g_desc_dev) + sizeof(BatchDesc) * kMaxSched);
        ESGD_HIP(hipMemsetAsync(g_slots, 0, slot_bytes, cs));   // ahead of every launch on this stream
        g_slot_seq = 0;
    }
    if (!st.ctr)
        if (int rc = ctr_words(s.id, cs, &st.ctr)) return rc;
    const size_t es = s.esize;
    const int r = s.rank;
    BatchDesc d;
    std::memset(&d, 0, sizeof(d));
    for (int j = 0; j < s.world; ++j) d.src[j] = st.peer[j] + st.off[r] * es;
    d.out = st.rb_dev + st.off[r] * es;
    d.pub = st.pub;
    d.n = st.len[r];
    batch_tiling(st.len[r] * es / 16, batch_workers_max(), &d.t1, &d.tv1);
    uint32_t m = 0;
    for (int j = 0; j < s.world; ++j)
        if (j != r && st.len[j]) ++m;
    const uint32_t per_seg = std::max<uint32_t>(1, batch_workers_max() / std::max<uint32_t>(1, m));
    m = 0;
    for (int j = 0; j < s.world; ++j) {
        if (j == r || st.len[j] == 0) continue;
        const uint64_t bytes = st.len[j] * es;
        d.gsrc[m] = st.pubmap[j].ptr;   // peer j's published shard j
        d.gdst[m] = st.rb_dev + st.off[j] * es;
        d.gvec[m] = uint32_t(bytes / 16);
        d.gtail[m] = uint32_t(bytes % 16);
        uint32_t tiles = 0;
        batch_tiling(d.gvec[m], per_seg, &tiles, &d.tvg[m]);
        d.t2pre[m + 1] = d.t2pre[m] + tiles;
        ++m;
    }
    d.nseg = m;
    d.strict = s.strict ? 1u : 0u;
    d.ready = pair_flags(s, s.sh->ready, 0);
    d.reduced = pair_flags(s, s.sh->reduced, 1);
    d.fin = dev_flag(&s.sh->fin[r]);
    d.err = dev_flag(&s.sh->gpu_err[r]);
    d.ctr = st.ctr + 6;   // words 6..10 of the schedule's device counters
    if (snap_eligible(s, st, nullptr)) {   // the in-launch snapshot's target (rb) fits it
        const size_t bytes = s.count * es;
        d.ssrc = s.in_place ? nullptr : s.sb;
        d.sdst = st.rb_dev;
        d.svec = uint32_t(bytes / 16);
        d.stail = uint32_t(bytes % 16);
    }
    d.rbase = st.rb_dev;
    d.rank = uint32_t(r);
    {
        const uint64_t b0 = st.off[r] * es, b1 = (st.off[r] + st.len[r]) * es, total = s.count * es;
        d.own_v0 = uint32_t(b0 / 16);
        d.own_v1 = uint32_t(b1 / 16);
        d.own_tail = (st.len[r] && b1 == total && total % 16) ? 1u : 0u;
        d.own_off = b0;
    }
    st.t1 = d.t1;
    st.t2 = std::max<uint32_t>(1, d.t2pre[m]);   // at least one tile: it writes fin
    g_desc_host[s.id] = d;
    ESGD_HIP(hipMemcpyAsync(&g_desc_dev[s.id], &g_desc_host[s.id], sizeof(BatchDesc), hipMemcpyHostToDevice, cs));
    st.desc_built = true;
    return ESGD_SUCCESS;
}

// ranks of this job whose GPU is this process's (1 with a GPU per rank; the rehearsal on
// a 1-GPU box puts every rank there).  Compared by PCI location, not by ordinal: with
// HIP_VISIBLE_DEVICES set per rank every process calls its GPU "device 0".
static int ranks_on_my_device() {
    Segment *seg = engine_segment();
    const int me = engine_rank(), world = engine_world();
    if (!seg) return 1;
    const uint64_t gid = seg->gpu_id[me].load();
    const int dev = seg->device[me].load();
    int n = 0;
    for (int q = 0; q < world; ++q)
        n += gid ? seg->gpu_id[q].load() == gid : seg->device[q].load() == dev;
    return std::max(1, n);
}

static int batch_flush_locked() {
    if (g_pend.empty()) return ESGD_SUCCESS;
    const int n = int(g_pend.size());
    BatchArgs a;
    std::memset(&a, 0, sizeof(a));
    a.table = g_desc_dev;
    a.nent = uint32_t(n);
    a.timeout = (long long)(engine_timeout() * double(g_ticks_per_s));
    uint32_t t0 = 0, t1 = 0, t2 = 0;
    for (int e = 0; e < n; ++e) {
        a.sid[e] = uint16_t(g_pend[e].s->id);
        a.value[e] = g_pend[e].round;
        a.tile0[e] = t0;
        a.tile1[e] = t1;
        a.tile2[e] = t2;
        a.isrc[e] = g_pend[e].snap ? g_pend[e].io.src : nullptr;   // read by phase 0 only
        a.iout[e] = g_pend[e].io.dst;
        a.idiv[e] = g_pend[e].io.div;
        if (const uint8_t k = g_pend[e].snap) {
            const BatchDesc &d = g_desc_host[g_pend[e].s->id];
            a.snap[e] = k;
            t0 += (d.svec + 1023) / 1024 + (d.svec == 0 && d.stail ? 1 : 0);
        }
        t1 += g_pend[e].st->t1;
        t2 += g_pend[e].st->t2;
    }
    a.tile0[n] = t0;
    a.tile1[n] = t1;
    a.tile2[n] = t2;
    const unsigned wmax = t0 ? snapshot_workers_max() : batch_workers_max();
    unsigned workers = std::min<unsigned>(wmax, std::max<unsigned>(1, std::max(t0, std::max(t1, t2))));
    // The launch's rounds complete with the agent and one worker resident (the tile
    // counter), but the stream's next launch starts only once every workgroup of this one
    // was dispatched and left -- so the grid is kept to what the GPU can hold beside the
    // other ranks' launches: with 8 ranks on one GPU, 8 x 65 workgroups of the fan-in-8
    // kernel (2 per CU) were all of it, and the five-launch rounds' pairing kernels (then
    // 256 spinning workgroups each; one since round 6) left some launch short (r04zp,
    // DESIGN.md §5).  Ranks sharing a GPU get half their share; one rank per GPU keeps
    // kBatchWorkers (far below the chip's capacity).
    const int capacity = round_batch_capacity(g_pend[0].s->dtype, g_pend[0].s->world);
    const int sharing = ranks_on_my_device();
    const int cap = capacity / (sharing > 1 ? 2 * sharing : 1) - 1;
    workers = std::max(1u, std::min<unsigned>(workers, unsigned(std::max(1, cap))));
    hipStream_t cs = g_pend[0].st->stream;
    int rc = ESGD_SUCCESS;
    if (capacity <= 0) {   // every entry of the launch fails (never a silent single worker)
        set_error("batched rounds: no residency figure for dtype %d at %d ranks", g_pend[0].s->dtype,
                  g_pend[0].s->world);
        rc = ESGD_ERROR;
    }
    // the launch's slot: zeroed by the previous launch that ran on this stream (every
    // launch zeroes all slots but its own), whatever the host believes of earlier launches
    a.slots = g_slots;
    a.slot = g_slot_seq++ % kLaunchSlots;
    // ranks sharing this GPU: a worker spinning on a closed gate for 2 ms gives its wave
    // slots back -- the peer launch that opens the gate may be waiting for them (DESIGN.md
    // §5, "Forward progress"); with a GPU per rank nothing of the job competes for them
    a.yield = sharing > 1 ? (long long)(2e-3 * double(g_ticks_per_s)) : 0;
    (void)hipGetLastError();   // a stale status (e.g. an event query's not-ready) is not this launch's
    if (!rc) rc = round_batch(g_pend[0].s->dtype, g_pend[0].s->world, a, workers, cs);
    if (!rc) g_batch_workers.store(int64_t(workers), std::memory_order_relaxed);
    std::shared_ptr<hipEvent_t> sp;
    if (!rc) {
        sp = pooled_event();
        if (!sp) rc = ESGD_ERROR;
        else if (hipEventRecord(*sp, cs) != hipSuccess) rc = hip_fail(hipGetLastError(), "hipEventRecord", __FILE__, __LINE__);
    }
    if (rc) {
        // a launch counted as failed may still have run, or may not have: either way the
        // next one finds every slot at zero (behind it on the stream), however many fail in
        // a row -- the zeroing by a launch that runs covers only the launches after it
        const size_t slot_bytes = size_t(kLaunchSlots) * kSlotWords * sizeof(uint32_t);
        if (hipMemsetAsync(g_slots, 0, slot_bytes, cs) != hipSuccess) (void)hipGetLastError();
    }
    ++g_batch_seq;
    for (BatchEntry &b : g_pend) {
        b.st->batch_ev = sp;
        b.st->batch_rc = rc;
        b.st->batch_seq = g_batch_seq;
        b.st->flushed.store(b.round, std::memory_order_release);
    }
    if (sp) g_outstanding.push_back(sp);
    g_pend.clear();
    ++g_launches;
    return rc;
}

static std::atomic<uint64_t> g_flush_ns{0};

int dataplane_flush() {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (g_pend.empty()) return ESGD_SUCCESS;
    const double t0 = now_s();
    const int rc = batch_flush_locked();
    g_flush_ns.fetch_add(uint64_t((now_s() - t0) * 1e9), std::memory_order_relaxed);
    return rc;
}

// The end of a pump: the pending launch goes out unless kBatchDepth shared launches
// are still queued.  A held launch cannot deadlock the node: the launches it waits behind
// hold only rounds earlier in the issue order, which every peer has launched already (it
// launched a later one) or will launch before any it holds back, so they complete, and
// the next pass sends the held rounds.
int dataplane_flush_soft() {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (g_pend.empty() || g_cfg_hold.load(std::memory_order_relaxed)) return ESGD_SUCCESS;
    while (!g_outstanding.empty() && hipEventQuery(*g_outstanding.front()) != hipErrorNotReady)
        g_outstanding.pop_front();   // finished (a fault is reported by its rounds)
    (void)hipGetLastError();   // the not-ready status is not an error of the next launch
    if (g_outstanding.size() >= kBatchDepth) return ESGD_SUCCESS;
    const double t0 = now_s();
    const int rc = batch_flush_locked();
    g_flush_ns.fetch_add(uint64_t((now_s() - t0) * 1e9), std::memory_order_relaxed);
    return rc;
}


// diagnostics for a timed-out wait: the shared launch being filled (schedule:round of each
// entry), shared launches queued and not yet seen finished, and a seal I/O in progress
std::string dataplane_state() {
    std::string m;
    char buf[64];
    {
        std::lock_guard<std::mutex> lk(g_batch_mu);
        snprintf(buf, sizeof(buf), "pending shared launch %zu rounds", g_pend.size());
        m += buf;
        for (size_t i = 0; i < g_pend.size() && i < 16; ++i) {
            snprintf(buf, sizeof(buf), "%s%d:%u", i ? "," : " [", g_pend[i].s->id, g_pend[i].round);
            m += buf;
        }
        if (!g_pend.empty()) m += g_pend.size() > 16 ? ",...]" : "]";
        size_t busy = 0;
        for (auto &e : g_outstanding) busy += hipEventQuery(*e) == hipErrorNotReady;
        (void)hipGetLastError();
        snprintf(buf, sizeof(buf), "; %zu shared launches unfinished", busy);
        m += buf;
        if (g_cfg_hold.load()) m += " (batch_hold)";
    }
    if (seal_io_busy()) m += "; a seal read/write is waiting for the round stream";
    return m;
}

void dataplane_profile(uint64_t *launches, uint64_t *flush_ns) {
    *launches = g_launches.load(std::memory_order_relaxed);
    *flush_ns = g_flush_ns.load(std::memory_order_relaxed);
}

// The snapshot of a round that goes out in a shared launch: the caller's producer and
// consumer events are waited for now, on the round stream; the copy itself (rb = sb, rb = 0
// for a FRESH_ONLY round this rank had not posted, or rb = src / divisor) is phase 0 of the
// launch when the buckets are 16-B aligned and the copy fits the 32-bit descriptor range
// (else it is queued now, as base_copy_in would).
static int batch_snapshot(Sched &s, IpcState &st, uint32_t round, bool fresh, hipStream_t cs) {
    if (int rc = consumer_wait(st, cs)) return rc;
    if (int rc = producer_wait(st, round, fresh, cs)) return rc;
    st.snap_kind = 0;
    const size_t bytes = s.count * s.esize;
    if (!bytes) return ESGD_SUCCESS;
    if (st.io_on) {   // the round's own data (post_io): rb = src / div
        if (snap_eligible(s, st, st.cur_io.src)) {   // phase 0 of the shared launch
            st.snap_kind = st.cur_io.div == 1.0f ? 1 : 3;
            return ESGD_SUCCESS;
        }
        return io_copy_in(s, st, cs);
    }
    // the order of base_copy_in: a FRESH_ONLY round this rank had not posted contributes
    // zeros and never reads (or zeroes) the send bucket the caller may be writing -- ahead
    // of ZERO_SB's fused move
    const void *src = nullptr;
    if (s.fresh_only && !fresh) src = nullptr;            // contributes zeros, sb unread
    else if (s.zero_sb) return move_zero(st.rb_dev, s.sb, bytes, cs);
    else if (!s.in_place) src = s.sb;
    else return ESGD_SUCCESS;                              // in place: nothing to move
    if (snap_eligible(s, st, src)) {   // phase 0 of the shared launch
        st.snap_kind = src ? 1 : 2;
        return ESGD_SUCCESS;
    }
    if (!src) ESGD_HIP(hipMemsetAsync(st.rb_dev, 0, bytes, cs));
    else ESGD_HIP(hipMemcpyAsync(st.rb_dev, src, bytes, hipMemcpyDeviceToDevice, cs));
    return ESGD_SUCCESS;
}

// The round joins the pending launch (its snapshot is queued on `cs` or deferred into the
// launch's copy kernel).
static int batch_append(Sched &s, IpcState &st, uint32_t round, hipStream_t cs) {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    if (!g_pend.empty() && (g_pend[0].s->dtype != s.dtype || g_pend[0].s->world != s.world ||
                            int64_t(g_pend.size()) >= batch_rounds()))
        batch_flush_locked();   // a failure is recorded in the rounds of that launch
    if (int rc = batch_desc(s, st, cs)) return rc;
    st.pub_round = round;
    st.fin_mode = true;
    st.batch_rc = 0;
    st.in_batch = true;
    const RoundIO none{nullptr, nullptr, 1.0f};
    g_pend.push_back({&s, &st, round, st.snap_kind, st.io_on ? st.cur_io : none});
    st.snap_kind = 0;
    return ESGD_SUCCESS;
}

static void batch_shutdown() {
    std::lock_guard<std::mutex> lk(g_batch_mu);
    (void)batch_flush_locked();
    for (auto &w : g_waited) {   // their events go back to the pool before it is emptied
        w.s = nullptr;
        w.ev.reset();
    }
    g_outstanding.clear();
    if (g_desc_dev) { hip_ignore(hipFree(g_desc_dev)); g_desc_dev = nullptr; g_slots = nullptr; }
    if (g_desc_host) { hip_ignore(hipHostFree(g_desc_host)); g_desc_host = nullptr; }
    std::lock_guard<std::mutex> ek(g_evfree_mu);
    for (hipEvent_t e : g_evfree) hip_ignore(hipEventDestroy(e));
    g_evfree.clear();
}

struct IpcTransport final : Transport {
    const char *name() const override { return "ipc"; }

    static IpcState &S(Sched &s) { return *static_cast<IpcState *>(s.tstate); }

    // size of this round's bucket, read by peers' size check (no re-map needed)
    static void publish_size(Sched &s) {
        s.sh->slot[s.rank].bytes = s.count * wire_esize(s);
    }

    // bytes per element of what peers read: the bf16 wire copy, or the bucket itself
    static size_t wire_esize(const Sched &s) { return s.wire_bf16 ? 2 : s.esize; }

    // Publish rb_dev (arena memory: the chunk's handle + the offset); ESGD_INVALID_ARG
    // when rb_dev is foreign memory, which is never exported.
    // Publish an arena buffer in this rank's slot (the chunk's handle + the offset);
    // ESGD_INVALID_ARG when `p` is foreign memory, which is never exported.
    static int publish_buf(Sched &s, IpcSlot &mine, char *p, size_t bytes, const char *what) {
        void *base = nullptr;
        uint64_t off = 0;
        uint8_t hb[64];
        SealInfo seal{0, 0, 0};
        if (int rc = arena_export(p, bytes, &base, &off, hb, &seal)) return rc;
        std::memcpy(mine.handle, hb, 64);
        mine.offset = off;
        mine.bytes = bytes;
        mine.chunk_bytes = seal.chunk_bytes;
        mine.chunk_base = seal.chunk_base;
        mine.seal_nonce = seal.nonce;
        mine.gen.store(s.gen, std::memory_order_release);
        mine.ver.fetch_add(1, std::memory_order_acq_rel);
        ESGD_TRACE("r%d publish sched %d %s %p chunk %p + %llu\n", s.rank, s.id, what, (void *)p, base,
                   (unsigned long long)off);
        return ESGD_SUCCESS;
    }

    // Publish a buffer this schedule owns.  When the runtime refuses to export its arena
    // chunk (arena_export marks the chunk; round 3 saw hipErrorInvalidValue for a fresh
    // process's first chunk now and then), the buffer is allocated again -- the arena no
    // longer carves from that chunk -- and the new one is published.  Contents need not
    // move: every caller publishes before the round that fills the buffer.
    static int publish_owned(Sched &s, IpcSlot &slot, char **buf, size_t *cap, size_t bytes, const char *what) {
        for (int attempt = 0;; ++attempt) {
            const int rc = publish_buf(s, slot, *buf, bytes, what);
            if (rc == ESGD_SUCCESS || attempt == 2 || !arena_unexportable(*buf)) return rc;
            char *old = *buf;
            const size_t want = *cap;
            if (int ra = alloc_bucket(want, buf, cap)) return ra;
            std::fprintf(stderr, "esgd: rank %d schedule %d: %s %p could not be exported, moved to %p\n", s.rank,
                         s.id, what, static_cast<void *>(old), static_cast<void *>(*buf));
            free_bucket(old);
        }
    }

    static int publish(Sched &s, IpcState &st) {
        if (s.wire_bf16) {   // peers read the wire copy; rb stays private (never shadowed)
            if (!st.wire)
                if (int rc = alloc_bucket(s.count * 2, &st.wire, &st.wire_cap)) return rc;
            const int rc = publish_owned(s, s.sh->slot[s.rank], &st.wire, &st.wire_cap, s.count * 2, "wire");
            st.peer[s.rank] = st.wire;
            return rc;
        }
        if (st.owns_rb) {
            const int rc = publish_owned(s, s.sh->slot[s.rank], &st.rb_dev, &st.cap, s.count * s.esize, "rb");
            st.peer[s.rank] = st.rb_dev;
            return rc;
        }
        st.peer[s.rank] = st.rb_dev;
        const int rc = publish_buf(s, s.sh->slot[s.rank], st.rb_dev, s.count * s.esize, "rb");
        // the caller's bucket sits in a chunk the runtime would not export: setup shadows
        // it, as it does foreign memory
        if (rc && arena_unexportable(st.rb_dev)) return ESGD_INVALID_ARG;
        return rc;
    }

    // rounds of this size run as one k_round_small launch
    static bool one_launch(const Sched &s) {
        return s.world > 1 && s.world <= ESGD_MAX_FANIN && !s.wire_bf16 && s.count * s.esize <= s.small_bytes;
    }

    // the published shard (one-launch rounds only): grown and re-published when the
    // largest shard outgrows it
    static int publish_pub(Sched &s, IpcState &st) {
        if (!one_launch(s)) return ESGD_SUCCESS;
        const size_t need = std::max<size_t>(st.len[0] * s.esize, 16);
        if (st.pub && need <= st.pub_cap) return ESGD_SUCCESS;
        if (st.pub) st.retired.push_back(st.pub);   // peers may still map it: back at teardown
        if (int rc = alloc_bucket(need, &st.pub, &st.pub_cap)) return rc;
        return publish_owned(s, s.sh->pub[s.rank], &st.pub, &st.pub_cap, st.pub_cap, "pub");
    }

    // (re)map one peer publication if it changed since we last mapped it; a fresh mapping
    // whose seal shows other memory asks peer q to move that publication (`bit` in
    // SchedShm::remap of this connect attempt; schedule creation retries)
    static int map_slot(Sched &s, int q, IpcSlot &ps, PeerMap &m, const char *what, uint32_t bit) {
        if (ps.gen.load(std::memory_order_acquire) != s.gen) {
            set_error("schedule %d: rank %d did not publish its %s", s.id, q, what);
            return ESGD_ERROR;
        }
        const uint32_t v = ps.ver.load(std::memory_order_acquire);
        if (m.base && v == m.ver) return ESGD_SUCCESS;   // nothing moved
        // a moved buffer may sit in the same arena chunk (same handle, new offset);
        // mappings are cached per (peer, chunk) and never closed before shutdown
        if (!(m.base && std::memcmp(m.handle, ps.handle, 64) == 0)) {
            void *pb = nullptr;
            if (int rc = ipc_open(q, ps.handle, &pb, &ps)) {
                if (t_seal_mismatch && s.connect_attempt <= kRemapTries)
                    s.sh->remap[s.connect_attempt][q].fetch_or(bit, std::memory_order_acq_rel);
                return rc;
            }
            m.base = pb;
            std::memcpy(m.handle, ps.handle, 64);
        }
        m.ptr = static_cast<char *>(m.base) + ps.offset;
        m.ver = v;
        return ESGD_SUCCESS;
    }

    // (re)map every peer's rb and published shard
    static int map_peers(Sched &s, IpcState &st) {
        const size_t bytes = s.count * wire_esize(s);
        for (int q = 0; q < s.world; ++q) {
            if (q == s.rank) continue;
            IpcSlot &ps = s.sh->slot[q];
            if (int rc = map_slot(s, q, ps, st.rbmap[q], "bucket", 1)) return rc;
            if (ps.bytes != bytes) {
                set_error("schedule %d: rank %d has %llu bytes, this rank %zu", s.id, q,
                          (unsigned long long)ps.bytes, bytes);
                return ESGD_INVALID_ARG;
            }
            st.peer[q] = st.rbmap[q].ptr;
            if (!one_launch(s)) continue;   // every rank has this size (checked above)
            if (int rc = map_slot(s, q, s.sh->pub[q], st.pubmap[q], "published shard", 2)) return rc;
            if (s.sh->pub[q].bytes < st.len[q] * s.esize) {
                set_error("schedule %d: rank %d's published shard is too small", s.id, q);
                return ESGD_ERROR;
            }
        }
        return ESGD_SUCCESS;
    }

    int setup(Sched &s) override {
        auto *st = new IpcState();
        s.tstate = st;
        if (int rc = base_setup(s, *st)) return rc;
        st->peer[s.rank] = st->rb_dev;
        if (s.world == 1) return ESGD_SUCCESS;
        if (s.wire_bf16 && s.resolve) {
            set_error("schedule: ESGD_SCHED_WIRE_BF16 does not take FFCOLL_BUFFERS buffers");
            return ESGD_INVALID_ARG;
        }
        if (int rc = register_segment()) return rc;
        if (s.flag_mode > 0)
            if (int rc = flags_publish(s.rank, s.flag_mode)) return rc;
        // publish this rank's rb (peers map it in connect())
        // ESGD_TEST shadow=1 shadows every device bucket (caller buckets that are freed and
        // re-allocated between rounds; also how the tests reach the fallback)
        static const bool force_shadow = test_knob("shadow", 0) == 1;
        if (int rc = publish_pub(s, *st)) return rc;
        if (s.host_mode || s.wire_bf16) return publish(s, *st);
        int rc = force_shadow ? ESGD_INVALID_ARG : publish(s, *st);
        if (rc == ESGD_INVALID_ARG) {
            // foreign device memory (torch tensors, plain hipMalloc) is never exported:
            // reduce through an arena bucket, copied in at the snapshot, out at the finish
            ESGD_TRACE("r%d sched %d: bucket %p is not arena memory, shadowing it\n", s.rank, s.id,
                       (void *)st->rb_dev);
            if ((rc = alloc_bucket(s.count * s.esize, &st->rb_dev, &st->cap))) return rc;
            st->owns_rb = st->shadow = true;
            st->peer[s.rank] = st->rb_dev;
            rc = publish(s, *st);
        }
        return rc;
    }

    int connect(Sched &s) override {
        if (s.world == 1) return ESGD_SUCCESS;
        if (s.flag_mode > 0)
            if (int rc = flags_connect(s.rank, s.world, s.flag_mode)) return rc;
        return map_peers(s, S(s));
    }

    // A peer's fresh mapping of this rank's publication showed other memory: whatever was
    // published from that chunk moves to a chunk allocated now (a new handle), contents
    // need not move (creation: no round has run).  The caller's own bucket cannot move --
    // it is shadowed instead, as a bucket in a refused chunk is.  The old block is left
    // allocated (quarantined): back on the free lists it could carry a later publication
    // of this rank through the same chunk handle, whose mapping went wrong once.
    int remap(Sched &s, uint32_t which) override {
        IpcState &st = S(s);
        auto move = [&](IpcSlot &slot, char **buf, size_t *cap, size_t bytes, const char *what) -> int {
            char *old = *buf;
            if (int rc = arena_alloc(std::max<size_t>(*cap, 1), reinterpret_cast<void **>(buf), false, true)) return rc;
            std::fprintf(stderr, "esgd: rank %d schedule %d: %s %p re-published from a new chunk at %p (the old "
                         "block quarantined)\n", s.rank, s.id, what, static_cast<void *>(old), static_cast<void *>(*buf));
            return publish_owned(s, slot, buf, cap, bytes, what);
        };
        // the published shard moves whichever was asked: it may share the suspect chunk
        if (st.pub && which)
            if (int rc = move(s.sh->pub[s.rank], &st.pub, &st.pub_cap, st.pub_cap, "pub")) return rc;
        if (which & 1) {
            IpcSlot &mine = s.sh->slot[s.rank];
            if (s.wire_bf16) {
                if (int rc = move(mine, &st.wire, &st.wire_cap, s.count * 2, "wire")) return rc;
                st.peer[s.rank] = st.wire;
            } else if (st.owns_rb) {
                if (int rc = move(mine, &st.rb_dev, &st.cap, s.count * s.esize, "rb")) return rc;
                st.peer[s.rank] = st.rb_dev;
            } else {   // the caller's bucket: reduce through a shadow in a new chunk
                if (int rc = arena_alloc(std::max<size_t>(s.count * s.esize, 1), reinterpret_cast<void **>(&st.rb_dev),
                                         false, true))
                    return rc;
                st.cap = std::max<size_t>(s.count * s.esize, 1);
                st.owns_rb = st.shadow = true;
                st.peer[s.rank] = st.rb_dev;
                std::fprintf(stderr, "esgd: rank %d schedule %d: bucket %p shadowed by %p in a new chunk\n", s.rank,
                             s.id, s.rb, static_cast<void *>(st.rb_dev));
                if (int rc = publish(s, st)) return rc;
            }
            st.desc_built = false;
        }
        return ESGD_SUCCESS;
    }

    int note_producer(Sched &s, uint32_t round, void *stream) override {
        return base_note_producer(S(s), round, stream);
    }

    int note_consumer(Sched &s, void *stream) override { return base_note_consumer(S(s), stream); }

    int note_io(Sched &s, uint32_t round, const RoundIO &io) override { return base_note_io(s, S(s), round, io); }

    // join: a moved bucket is re-published before this rank's join counts (peers map it
    // when they launch the round); a size change alone only updates the published size
    int prepare(Sched &s, uint32_t round, bool fresh) override {
        IpcState &st = S(s);
        const int moved = base_refit(s, st);
        if (moved < 0) return moved;
        if (s.world > 1 && moved)
            if (int rc = publish(s, st)) return rc;
        if (s.world > 1 && s.resolve) {
            publish_size(s);
            if (int rc = publish_pub(s, st)) return rc;   // larger shards need a larger pub
        }
        st.peer[s.rank] = s.wire_bf16 ? st.wire : st.rb_dev;   // what peers read
        ESGD_TRACE("r%d sched %d round %u join count=%llu rb_dev=%p moved=%d staged=%d\n", s.rank, s.id,
                   round, (unsigned long long)s.count, (void *)st.rb_dev, moved, int(staged(s, st)));
        return base_prepare(s, st, fresh);
    }

    // The whole round, queued on the round stream:
    //   move -> [pair: ready] -> reduce-scatter (tree kernel over peer HBM)
    //        -> [pair: reduced] -> all-gather -> [pair: done] -> copy-out -> event.
    // The last pairing keeps this rank's shard unchanged until every peer has gathered
    // it (the caller may overwrite rb once wait() returns).  Buckets up to
    // small_round_bytes() run as one k_round_small launch instead (launch_small: two
    // pairings, the gather reads the published shards).
    // rounds that go out in a shared k_round_batch launch
    static bool batched(const Sched &s, const IpcState &st) {
        // (a post_iov round ends with its unpack on the round stream: a launch of its own)
        return one_launch(s) && !s.host_mode && !st.shadow && !s.resolve && batch_rounds() > 1 &&
               !(st.io_on && st.cur_io.segs) &&
               !gpu_trace_on() && st.len[0] * s.esize <= (uint64_t(1) << 30);
    }

    int launch(Sched &s, uint32_t round, bool fresh) override {
        IpcState &st = S(s);
        hipStream_t cs = st.stream;
        st.fin_mode = false;
        st.batch_ev.reset();
        st.batch_rc = 0;
        st.in_batch = false;
        take_io(st, round, fresh);
        const bool batch = batched(s, st);
        // anything else queued on the round stream goes behind the pending shared launch
        if (!batch)
            if (int rc = dataplane_flush()) return rc;
        if (s.host_mode && !s.resolve && !s.wire_bf16 && host_chunk_bytes() &&
            s.count * s.esize >= 2 * host_chunk_bytes())
            return launch_chunked(s, st, round, fresh);
        if (s.wire_bf16 && s.world > 1 && !s.host_mode) {
            // wire rounds of device buckets: the snapshot is the narrowing itself (sb, or rb
            // in place, -> wire copy); rb is entirely rewritten by the two phases
            if (int rc = consumer_wait(st, cs)) return rc;
            if (int rc = producer_wait(st, round, fresh, cs)) return rc;
        } else if (batch) {
            if (int rc = batch_snapshot(s, st, round, fresh, cs)) return rc;
        } else if (int rc = base_copy_in(s, st, round, fresh, cs)) {
            return rc;
        }
        if (s.world > 1) {
            if (s.resolve)
                if (int rc = map_peers(s, st)) return rc;
            if (one_launch(s)) {
                if (batch) return batch_append(s, st, round, cs);
                ++g_launches;
                if (int rc = launch_small(s, st, round, cs)) return rc;
                // device buckets: nothing follows the kernel, the host polls its fin flag
                // (the event only reports faults)
                if (!s.host_mode && !st.shadow && !st.io_on) {
                    st.fin_mode = true;
                    ESGD_HIP(hipEventRecord(st.ev, cs));
                    return ESGD_SUCCESS;
                }
                return base_copy_out(s, st, cs);
            }
            ++g_launches;
            const bool io_direct = st.io_on && !st.cur_io.segs && !s.host_mode && !st.shadow && !s.wire_bf16;
            if (s.wire_bf16) {
                if (int rc = wire_phases(s, st, round, fresh, cs)) return rc;
            } else {
            if (int rc = pair_ranks(s, s.sh->ready, 0, round, cs)) return rc;
            // Launches move at most kPiece bytes per input / segment (the kernels address
            // a shard through 32-bit buffer offsets); buckets up to the reference's
            // 2^31 - 1 elements (ff.h: int count) at any P are cut into pieces.
            const size_t es = s.esize;
            const uint64_t piece = piece_bytes() / es;
            const uint64_t n = st.len[s.rank];
            for (uint64_t o = 0; o < n; o += piece) {
                const uint64_t c = std::min(piece, n - o);
                const void *in[kMaxRanks];
                for (int j = 0; j < s.world; ++j) in[j] = st.peer[j] + (st.off[s.rank] + o) * es;
                if (int rc = reduce_remote(s.dtype, s.world, in, st.rb_dev + (st.off[s.rank] + o) * es, c,
                                           1.0f, cs))
                    return rc;
            }
            if (int rc = pair_ranks(s, s.sh->reduced, 1, round, cs)) return rc;
            // a round with its own output (post_io) gathers straight into it, its own
            // reduced shard too (one more segment of the same launch): no copy-out
            char *gbase = io_direct ? static_cast<char *>(st.cur_io.dst) : st.rb_dev;
            const void *src[kMaxSegs];
            void *dst[kMaxSegs];
            uint64_t bytes[kMaxSegs];
            int m = 0;
            for (int j = 0; j < s.world; ++j) {
                if (j == s.rank && !io_direct) continue;
                for (uint64_t o = 0; o < st.len[j]; o += piece) {
                    src[m] = (j == s.rank ? st.rb_dev : st.peer[j]) + (st.off[j] + o) * es;
                    dst[m] = gbase + (st.off[j] + o) * es;
                    bytes[m] = std::min(piece, st.len[j] - o) * es;
                    if (++m == kMaxSegs) {
                        if (int rc = gather_remote(m, src, dst, bytes, cs)) return rc;
                        m = 0;
                    }
                }
            }
            if (m)
                if (int rc = gather_remote(m, src, dst, bytes, cs)) return rc;
            }
            // device buckets: the done pairing ends the round and reports it in fin, which
            // the host polls (as for one-launch rounds; the event only reports faults)
            const bool last = !s.host_mode && !st.shadow && (!st.io_on || io_direct);
            if (int rc = pair_ranks(s, s.sh->done, 2, round, cs, 0, last ? &s.sh->fin[s.rank] : nullptr))
                return rc;
            if (last) {
                st.fin_mode = true;
                ESGD_HIP(hipEventRecord(st.ev, cs));
                return ESGD_SUCCESS;
            }
        }
        return base_copy_out(s, st, cs);
    }

    // Both phases of a wire-mode round (ESGD_SCHED_WIRE_BF16), up to the done pairing:
    //   wire = bf16(rb) -> [pair: ready] -> phase 1: shard `rank` of every rank's wire copy
    //   (peer HBM), folded in fp32, rounded once -> own wire shard (bf16) + rb shard (fp32)
    //   -> [pair: reduced] -> phase 2: every other rank's reduced wire shard, widened into rb.
    // Peers read S/2 bytes per phase and rank pair instead of S: half the xGMI traffic, for
    // one more local pass (4 B read + 2 B written per element).  The done pairing that
    // follows keeps the wire copy unchanged until every peer has gathered from it.
    static int wire_phases(Sched &s, IpcState &st, uint32_t round, bool fresh, hipStream_t cs) {
        // device buckets: straight from the send bucket (zeroing it if asked); host buckets
        // were copied into rb by the snapshot; FRESH_ONLY rounds this rank had not posted
        // contribute zeros (nothing read)
        const bool from_sb = !s.host_mode && !s.in_place;
        if (s.fresh_only && !fresh && !s.host_mode) {
            ESGD_HIP(hipMemsetAsync(st.wire, 0, s.count * 2, cs));
        } else {
            float *nsrc = reinterpret_cast<float *>(from_sb ? static_cast<char *>(s.sb) : st.rb_dev);
            if (int rc = narrow_bf16(nsrc, reinterpret_cast<uint16_t *>(st.wire), s.count, from_sb && s.zero_sb, cs))
                return rc;
        }
        if (int rc = pair_ranks(s, s.sh->ready, 0, round, cs)) return rc;
        const uint64_t piece = piece_bytes() / 4;   // elements, as for fp32 rounds
        const int r = s.rank;
        for (uint64_t o = 0; o < st.len[r]; o += piece) {
            const uint64_t c = std::min(piece, st.len[r] - o);
            const void *in[kMaxRanks];
            for (int j = 0; j < s.world; ++j) in[j] = st.peer[j] + (st.off[r] + o) * 2;
            if (int rc = reduce_wire(s.world, in, reinterpret_cast<uint16_t *>(st.wire + (st.off[r] + o) * 2),
                                     reinterpret_cast<float *>(st.rb_dev + (st.off[r] + o) * 4), c, cs))
                return rc;
        }
        if (int rc = pair_ranks(s, s.sh->reduced, 1, round, cs)) return rc;
        const void *src[kMaxSegs];
        void *dst[kMaxSegs];
        uint64_t cnt[kMaxSegs];
        int m = 0;
        for (int j = 0; j < s.world; ++j) {
            if (j == r) continue;
            for (uint64_t o = 0; o < st.len[j]; o += piece) {
                src[m] = st.peer[j] + (st.off[j] + o) * 2;
                dst[m] = st.rb_dev + (st.off[j] + o) * 4;
                cnt[m] = std::min(piece, st.len[j] - o);
                if (++m == kMaxSegs) {
                    if (int rc = gather_widen(m, src, dst, cnt, cs)) return rc;
                    m = 0;
                }
            }
        }
        return m ? gather_widen(m, src, dst, cnt, cs) : ESGD_SUCCESS;
    }

    // Host buckets (the reference's contract) of >= 2 chunks: the round runs chunk by
    // chunk so that the copies overlap -- chunk c's H2D (copy stream 1) -> on the round
    // stream [pair: ready] reduce-scatter [pair: reduced] all-gather [pair: done] of
    // chunk c, each chunk split into P shards like a whole bucket -> chunk c's D2H (copy
    // stream 2), while chunk c+1 is uploaded.  Pairing values number the chunks,
    // (round - 1) * C + c + 1, so they keep increasing (C is fixed: the bucket size of a
    // non-FFCOLL_BUFFERS schedule never changes).  A chunk is overwritten by the next
    // round's H2D only after this round's D2H of it, which follows its done pairing
    // (no peer still reads it).  Sums are element-wise, so the result is bit-identical
    // to the one-piece round.
    static int launch_chunked(Sched &s, IpcState &st, uint32_t round, bool fresh) {
        hipStream_t cs = st.stream, hs = nullptr, ds = nullptr;
        if (int rc = copy_streams(&hs, &ds)) return rc;
        if (int rc = consumer_wait(st, hs)) return rc;
        if (int rc = producer_wait(st, round, fresh, hs)) return rc;
        const size_t es = s.esize;
        const uint64_t count = s.count, align = 1024;   // elements: 1 KiB+ aligned chunks
        const uint64_t want = std::min<uint64_t>(64, (count * es + host_chunk_bytes() - 1) / host_chunk_bytes());
        uint64_t Q = (count + want - 1) / want;
        Q = (Q + align - 1) / align * align;
        const uint32_t C = uint32_t((count + Q - 1) / Q);
        while (st.cev.size() < 3 * size_t(C)) {
            hipEvent_t e;
            ESGD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            st.cev.push_back(e);
        }
        const bool stg = staged(s, st);
        const char *src = stg ? st.pin : static_cast<const char *>(s.sb ? s.sb : s.rb);
        char *dst = stg ? st.pin : static_cast<char *>(s.rb);
        const uint64_t salign = 1024 / es;
        for (uint32_t c = 0; c < C; ++c) {
            const uint64_t c0 = uint64_t(c) * Q, n = std::min(Q, count - c0);
            hipEvent_t eh = st.cev[3 * c], er = st.cev[3 * c + 1], ed = st.cev[3 * c + 2];
            if (st.chunked_before) ESGD_HIP(hipStreamWaitEvent(hs, ed, 0));   // last round's D2H
            if (s.fresh_only && !fresh) {   // not posted: zeros, the host bucket is not read
                ESGD_HIP(hipMemsetAsync(st.rb_dev + c0 * es, 0, n * es, hs));
            } else {
                ESGD_HIP(hipMemcpyAsync(st.rb_dev + c0 * es, src + c0 * es, n * es, hipMemcpyHostToDevice, hs));
            }
            ESGD_HIP(hipEventRecord(eh, hs));
            ESGD_HIP(hipStreamWaitEvent(cs, eh, 0));
            if (s.world > 1) {
                uint64_t per = (n + uint64_t(s.world) - 1) / uint64_t(s.world);
                per = (per + salign - 1) / salign * salign;
                uint64_t off[kMaxRanks], len[kMaxRanks];
                for (int j = 0; j < s.world; ++j) {
                    const uint64_t o = std::min<uint64_t>(n, per * uint64_t(j));
                    off[j] = c0 + o;
                    len[j] = std::min<uint64_t>(per, n - o);
                }
                const uint32_t v = (round - 1) * C + c + 1;
                if (int rc = pair_ranks(s, s.sh->ready, 0, round, cs, v)) return rc;
                if (len[s.rank]) {
                    const void *in[kMaxRanks];
                    for (int j = 0; j < s.world; ++j) in[j] = st.peer[j] + off[s.rank] * es;
                    if (int rc = reduce_remote(s.dtype, s.world, in, st.rb_dev + off[s.rank] * es, len[s.rank],
                                               1.0f, cs))
                        return rc;
                }
                if (int rc = pair_ranks(s, s.sh->reduced, 1, round, cs, v)) return rc;
                const void *gs[kMaxSegs];
                void *gd[kMaxSegs];
                uint64_t gb[kMaxSegs];
                int m = 0;
                for (int j = 0; j < s.world; ++j) {
                    if (j == s.rank || !len[j]) continue;
                    gs[m] = st.peer[j] + off[j] * es;
                    gd[m] = st.rb_dev + off[j] * es;
                    gb[m++] = len[j] * es;
                }
                if (int rc = gather_remote(m, gs, gd, gb, cs)) return rc;
                if (int rc = pair_ranks(s, s.sh->done, 2, round, cs, v)) return rc;
            }
            ESGD_HIP(hipEventRecord(er, cs));
            ESGD_HIP(hipStreamWaitEvent(ds, er, 0));
            ESGD_HIP(hipMemcpyAsync(dst + c0 * es, st.rb_dev + c0 * es, n * es, hipMemcpyDeviceToHost, ds));
            ESGD_HIP(hipEventRecord(ed, ds));
        }
        ESGD_HIP(hipStreamWaitEvent(cs, st.cev[3 * (C - 1) + 2], 0));   // ds is in order
        st.copyout_pending = stg;
        st.chunked_before = true;
        return finish_round(s, st, cs);
    }

    // the whole round as one k_round_small launch (small buckets)
    static int launch_small(Sched &s, IpcState &st, uint32_t round, hipStream_t cs) {
        if (!st.ctr)   // first one-launch round of this schedule
            if (int rc = ctr_words(s.id, cs, &st.ctr)) return rc;
        st.pub_round = round;
        const void *in[kMaxRanks];
        for (int j = 0; j < s.world; ++j) in[j] = st.peer[j] + st.off[s.rank] * s.esize;
        const void *src[kMaxRanks];
        void *dst[kMaxRanks];
        uint64_t bytes[kMaxRanks];
        int m = 0;
        for (int j = 0; j < s.world; ++j) {
            if (j == s.rank || st.len[j] == 0) continue;
            src[m] = st.pubmap[j].ptr;   // peer j's published shard j
            dst[m] = st.rb_dev + st.off[j] * s.esize;
            bytes[m] = st.len[j] * s.esize;
            ++m;
        }
        const long long ticks = (long long)(engine_timeout() * double(g_ticks_per_s));
        uint64_t *ts = gpu_trace_on() ? reinterpret_cast<uint64_t *>(dev_flag(&s.sh->gpu_ts[s.rank][0])) : nullptr;
        return round_small(s.dtype, in, st.rb_dev + st.off[s.rank] * s.esize, st.pub, st.len[s.rank], m, src,
                           dst, bytes, pair_flags(s, s.sh->ready, 0), pair_flags(s, s.sh->reduced, 1),
                           (s.host_mode || st.shadow || st.io_on) ? nullptr : dev_flag(&s.sh->fin[s.rank]),
                           dev_flag(&s.sh->gpu_err[s.rank]), ts, st.ctr,
                           s.rank, s.world, round, ticks, s.strict ? 1 : 0, cs);
    }

    int query(Sched &s) override { return base_query(s, S(s)); }

    int complete(Sched &s) override { return base_complete(s, S(s)); }

    std::string diagnose(Sched &s) override { return base_diagnose(s); }

    // Deletion is local: peers may still be gathering this rank's published shard of the
    // last round (they passed the same `reduced` pairing; their gather is queued right
    // behind it).  pub goes back to the arena once every peer's fin shows that round;
    // if a peer never gets there (it failed), pub is kept out of the arena instead.
    void teardown(Sched &s) override {
        IpcState *st = static_cast<IpcState *>(s.tstate);
        if (!st) return;
        if (st->stream) hip_ignore(hipStreamSynchronize(st->stream));
        for (hipEvent_t e : st->cev) hip_ignore(hipEventDestroy(e));
        bool pub_free = true;
        if (st->pub && st->pub_round && s.world > 1) {
            const double t0 = now_s(), limit = std::min(engine_timeout(), 10.0);
            for (int q = 0; q < s.world && pub_free; ++q) {
                if (q == s.rank) continue;
                while (int32_t(s.sh->fin[q].load(std::memory_order_acquire) - st->pub_round) < 0) {
                    if (now_s() - t0 > limit) { pub_free = false; break; }
                    std::this_thread::yield();
                }
            }
            if (!pub_free)
                ESGD_TRACE("r%d sched %d: a peer never finished round %u, its published shard is kept\n",
                           s.rank, s.id, st->pub_round);
        }
        if (close_on_delete())
            for (int q = 0; q < s.world; ++q) {
                if (q == s.rank) continue;
                if (st->rbmap[q].base) ipc_close_one(q, st->rbmap[q].handle);
                if (st->pubmap[q].base) ipc_close_one(q, st->pubmap[q].handle);
            }
        if (st->pub && pub_free) free_bucket(st->pub);
        if (st->wire) free_bucket(st->wire);   // the done pairing: no peer still reads it
        if (!pub_free) st->retired.clear();   // earlier pubs too: a peer may be stuck on any
        base_teardown(s, *st);
        delete st;
        s.tstate = nullptr;
    }
};

struct NullTransport final : Transport {
    explicit NullTransport(bool ord = false) : ordered_(ord) {}
    bool ordered_;   // the "rccl" flavour (same protocol; named for the issue-order tests)
    const char *name() const override { return ordered_ ? "none-ordered" : "none"; }
    int setup(Sched &) override { return ESGD_SUCCESS; }
    // ESGD_TEST fail_connect=<rank>: that rank's connect fails (control-plane tests of the
    // creation protocol; this transport moves no data)
    int connect(Sched &s) override {
        if (test_knob("fail_connect", -1) == s.rank) {
            set_error("connect failed on rank %d (ESGD_TEST fail_connect)", s.rank);
            return ESGD_ERROR;
        }
        return ESGD_SUCCESS;
    }
    int note_producer(Sched &, uint32_t, void *) override { return ESGD_SUCCESS; }
    int prepare(Sched &, uint32_t, bool) override { return ESGD_SUCCESS; }
    int launch(Sched &, uint32_t, bool) override { return ESGD_SUCCESS; }
    int query(Sched &) override { return 1; }
    void teardown(Sched &) override {}
};

Transport *ipc_transport() {
    static IpcTransport t;
    return &t;
}

Transport *null_transport(bool ordered) {
    static NullTransport plain(false), ord(true);
    return ordered ? &ord : &plain;
}

Transport *rccl_transport();

hipStream_t sched_stream(Sched &s) {
    if (!s.tstate || (s.tp != ipc_transport() && s.tp != rccl_transport())) return nullptr;
    return static_cast<BaseState *>(s.tstate)->stream;
}

// ---- RcclTransport: RCCL point-to-point over xGMI + the tree kernel on a side stream --
//
// The north-star shape of SURVEY.md §8(e): per round, on ONE process-wide communicator
// stream, grouped ncclSend/ncclRecv move shard j of this rank's rb to rank j and every
// peer's copy of shard `rank` into a staging area, chunk by chunk; the schedule's own
// stream waits for each chunk and folds it with the tree kernel (same order as the
// reference); a second group all-gathers the reduced shards.  RCCL matches operations
// by issue order: the engine launches rounds in the node's issue-ring order, on the
// process's round stream, which is also the communicator stream.
// RCCL refuses two ranks on one GPU, so this transport only runs with one GPU per rank.
// ESGD_SCHED_WIRE_BF16 rounds move bf16 copies: rb is narrowed into a wire bucket, the
// reduce-scatter groups carry bf16 shards, the fold is the wire tree kernel (same kernel
// and operand order as IpcTransport::wire_phases, so both transports give the same bits)
// and the all-gather carries the reduced bf16 shards, widened into rb.
}  // namespace esgd

#include <rccl/rccl.h>

namespace esgd {

static std::mutex g_nccl_mu;
static ncclComm_t g_nccl = nullptr;

static int nccl_fail(ncclResult_t r, const char *what) {
    set_error("%s: %s", what, ncclGetErrorString(r));
    return ESGD_ERROR;
}
#define ESGD_NCCL(call)                                                       \
    do {                                                                      \
        ncclResult_t esgd_r_ = (call);                                        \
        if (esgd_r_ != ncclSuccess) return nccl_fail(esgd_r_, #call);         \
    } while (0)

static int nccl_ensure(Sched &s) {
    std::lock_guard<std::mutex> lk(g_nccl_mu);
    if (g_nccl) return ESGD_SUCCESS;
    Segment *seg = engine_segment();
    ncclUniqueId id;
    static_assert(sizeof(id) <= sizeof(seg->nccl_id), "nccl id does not fit the segment");
    if (s.rank == 0) {
        ESGD_NCCL(ncclGetUniqueId(&id));
        std::memcpy(seg->nccl_id, &id, sizeof(id));
    }
    if (int rc = engine_barrier()) return rc;   // connect() runs on every rank
    std::memcpy(&id, seg->nccl_id, sizeof(id));
    ESGD_NCCL(ncclCommInitRank(&g_nccl, s.world, id, s.rank));
    return ESGD_SUCCESS;
}

void rccl_shutdown() {
    std::lock_guard<std::mutex> lk(g_nccl_mu);
    if (g_rs) hip_ignore(hipStreamSynchronize(g_rs));
    if (g_nccl) { (void)ncclCommDestroy(g_nccl); g_nccl = nullptr; }
}

struct RcclState : BaseState {
    hipStream_t red = nullptr;       // tree folds of arrived chunks
    char *stage = nullptr;           // P x L elements: every peer's copy of this rank's shard
    char *wire = nullptr;            // wire rounds: bf16 copy of rb (count elements)
    size_t stage_cap = 0, wire_cap = 0;   // bytes of the arena blocks behind stage / wire
    uint64_t wire_n = 0;
    uint64_t L = 0;                  // shard pitch (elements)
    uint64_t chunk = 0;              // pipeline chunk (elements)
    hipEvent_t ev_red = nullptr;
    std::vector<hipEvent_t> ev_chunk;
};

struct RcclTransport final : Transport {
    const char *name() const override { return "rccl"; }

    static RcclState &S(Sched &s) { return *static_cast<RcclState *>(s.tstate); }

    // bytes per element on the wire (and in the staging area)
    static size_t stage_esize(const Sched &s) { return s.wire_bf16 ? 2 : s.esize; }

    // A buffer of at least `need` bytes in *buf (capacity *cap): grown geometrically from
    // the arena, never shrunk.  Called at setup (caller's thread) and at every join of an
    // FFCOLL_BUFFERS round (the progress thread): the arena hands out and takes back blocks
    // without hipFree -- whose device-wide synchronisation would stall every schedule's
    // rounds in flight -- and the old block is free to go: a join follows the schedule's
    // previous round, which was the last user of it.
    static int fit_buf(char **buf, size_t *cap, size_t need) {
        if (need <= *cap) return ESGD_SUCCESS;
        char *p = nullptr;
        const size_t want = std::max(need, 2 * *cap);
        if (int rc = arena_alloc(want, reinterpret_cast<void **>(&p))) return rc;
        if (*buf) arena_free(*buf);
        *buf = p;
        *cap = want;
        return ESGD_SUCCESS;
    }

    static int fit_stage(Sched &s, RcclState &st) {
        if (s.wire_bf16 && s.world > 1 && st.wire_n != s.count) {
            if (int rc = fit_buf(&st.wire, &st.wire_cap, size_t(s.count) * 2)) return rc;
            st.wire_n = s.count;
        }
        // pitch rounded to 8 elements: every staged shard starts 16-B aligned (the wire
        // kernels' vectors) even when one ragged shard holds the whole bucket
        const uint64_t pitch = (st.len[0] + 7) / 8 * 8;
        if (st.stage && st.L == pitch) return ESGD_SUCCESS;
        st.L = pitch;
        if (s.world > 1 && st.L)
            if (int rc = fit_buf(&st.stage, &st.stage_cap, size_t(s.world) * st.L * stage_esize(s))) return rc;
        // ~8 chunks per shard, at least 1 MiB each, 1 KiB aligned
        const uint64_t align = 1024 / s.esize, minc = (1u << 20) / s.esize;
        const uint64_t c = std::max<uint64_t>(minc, (st.L + 7) / 8);
        st.chunk = (c + align - 1) / align * align;
        return ESGD_SUCCESS;
    }

    int setup(Sched &s) override {
        auto *st = new RcclState();
        s.tstate = st;
        if (int rc = base_setup(s, *st)) return rc;
        if (s.wire_bf16 && s.resolve && s.world > 1) {
            set_error("schedule: ESGD_SCHED_WIRE_BF16 does not take FFCOLL_BUFFERS buffers");
            return ESGD_INVALID_ARG;
        }
        ESGD_HIP(hipStreamCreateWithFlags(&st->red, hipStreamNonBlocking));
        ESGD_HIP(hipEventCreateWithFlags(&st->ev_red, hipEventDisableTiming));
        return fit_stage(s, *st);
    }

    int connect(Sched &s) override { return nccl_ensure(s); }

    int note_producer(Sched &s, uint32_t round, void *stream) override {
        return base_note_producer(S(s), round, stream);
    }

    int note_consumer(Sched &s, void *stream) override { return base_note_consumer(S(s), stream); }

    int note_io(Sched &s, uint32_t round, const RoundIO &io) override { return base_note_io(s, S(s), round, io); }

    int prepare(Sched &s, uint32_t, bool fresh) override {
        RcclState &st = S(s);
        const int moved = base_refit(s, st);
        if (moved < 0) return moved;
        if (int rc = fit_stage(s, st)) return rc;
        return base_prepare(s, st, fresh);
    }

    static uint64_t piece(uint64_t len, uint64_t c, uint64_t chunk) {
        const uint64_t o = c * chunk;
        return o >= len ? 0 : std::min(chunk, len - o);
    }

    // The whole round, in issue order on the round stream: move -> RS groups, each
    // chunk folded with the tree kernel on the side stream as it lands -> AG group ->
    // copy-out -> event.
    int launch(Sched &s, uint32_t round, bool fresh) override {
        RcclState &st = S(s);
        hipStream_t cs = st.stream;
        const int P = s.world, r = s.rank;
        const size_t es = s.esize;
        if (int rc = dataplane_flush()) return rc;   // ring order on the round stream
        take_io(st, round, fresh);
        if (int rc = base_copy_in(s, st, round, fresh, cs)) return rc;
        if (P > 1 && st.L && s.wire_bf16) {
            if (int rc = wire_round(s, st)) return rc;
        } else if (P > 1 && st.L) {
            const uint64_t nch = (st.L + st.chunk - 1) / st.chunk;
            while (st.ev_chunk.size() < nch) {
                hipEvent_t e;
                ESGD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                st.ev_chunk.push_back(e);
            }
            for (uint64_t c = 0; c < nch; ++c) {
                ESGD_NCCL(ncclGroupStart());
                for (int j = 0; j < P; ++j) {
                    if (j == r) continue;
                    const uint64_t ns = piece(st.len[j], c, st.chunk);
                    if (ns) ESGD_NCCL(ncclSend(st.rb_dev + (st.off[j] + c * st.chunk) * es, ns * es,
                                               ncclChar, j, g_nccl, cs));
                    const uint64_t nr = piece(st.len[r], c, st.chunk);
                    if (nr) ESGD_NCCL(ncclRecv(st.stage + (uint64_t(j) * st.L + c * st.chunk) * es,
                                               nr * es, ncclChar, j, g_nccl, cs));
                }
                ESGD_NCCL(ncclGroupEnd());
                ESGD_HIP(hipEventRecord(st.ev_chunk[c], cs));
                const uint64_t n = piece(st.len[r], c, st.chunk);
                if (!n) continue;
                ESGD_HIP(hipStreamWaitEvent(st.red, st.ev_chunk[c], 0));
                const void *in[kMaxRanks];
                char *own = st.rb_dev + (st.off[r] + c * st.chunk) * es;
                for (int j = 0; j < P; ++j)
                    in[j] = j == r ? own : st.stage + (uint64_t(j) * st.L + c * st.chunk) * es;
                if (int rc = esgd_reduce(s.dtype, P, in, own, n, st.red)) return rc;
            }
            ESGD_HIP(hipEventRecord(st.ev_red, st.red));
            ESGD_HIP(hipStreamWaitEvent(cs, st.ev_red, 0));
            ESGD_NCCL(ncclGroupStart());
            for (int j = 0; j < P; ++j) {
                if (j == r) continue;
                if (st.len[r]) ESGD_NCCL(ncclSend(st.rb_dev + st.off[r] * es, st.len[r] * es, ncclChar, j,
                                                  g_nccl, cs));
                if (st.len[j]) ESGD_NCCL(ncclRecv(st.rb_dev + st.off[j] * es, st.len[j] * es, ncclChar, j,
                                                  g_nccl, cs));
            }
            ESGD_NCCL(ncclGroupEnd());
        }
        return base_copy_out(s, st, cs);
    }

    // A wire round after the copy-in (rb = this rank's contribution): rb -> bf16 wire
    // copy; per chunk, bf16 shard j to rank j and every peer's bf16 copy of shard `rank`
    // into the staging area, folded by the wire tree kernel in rank order (own operand
    // from the wire copy, so every rank sums the same rounded inputs) into the own wire
    // shard (bf16, in place) and rb's shard (its widened value); then the reduced bf16
    // shards are all-gathered into the wire copy and widened into rb.
    static int wire_round(Sched &s, RcclState &st) {
        hipStream_t cs = st.stream;
        const int P = s.world, r = s.rank;
        uint16_t *w = reinterpret_cast<uint16_t *>(st.wire);
        float *rbf = reinterpret_cast<float *>(st.rb_dev);
        uint16_t *stg = reinterpret_cast<uint16_t *>(st.stage);
        if (int rc = narrow_bf16(rbf, w, s.count, false, cs)) return rc;
        const uint64_t nch = (st.L + st.chunk - 1) / st.chunk;
        while (st.ev_chunk.size() < nch) {
            hipEvent_t e;
            ESGD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            st.ev_chunk.push_back(e);
        }
        for (uint64_t c = 0; c < nch; ++c) {
            const uint64_t o = c * st.chunk;
            ESGD_NCCL(ncclGroupStart());
            for (int j = 0; j < P; ++j) {
                if (j == r) continue;
                const uint64_t ns = piece(st.len[j], c, st.chunk);
                if (ns) ESGD_NCCL(ncclSend(w + st.off[j] + o, ns * 2, ncclChar, j, g_nccl, cs));
                const uint64_t nr = piece(st.len[r], c, st.chunk);
                if (nr) ESGD_NCCL(ncclRecv(stg + uint64_t(j) * st.L + o, nr * 2, ncclChar, j, g_nccl, cs));
            }
            ESGD_NCCL(ncclGroupEnd());
            ESGD_HIP(hipEventRecord(st.ev_chunk[c], cs));
            const uint64_t n = piece(st.len[r], c, st.chunk);
            if (!n) continue;
            ESGD_HIP(hipStreamWaitEvent(st.red, st.ev_chunk[c], 0));
            const void *in[kMaxRanks];
            for (int j = 0; j < P; ++j)
                in[j] = j == r ? static_cast<const void *>(w + st.off[r] + o)
                               : static_cast<const void *>(stg + uint64_t(j) * st.L + o);
            if (int rc = reduce_wire(P, in, w + st.off[r] + o, rbf + st.off[r] + o, n, st.red)) return rc;
        }
        ESGD_HIP(hipEventRecord(st.ev_red, st.red));
        ESGD_HIP(hipStreamWaitEvent(cs, st.ev_red, 0));
        ESGD_NCCL(ncclGroupStart());
        for (int j = 0; j < P; ++j) {
            if (j == r) continue;
            if (st.len[r]) ESGD_NCCL(ncclSend(w + st.off[r], st.len[r] * 2, ncclChar, j, g_nccl, cs));
            if (st.len[j]) ESGD_NCCL(ncclRecv(w + st.off[j], st.len[j] * 2, ncclChar, j, g_nccl, cs));
        }
        ESGD_NCCL(ncclGroupEnd());
        const uint64_t pc = piece_bytes() / 4;
        const void *src[kMaxSegs];
        void *dst[kMaxSegs];
        uint64_t cnt[kMaxSegs];
        int m = 0;
        for (int j = 0; j < P; ++j) {
            if (j == r) continue;
            for (uint64_t o = 0; o < st.len[j]; o += pc) {
                src[m] = w + st.off[j] + o;
                dst[m] = rbf + st.off[j] + o;
                cnt[m] = std::min(pc, st.len[j] - o);
                if (++m == kMaxSegs) {
                    if (int rc = gather_widen(m, src, dst, cnt, cs)) return rc;
                    m = 0;
                }
            }
        }
        return m ? gather_widen(m, src, dst, cnt, cs) : ESGD_SUCCESS;
    }

    int query(Sched &s) override { return base_query(s, S(s)); }
    int complete(Sched &s) override { return base_complete(s, S(s)); }

    void teardown(Sched &s) override {
        RcclState *st = static_cast<RcclState *>(s.tstate);
        if (!st) return;
        if (st->stream) hip_ignore(hipStreamSynchronize(st->stream));
        if (st->red) { hip_ignore(hipStreamSynchronize(st->red)); hip_ignore(hipStreamDestroy(st->red)); }
        if (st->stage) arena_free(st->stage);
        if (st->wire) arena_free(st->wire);
        for (hipEvent_t e : st->ev_chunk) hip_ignore(hipEventDestroy(e));
        if (st->ev_red) hip_ignore(hipEventDestroy(st->ev_red));
        base_teardown(s, *st);
        delete st;
        s.tstate = nullptr;
    }
};

Transport *rccl_transport() {
    static RcclTransport t;
    return &t;
}

}  // namespace esgd
