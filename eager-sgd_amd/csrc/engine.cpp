// engine.cpp — partial-allreduce schedules, the round protocol and the progress thread.
//
// Per schedule and round t, every rank walks the same stages (engine.h: Stage):
//   join (activation rules, prepare: host staging / buffer re-resolution)
//     -> the last rank to join appends (schedule, t) to the node's issue ring
//     -> every rank launches the ring's rounds in ring order: the whole round is queued
//        on the GPU, whose own flag waits pair the ranks (dataplane.cpp)
//     -> the round's completion event -> copy-out hook -> completed = t, wake wait().
// "Join" is decided by the activation rules of fflib2 (see engine.h).  The pairing of
// ranks is what fflib2's matched MPI send/recv pairs guarantee implicitly
// (src/colls/ffallreduce.c:145-162: a send of rb after the previous comp, the comp after
// the recv); here it costs no host round trip inside a round.
#include "engine.h"

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_set>
#include <ctime>

#include "esgd_internal.h"

namespace esgd {

static Segment *g_seg = nullptr;
static int g_rank = 0, g_world = 1, g_device = -1;
static std::string g_job;
static double g_timeout = 600.0;
static std::mutex g_reg_mu;
static std::vector<Sched *> g_reg;
static std::unordered_set<const Sched *> g_reg_set;   // = g_reg, for O(1) handle checks
// = g_reg by schedule id, for the issue-ring pump (written under g_reg_mu; a schedule is
// freed only two progress epochs after its entry is cleared, like its g_reg entry)
static std::atomic<Sched *> g_by_id[kMaxSched];
static std::atomic<int> g_id_end{0};   // ids below this were handed out (the pass's scan range)
// What the progress pass needs to skip a quiet schedule, packed by id: its posted and joined
// counters and whether it is busy (stage != idle, or posted and awaiting its activation) --
// written wherever the Sched's own fields change.  A pass reads these and the segment's
// packed activation counters, and touches a Sched object only when there is work: with
// ~1700 schedules alive (the bench's legs) the per-schedule Sched reads were most of a pass.
struct alignas(16) HotState {
    std::atomic<uint32_t> posted{0}, joined{0}, busy{0};
};
static HotState g_hot[kMaxSched];

static void hot_busy(const Sched &s) {
    g_hot[s.id].busy.store((s.stage.load(std::memory_order_relaxed) != ST_IDLE || s.awaiting.load(std::memory_order_relaxed))
                               ? 1u : 0u, std::memory_order_release);
}
static std::mutex g_create_mu;
static int g_next_id = 0;
static std::thread g_thread;
static std::atomic<bool> g_running{false};
static std::atomic<uint64_t> g_epoch{0};             // progress passes completed
// next ticket this rank issues (written by the thread pumping the ring; atomic so that a
// timed-out wait on another thread can report it)
static std::atomic<uint64_t> g_cursor{0};
static std::mutex g_issue_mu;
static std::vector<std::pair<uint32_t, uint32_t>> g_issued;

bool engine_ready() { return g_seg != nullptr; }
int engine_rank() { return g_rank; }
int engine_world() { return g_world; }
Segment *engine_segment() { return g_seg; }
double engine_timeout() { return g_timeout; }

int engine_barrier() {
    if (!g_seg) { set_error("esgd: communicator not initialised"); return ESGD_ERROR; }
    return shm_barrier(g_seg, g_world, g_timeout);
}

bool round_is_sync(const Sched &s, uint32_t round) {
    switch (s.kind) {
    case KIND_SOLO:  // limiter: posts 1..async asynchronous, post async+1 synchronous
        return s.async <= 0 || round % uint32_t(s.async + 1) == 0;
    case KIND_MAJORITY: return false;
    default: return true;
    }
}

// ESGD_ROCTX=1: roctx ranges for rocprofv3 --marker-trace (SURVEY.md §5 "tracing"): one
// range per round from join to completion ("esgd s<id> r<round>"), one per launch and one
// per blocking wait; the kernels of a round appear in the kernel trace by name
// (k_round_small, k_round_sync, k_tree_sum_buf, k_gather).
static bool roctx_on() {
    static const bool on = getenv("ESGD_ROCTX") && *getenv("ESGD_ROCTX") == '1';
    return on;
}

static std::atomic<int> g_active{0};   // schedules with a round in flight or a post pending
// esgd_comm_profile: written by the thread running progress passes, read by any
static std::atomic<uint64_t> g_prof_passes{0}, g_prof_pass_ns{0}, g_prof_pump_ns{0}, g_prof_joins{0},
    g_prof_join_ns{0};

// A process that exits without fffinalize / esgd_comm_finalize must not die in
// std::thread's destructor: stop and join the progress thread at static destruction.
static struct ProgressGuard {
    ~ProgressGuard() {
        if (g_running.exchange(false) && g_thread.joinable()) g_thread.join();
    }
} g_progress_guard;

// Idle, the thread sleeps on the segment's wake word: a peer's activation, an issue-ring
// append or a local post wakes it at once (the reference's progress thread busy-polls
// MPI_Testsome instead, ffprogress.c:39-57).  A round in flight is latency-critical: the
// thread spins / yields then, never sleeps.
static void progress_main() {
    if (g_device >= 0) hip_ignore(hipSetDevice(g_device));
    unsigned polls = 0;
    while (g_running.load(std::memory_order_acquire)) {
        const uint32_t ws = g_seg->wake_seq.load(std::memory_order_acquire);
        if (engine_progress_once()) { polls = 0; continue; }
        if (g_seg->wake_seq.load(std::memory_order_acquire) != ws) { polls = 0; continue; }
        ++polls;
        if (g_active.load(std::memory_order_relaxed) > 0) {
            if (polls > 64) sched_yield();
            continue;
        }
        if (polls < 64) continue;
        if (polls < 256) { sched_yield(); continue; }
        seg_idle_wait(g_seg, ws, 1000);   // 1 ms backstop
    }
}

int engine_init(const char *job, int rank, int world, bool start_progress) {
    if (g_seg) {
        if (rank == g_rank && world == g_world) return ESGD_SUCCESS;
        set_error("esgd: already initialised as rank %d/%d", g_rank, g_world);
        return ESGD_INVALID_ARG;
    }
    if (world > 1 && dataplane_mappings_closed()) {
        set_error("esgd: this process already finalized a job whose peers' buckets it mapped over IPC; "
                  "re-opening closed IPC handles is unsafe on this driver (DESIGN.md §5): run each "
                  "multi-process job in a fresh process");
        return ESGD_ERROR;
    }
    if (const char *t = getenv("ESGD_TIMEOUT_S")) g_timeout = atof(t) > 0 ? atof(t) : g_timeout;
    Segment *seg = shm_attach(job, rank, world, g_timeout);
    if (!seg) return ESGD_ERROR;
    g_seg = seg; g_rank = rank; g_world = world; g_job = job;
    int dev = -1;
    if (start_progress && hipGetDevice(&dev) == hipSuccess) g_device = dev;
    seg->device[rank].store(g_device);
    uint64_t gid = 0;
    if (g_device >= 0) {
        int dom = 0, bus = 0, slot = 0;
        if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, g_device) == hipSuccess &&
            hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, g_device) == hipSuccess &&
            hipDeviceGetAttribute(&slot, hipDeviceAttributePciDeviceId, g_device) == hipSuccess)
            gid = ((uint64_t(uint32_t(dom)) << 32) | (uint64_t(uint32_t(bus) & 0xffff) << 16) |
                   uint64_t(uint32_t(slot) & 0xffff)) + 1;
        else
            (void)hipGetLastError();
    }
    seg->gpu_id[rank].store(gid);
    if (int rc = shm_barrier(seg, world, g_timeout)) { g_seg = nullptr; shm_detach(seg, job, rank); return rc; }
    // every rank is attached: drop the name so nothing outlives the job in /dev/shm
    if (rank == 0) shm_unlink_name(job);
    if (start_progress) {
        g_running.store(true);
        g_thread = std::thread(progress_main);
    }
    if (world > 1 && g_device >= 0) arena_warm();   // before any bucket of the job is exported
    return ESGD_SUCCESS;
}

static void free_sched(Sched *s) {
    if (s->resolve_free && s->resolve_ctx) s->resolve_free(s->resolve_ctx);
    delete s;
}

int engine_finalize() {
    if (!g_seg) return ESGD_SUCCESS;
    int rc = shm_barrier(g_seg, g_world, g_timeout);
    if (g_running.exchange(false)) g_thread.join();
    // rounds held for the next shared launch (ESGD_BATCH_DEPTH) go out now, while their
    // schedules are alive: every rank launched them in ring order, so they pair up, and the
    // teardowns below wait for them on the round stream
    (void)dataplane_flush();
    std::vector<Sched *> left;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        left.swap(g_reg);
        g_reg_set.clear();
        for (auto &e : g_by_id) e.store(nullptr, std::memory_order_relaxed);
        for (auto &h : g_hot) { h.posted.store(0); h.joined.store(0); h.busy.store(0); }
        g_id_end.store(0);
    }
    for (Sched *s : left) {
        if (s->tp) s->tp->teardown(*s);
        free_sched(s);
    }
    dataplane_shutdown();
    shm_detach(g_seg, nullptr, -1);
    g_seg = nullptr;
    g_next_id = 0;
    g_cursor.store(0);
    {
        std::lock_guard<std::mutex> lk(g_issue_mu);
        g_issued.clear();
    }
    return rc;
}

// ---- schedules -------------------------------------------------------------------

void gpu_trace_read(Sched &s, uint64_t out[6]);   // dataplane.cpp

static uint64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

void Sched::mark(uint32_t round, int what) {   // caller holds mu
    if (round == 0 || round > 65536) return;
    if (tl.size() < round) tl.resize(std::max<size_t>(round, std::min<size_t>(65536, 2 * tl.size())));
    tl[round - 1][what] = mono_ns();
}

// What a schedule is doing, for the message of a timed-out wait or join (caller holds
// s.mu): this rank's round counters and stage, the node's activation and join counts, how
// far this rank has launched the node's issue ring, then the transport's flag words and
// the data plane's pending launches -- so a stall names the stage and the rank it is in.
static const char *stage_name(Stage st) {
    return st == ST_IDLE ? "idle" : st == ST_WAIT_TICKET ? "joined, waiting for its issue-ring turn" : "launched";
}

static std::string sched_state(Sched &s) {
    char buf[512];
    snprintf(buf, sizeof(buf),
             "[rank %d: posted %u joined %u completed %u waited %u released %u; round %u %s (%s) for %.1f s%s; "
             "node: activated %u, joins %u; issue ring: %llu launched here of %llu]",
             s.rank, s.posted.load(), s.joined.load(), s.completed, s.waited, s.released, s.cur,
             stage_name(s.stage.load()), s.cur_fresh ? "posted" : "carried by a peer", now_s() - s.stage_t0,
             s.hold_mode && s.released < s.joined ? ", held until release()" : "", s.activated->load(),
             s.sh->ready_count.load(), (unsigned long long)g_cursor.load(std::memory_order_relaxed),
             (unsigned long long)(g_seg ? g_seg->ticket_next.load() : 0));
    std::string m = buf;
    if (s.tp) m += " " + s.tp->diagnose(s);
    return m + " [" + dataplane_state() + "]";
}

static void fail_locked(Sched &s, int rc, const char *msg) {
    if (s.roctx_round) { roctxRangeStop(s.roctx_round); s.roctx_round = 0; }
    // the failure contract across ranks: a round this rank joined and has not
    // completed fails on every rank now -- peers' GPU flag waits and host queries watch this
    // word -- rather than at their own timeouts.  A failure on the host side (a launch, a
    // join, the wait limit) runs no kernel that would have recorded it; where the GPU did,
    // it stored this same round.
    if (s.world > 1 && s.sh && int32_t(s.cur - s.completed) > 0)
        s.sh->gpu_err[s.rank].store(s.cur, std::memory_order_release);
    s.error = rc ? rc : ESGD_ERROR;
    snprintf(s.errmsg, sizeof(s.errmsg), "schedule %d round %u: %s", s.id, s.cur, msg);
    s.cv.notify_all();
}

int sched_create(int kind, int dtype, uint64_t count, void *sb, void *rb, bool host_mode,
                 int async, unsigned seed, Transport *tp, Sched **out, unsigned flags, int tag) {
    return sched_create_with(kind, dtype, count, sb, rb, host_mode, async, seed, tp, nullptr,
                             nullptr, nullptr, out, flags, tag);
}

int sched_create_with(int kind, int dtype, uint64_t count, void *sb, void *rb, bool host_mode,
                      int async, unsigned seed, Transport *tp, int (*resolve)(Sched &),
                      void *ctx, void (*ctx_free)(void *), Sched **out, unsigned flags, int tag) {
    ESGD_ARG(out, "schedule create: null output");
    ESGD_ARG(kind >= KIND_ALLREDUCE && kind <= KIND_MAJORITY, "schedule create: bad kind %d", kind);
    ESGD_ARG(tp, "schedule create: no transport");
    if (!g_seg) { set_error("esgd: communicator not initialised (ffinit / esgd_comm_init)"); return ESGD_ERROR; }
    std::lock_guard<std::mutex> clk(g_create_mu);
    if (g_next_id >= kMaxSched) { set_error("schedule create: more than %d schedules", kMaxSched); return ESGD_ENOMEM; }
    Sched *s = new Sched();
    s->id = g_next_id++;
    s->kind = kind; s->dtype = dtype; s->count = count; s->esize = esgd_dtype_size(dtype);
    s->sb = sb; s->rb = rb; s->host_mode = host_mode; s->in_place = (sb == nullptr || sb == rb);
    s->async = async; s->seed = seed;
    s->rank = g_rank; s->world = g_world;
    s->sh = &g_seg->sched[s->id];
    s->activated = &g_seg->activated[s->id];
    s->tp = tp;
    s->resolve = resolve;
    s->resolve_ctx = ctx;
    s->resolve_free = ctx_free;
    s->hold_mode = (flags & ESGD_SCHED_HOLD) != 0;
    s->zero_sb = (flags & ESGD_SCHED_ZERO_SB) != 0 && !host_mode && !s->in_place;
    s->wire_bf16 = (flags & ESGD_SCHED_WIRE_BF16) != 0;
    s->fresh_only = (flags & ESGD_SCHED_FRESH_ONLY) != 0;
    s->small_bytes = config_small_round_bytes();
    s->flag_mode = config_device_flags();
    s->strict = config_strict_handoffs();
    // Schedule ids are never reused within a job and the segment starts zeroed, so the
    // shared state of this id needs no reset (no barrier before setup).  Creation costs TWO
    // node barriers: setup (local: buckets, streams, publication) -> vote 1 (setup failures)
    // -> every rank checks every rank's signature (kind, dtype, tag, data-plane settings: the
    // same data on every rank, so all fail alike) -> connect (mapping peers' publications,
    // which vote 1 guarantees) -> vote 2 (connect failures).  Vote 2 is not optional: without
    // it a rank that returned early posts round 1 while a peer is still mapping its
    // publication, and a resolve-mode schedule re-publishes its bucket at that post -- the
    // peer then maps a torn (handle, offset, ver) and pulls a stale bucket (round 3's r03f
    // session: FFCOLL_BUFFERS sums with zeroed shards at 4 ranks).
    s->gen = 1;   // IpcSlot::gen == 1: published for this id
    const bool small = count * s->esize <= s->small_bytes;
    const uint64_t sig = (uint64_t(s->strict) << 53) | (uint64_t(small) << 52) | (uint64_t(s->flag_mode & 3) << 50) |
                         (uint64_t(s->wire_bf16) << 48) | (uint64_t(uint32_t(kind)) << 40) |
                         (uint64_t(uint32_t(dtype) & 0xff) << 32) |
                         (tag == kNoTag ? 0 : (0x10000u | uint16_t(tag)));
    int rc = ESGD_SUCCESS;
    // each vote has its own failure counter: a rank already failing the second vote must
    // not make a slower rank, still reading the first vote's result, report the wrong cause
    auto vote = [&](int r, std::atomic<uint32_t> &errs) -> int {
        if (r) errs.fetch_add(1, std::memory_order_acq_rel);
        const int rb = shm_barrier(g_seg, g_world, g_timeout);
        if (r) return r;
        if (rb) return rb;
        if (errs.load(std::memory_order_acquire)) {
            set_error("schedule create: another rank failed to register schedule %d", s->id);
            return ESGD_ERROR;
        }
        return ESGD_SUCCESS;
    };
    static const bool dbg = getenv("ESGD_DEBUG") && *getenv("ESGD_DEBUG") == '1';
    const double c0 = now_s();
    s->sh->sig[g_rank].store(sig, std::memory_order_release);
    if (!rc) rc = tp->setup(*s);     // local: buffers, streams, publication
    const double c1 = now_s();
    rc = vote(rc, s->sh->setup_err);
    for (int q = 0; !rc && q < g_world; ++q) {
        const uint64_t o = s->sh->sig[q].load(std::memory_order_acquire);
        if (o != sig) {
            set_error("schedule create: rank %d created (kind %d, dtype %d, tag %d, flags mode %d, one-launch %d), "
                      "rank %d (kind %d, dtype %d, tag %d, flags mode %d, one-launch %d): creation order must "
                      "match, and so must the data-plane settings", g_rank, kind, dtype, tag == kNoTag ? -1 : tag,
                      s->flag_mode, int(small), q, int((o >> 40) & 0xff), int((o >> 32) & 0xff),
                      (o & 0x10000) ? int(int16_t(o & 0xffff)) : -1, int((o >> 50) & 3), int((o >> 52) & 1));
            rc = ESGD_INVALID_ARG;   // every rank sees the same signatures: all fail
        }
    }
    const double c2 = now_s();
    if (!rc) {
        rc = tp->connect(*s);   // needs every peer's publication
        rc = vote(rc, s->sh->connect_err);
    }
    // A fresh mapping of a peer's chunk that showed other memory (its seal: round 5 caught
    // the runtime handing an importer its OWN exported chunk for a peer's handle, DESIGN.md
    // §5) asked that peer to move the publication (SchedShm::remap): every rank sees the same
    // requests after the vote, the asked ranks re-publish from chunks allocated anew, a vote,
    // and every rank maps again -- up to kRemapTries times before the creation fails.
    for (int a = 0; rc && a < kRemapTries; ++a) {
        uint32_t any = 0;
        for (int q = 0; q < g_world; ++q) any |= s->sh->remap[a][q].load(std::memory_order_acquire);
        if (!any) break;
        const uint32_t mine = s->sh->remap[a][g_rank].load(std::memory_order_acquire);
        if (mine)
            fprintf(stderr, "esgd: rank %d schedule %d: a peer's mapping of this rank's %s showed other memory; "
                    "re-publishing from a new chunk (attempt %d)\n", g_rank, s->id,
                    mine == 3 ? "bucket and shard" : mine == 1 ? "bucket" : "shard", a + 1);
        clear_error();
        int r2 = mine ? tp->remap(*s, mine) : ESGD_SUCCESS;
        r2 = vote(r2, s->sh->retry_err[2 * a]);
        if (!r2) {
            s->connect_attempt = a + 1;
            r2 = tp->connect(*s);
            r2 = vote(r2, s->sh->retry_err[2 * a + 1]);
        }
        ++s->remaps;
        rc = r2;
    }
    if (dbg)
        fprintf(stderr, "[esgd] r%d create sched %d (%llu x %d B): setup %.1f ms, vote %.1f ms, connect %.1f ms\n",
                g_rank, s->id, (unsigned long long)count, int(s->esize), (c1 - c0) * 1e3, (c2 - c1) * 1e3,
                (now_s() - c2) * 1e3);
    if (rc) {
        if (s->tstate) tp->teardown(*s);
        s->resolve_free = nullptr;   // the caller still owns ctx on failure
        delete s;
        return rc;
    }
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.push_back(s);
        g_reg_set.insert(s);
        g_hot[s->id].posted.store(0);
        g_hot[s->id].joined.store(0);
        g_hot[s->id].busy.store(0);
        g_by_id[s->id].store(s, std::memory_order_release);
        if (g_id_end.load() < s->id + 1) g_id_end.store(s->id + 1, std::memory_order_release);
    }
    *out = s;
    return ESGD_SUCCESS;
}

// Activate `round` (the activation flood of colls/ffactivation.c): claim the round's
// slot first (first claimant = activator), then raise the shared counter.
static void activate(Sched &s, uint32_t round, int rank, bool *won) {
    SchedShm *sh = s.sh;
    std::atomic<uint64_t> &slot = sh->act_of[round % 256];
    uint64_t cur = slot.load(std::memory_order_acquire);
    const uint64_t mine = (uint64_t(round) << 32) | uint64_t(rank + 1);
    *won = false;
    while ((cur >> 32) < round) {
        if (slot.compare_exchange_weak(cur, mine, std::memory_order_acq_rel)) {
            *won = true;
            sh->last_activator.store(rank, std::memory_order_relaxed);
            sh->activations[rank].fetch_add(1, std::memory_order_relaxed);
            break;
        }
    }
    uint32_t a = s.activated->load(std::memory_order_acquire);
    while (a < round && !s.activated->compare_exchange_weak(a, round, std::memory_order_acq_rel)) {
    }
    seg_wake(g_seg);   // the flood: every idle progress thread joins now
}

static int activator_of(SchedShm *sh, uint32_t round) {
    const uint64_t v = sh->act_of[round % 256].load(std::memory_order_acquire);
    return (v >> 32) == round ? int(v & 0xffffffffu) - 1 : -1;
}

static bool step(Sched &s, bool join_only);

int sched_post(Sched *s, void *producer_stream, int *role, const RoundIO *io) {
    ESGD_ARG(s, "schedule post: null schedule");
    int r = 0;
    {
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->error) { set_error("%s", s->errmsg); return s->error; }
        const uint32_t t = s->posted.load() + 1;
        // FFCOLL_BUFFERS: the buffers of round t are resolved at its post -- unless a peer's
        // activation already carried this rank into round t (re-resolved at that join,
        // possibly still in flight: nothing to do).  A round not yet joined must not start
        // while an earlier one is in flight with the old buffers.
        if (s->resolve && s->joined < t) {
            if (s->stage != ST_IDLE) {
                set_error("schedule %d: FFCOLL_BUFFERS rounds must not overlap", s->id);
                return ESGD_INVALID_ARG;
            }
            if (int rc = s->resolve(*s)) return rc;
        }
        // the producer first, the round's own data last (both before the post counts: a join
        // that sees it fresh finds them): a failed note_producer leaves no RoundIO behind
        // for a later post of round t to launch with stale pointers
        if (producer_stream)
            if (int rc = s->tp->note_producer(*s, t, producer_stream)) return rc;
        if (io)
            if (int rc = s->tp->note_io(*s, t, *io)) return rc;
        s->posted.store(t, std::memory_order_release);
        g_hot[s->id].posted.store(t, std::memory_order_release);
        s->mark(t, 0);
        if (s->kind == KIND_MAJORITY) {
            // colls/ffrand_allreduce.c:88 — the same glibc draw on every rank
            const int act = int(unsigned(rand_r(&s->seed)) % unsigned(s->world));
            if (act == s->rank) {
                bool won;
                activate(*s, t, s->rank, &won);
                s->passive = 0;   // catch-up of :93-96 is implicit in the round counter
                r = 1;
                if (won) ++s->n_activated;
            } else {
                ++s->passive;
                r = 0;
            }
        } else if (round_is_sync(*s, t)) {
            r = 2;
        } else {
            bool won;
            activate(*s, t, s->rank, &won);   // the first poster activates the round
            r = won ? 1 : 0;
            if (won) ++s->n_activated;
        }
    }
    // the round this post makes due is joined right here, on the caller's thread, instead
    // of at the progress thread's next pass: the join is
    // per-schedule work under its mutex plus the issue-ring append (atomics), and joining at
    // the post takes it off the progress thread, which then only launches.  Device buckets
    // without FFCOLL_BUFFERS only (a host bucket's join stages the bucket; a resolve
    // schedule's re-resolves it).
    if (!s->resolve && !s->host_mode) (void)step(*s, true);
    seg_wake(g_seg);
    if (role) *role = r;
    return ESGD_SUCCESS;
}

int sched_wait(Sched *s) { return sched_wait_ex(s, nullptr); }

int sched_wait_ex(Sched *s, int *fresh) {
    ESGD_ARG(s, "schedule wait: null schedule");
    uint32_t target;
    {
        std::lock_guard<std::mutex> lk(s->mu);
        ESGD_ARG(!s->held, "schedule %d: release() the round wait() returned before waiting for the next", s->id);
        target = s->waited + 1;
    }
    // a round about to complete is seen ~5 us sooner by spinning than through the
    // condition variable's futex wake: spin briefly, then block
    constexpr double spin_s = 200e-6;
    const double t0 = now_s();
    if (roctx_on()) roctxRangePushA("esgd wait");
    while (int32_t(s->completed_a.load(std::memory_order_acquire) - target) < 0 && now_s() - t0 < spin_s)
        std::this_thread::yield();
    std::unique_lock<std::mutex> lk(s->mu);
    while (s->completed < target && !s->error) {
        s->cv.wait_for(lk, std::chrono::milliseconds(50));
        if (now_s() - t0 > g_timeout) {
            const std::string m = "wait timed out " + sched_state(*s);
            fail_locked(*s, ESGD_ERROR, m.c_str());
            break;
        }
    }
    if (roctx_on()) roctxRangePop();
    if (s->error) { set_error("%s", s->errmsg); return s->error; }
    s->waited = target;
    s->mark(target, 5);
    if (s->hold_mode) s->held = true;
    // the fresh bit of the round returned
    const int f = s->fresh_take(target) ? 1 : 0;
    if (fresh) *fresh = f;
    return ESGD_SUCCESS;
}

int sched_release(Sched *s, void *stream) {
    ESGD_ARG(s, "schedule release: null schedule");
    {
        std::lock_guard<std::mutex> lk(s->mu);
        if (s->error) { set_error("%s", s->errmsg); return s->error; }
        ESGD_ARG(s->hold_mode, "schedule %d: release() needs a schedule created with ESGD_SCHED_HOLD", s->id);
        ESGD_ARG(s->held, "schedule %d: nothing to release (no round returned since the last release)", s->id);
        if (stream)
            if (int rc = s->tp->note_consumer(*s, stream)) return rc;
        s->held = false;
        s->released = s->waited;
    }
    seg_wake(g_seg);
    return ESGD_SUCCESS;
}

int sched_test(Sched *s, int *flag) {
    ESGD_ARG(s && flag, "schedule test: null argument");
    std::lock_guard<std::mutex> lk(s->mu);
    if (s->error) { set_error("%s", s->errmsg); return s->error; }
    ESGD_ARG(!s->held, "schedule %d: release() the round test() returned before testing for the next", s->id);
    *flag = s->completed >= s->waited + 1;
    if (*flag) {
        ++s->waited;
        (void)s->fresh_take(s->waited);
        if (s->hold_mode) s->held = true;
    }
    return ESGD_SUCCESS;
}

int sched_delete(Sched *s) {
    ESGD_ARG(s, "schedule delete: null schedule");
    const double t0 = now_s();
    // an in-flight round of this schedule may sit in the pending shared launch (held behind
    // ESGD_BATCH_DEPTH launches, or by batch_hold): send it, so that it can finish
    (void)dataplane_flush();
    for (;;) {   // let an in-flight round finish (peers may still need our flags)
        {
            std::lock_guard<std::mutex> lk(s->mu);
            if (s->stage == ST_IDLE || s->error) { s->live.store(false); break; }
        }
        if (now_s() - t0 > g_timeout) break;
        std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        g_reg.erase(std::remove(g_reg.begin(), g_reg.end(), s), g_reg.end());
        g_reg_set.erase(s);
        if (s->id >= 0 && s->id < kMaxSched) g_by_id[s->id].store(nullptr, std::memory_order_release);
    }
    // The progress thread may be inside a pass over a registry copy that still holds s:
    // wait until a pass that began after the erase has finished (two epochs).
    if (g_running.load(std::memory_order_acquire) && std::this_thread::get_id() != g_thread.get_id()) {
        const uint64_t e0 = g_epoch.load(std::memory_order_acquire);
        while (g_epoch.load(std::memory_order_acquire) < e0 + 2 && g_running.load(std::memory_order_acquire)) {
            seg_wake(g_seg);
            std::this_thread::yield();
        }
    }
    // A round of this schedule may still wait in the pending shared launch (the loop above
    // gave up on an error or the timeout): it goes out now, while the schedule is alive --
    // peers launched it too -- and the teardown's stream synchronisation waits for it.
    (void)dataplane_flush();
    // Local, like ffschedule_delete: every peer finished reading this rank's buckets for
    // the rounds it joined (the done pairing), and the buckets go back to the IPC arena,
    // which never unmaps them under a peer (arena.cpp).
    s->tp->teardown(*s);
    free_sched(s);
    return ESGD_SUCCESS;
}

Sched *sched_lookup(uint64_t handle) {
    Sched *p = reinterpret_cast<Sched *>(handle);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    return g_reg_set.count(p) ? p : nullptr;
}

// ---- the progress step -------------------------------------------------------------

// join_only: only the IDLE -> joined transition (a caller's thread joining the round it
// has just posted, sched_post); every other stage is left to the progress thread
static bool step(Sched &s, bool join_only = false) {
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.error || !s.live.load()) { s.awaiting = false; hot_busy(s); return false; }
    if (join_only && s.stage != ST_IDLE) return false;
    SchedShm *sh = s.sh;
    auto enter = [&](Stage st) { s.stage = st; s.stage_t0 = now_s(); hot_busy(s); };
    auto check = [&](int rc, const char *what) {
        if (rc < 0) {
            std::string m = std::string(what) + ": " + esgd_last_error();
            fail_locked(s, rc, m.c_str());
            return false;
        }
        return true;
    };
    switch (s.stage) {
    case ST_IDLE: {
        s.awaiting = false;
        hot_busy(s);
        // hold mode: the caller has not yet taken (wait) and released the last round
        if (s.hold_mode && s.released < s.joined) return false;
        const uint32_t next = s.joined + 1;
        const bool sync = round_is_sync(s, next);
        const uint32_t posted = s.posted.load(std::memory_order_acquire);
        const bool go = sync ? posted >= next : s.activated->load(std::memory_order_acquire) >= next;
        if (!go) {
            s.awaiting = posted >= next;
            hot_busy(s);
            return false;
        }
        const uint64_t j0 = mono_ns();
        struct JoinProf {   // rounds joined and the ns they took (esgd_comm_profile)
            uint64_t t0;
            ~JoinProf() {
                g_prof_joins.fetch_add(1, std::memory_order_relaxed);
                g_prof_join_ns.fetch_add(mono_ns() - t0, std::memory_order_relaxed);
            }
        } join_prof{j0};
        s.cur = next;
        s.cur_fresh = posted >= next;
        s.joined = next;
        g_hot[s.id].joined.store(next, std::memory_order_release);
        s.fresh_set(next, s.cur_fresh);
        // FFCOLL_BUFFERS: a round joined on a peer's activation re-resolves the buffers
        // here (a fresh round did at its post)
        if (s.resolve && !s.cur_fresh && !check(s.resolve(s), "join")) return true;
        s.mark(next, 1);
        sh->joined[s.rank].store(next, std::memory_order_release);
        if (s.cur_fresh) ++s.n_fresh; else ++s.n_auto;
        if (s.log.size() < 65536)
            s.log.push_back({next, uint8_t(s.cur_fresh), uint8_t(sync),
                             int16_t(sync ? -1 : activator_of(sh, next))});
        if (!check(s.tp->prepare(s, next, s.cur_fresh), "join")) return true;
        if (roctx_on()) {
            char name[64];
            snprintf(name, sizeof(name), "esgd s%d r%u%s", s.id, next, s.cur_fresh ? "" : " (auto)");
            s.roctx_round = roctxRangeStartA(name);
        }
        enter(ST_WAIT_TICKET);
        // the rank whose join completes the round appends it to the issue ring (every
        // rank has joined round t-1 of this schedule before any joins round t)
        const uint32_t prev = sh->ready_count.fetch_add(1, std::memory_order_acq_rel);
        if (prev + 1 == next * uint32_t(s.world)) {
            const uint64_t tk = g_seg->ticket_next.fetch_add(1, std::memory_order_acq_rel);
            TicketSlot &slot = g_seg->ring[tk % kRing];
            slot.sched = uint32_t(s.id);
            slot.round = next;
            slot.tag.store(tk + 1, std::memory_order_release);
            seg_wake(g_seg);
        }
        return true;
    }
    case ST_WAIT_TICKET:
        if (now_s() - s.stage_t0 > g_timeout) {
            const std::string m = "not every rank joined the round (a peer never posted / activated?) " + sched_state(s);
            fail_locked(s, ESGD_ERROR, m.c_str());
        }
        return false;
    case ST_INFLIGHT: {
        const int q = s.tp->query(s);
        if (!check(q, "round")) return true;
        if (!q) {
            // the GPU's flag waits give up after the timeout and complete the round with
            // an error flag; this is the host's backstop
            if (now_s() - s.stage_t0 > 1.5 * g_timeout + 5) {
                std::string m = "round did not finish on the GPU " + sched_state(s);
                fail_locked(s, ESGD_ERROR, m.c_str());
                return true;
            }
            return false;
        }
        s.mark(s.cur, 4);
        if (s.cur <= s.tl.size()) {
            uint64_t g[6];
            gpu_trace_read(s, g);
            for (int k = 0; k < 6; ++k) s.tl[s.cur - 1][6 + k] = g[k];
        }
        if (!check(s.tp->complete(s), "round")) return true;
        if (s.roctx_round) { roctxRangeStop(s.roctx_round); s.roctx_round = 0; }
        s.completed = s.cur;
        s.completed_a.store(s.cur, std::memory_order_release);
        s.stage = ST_IDLE;
        hot_busy(s);
        s.cv.notify_all();
        return true;
    }
    }
    return false;
}

// An idle schedule whose next round is neither posted here nor activated by a peer has
// nothing to do: the pass skips it without taking its mutex (step() would return false).
// With hundreds of schedules (one per gradient tensor) most are quiet in any pass.
static bool quiet(int id) {
    const HotState &h = g_hot[id];
    if (h.busy.load(std::memory_order_acquire)) return false;
    const uint32_t next = h.joined.load(std::memory_order_acquire) + 1;
    return h.posted.load(std::memory_order_acquire) < next && g_seg->activated[id].load(std::memory_order_acquire) < next;
}

// Launch rounds strictly in ring order (the same sequence on every rank).
static bool pump_tickets() {
    if (!g_seg) return false;
    bool any = false;
    for (;;) {
        const uint64_t cur = g_cursor.load(std::memory_order_relaxed);
        TicketSlot &slot = g_seg->ring[cur % kRing];
        if (slot.tag.load(std::memory_order_acquire) != cur + 1) break;
        // by id: a scan of the registry cost O(schedules) per round -- in a process holding
        // ~1700 schedules (the bench's legs) most of the pass
        Sched *target = slot.sched < uint32_t(kMaxSched) ? g_by_id[slot.sched].load(std::memory_order_acquire) : nullptr;
        if (!target) break;                      // schedule not registered here yet
        {
            std::lock_guard<std::mutex> lk(target->mu);
            if (target->error) {
                // a failed schedule still consumes its tickets (its peers fail the same
                // round: by their own timeout, or at once through this rank's error word --
                // DESIGN.md §5, "Failure contract"); later rounds of other schedules must
                // not stall
            } else if (target->stage != ST_WAIT_TICKET || target->cur != slot.round) {
                break;
            } else {
                target->mark(target->cur, 2);
                if (roctx_on()) roctxRangePushA("esgd launch");
                int rc = target->tp->launch(*target, target->cur, target->cur_fresh);
                if (roctx_on()) roctxRangePop();
                target->mark(target->cur, 3);
                if (rc < 0) {
                    std::string m = std::string("launch: ") + esgd_last_error();
                    fail_locked(*target, rc, m.c_str());
                } else {
                    target->stage = ST_INFLIGHT;
                    target->stage_t0 = now_s();
                    hot_busy(*target);
                }
            }
        }
        {
            std::lock_guard<std::mutex> lk(g_issue_mu);
            if (g_issued.size() < 65536) g_issued.emplace_back(slot.sched, slot.round);
        }
        g_cursor.store(cur + 1, std::memory_order_relaxed);
        any = true;
    }
    // the one-launch rounds this pump appended go out in one launch (now, or once a
    // queued shared launch has finished); a failure is recorded in every round of that
    // launch (the transport reports it at its query)
    // (every pass: a launch held back behind ESGD_BATCH_DEPTH queued ones goes out as soon
    // as one of them has finished)
    (void)dataplane_flush_soft();
    return any;
}

int engine_issue_log(uint32_t *sched, uint32_t *round, uint32_t cap, uint32_t *n) {
    std::lock_guard<std::mutex> lk(g_issue_mu);
    for (uint32_t i = 0; i < g_issued.size() && i < cap; ++i) {
        if (sched) sched[i] = g_issued[i].first;
        if (round) round[i] = g_issued[i].second;
    }
    if (n) *n = uint32_t(g_issued.size());
    return ESGD_SUCCESS;
}

void engine_profile(uint64_t out[7]) {
    out[0] = g_prof_passes.load(std::memory_order_relaxed);
    out[1] = g_prof_pass_ns.load(std::memory_order_relaxed);
    out[2] = g_prof_pump_ns.load(std::memory_order_relaxed);
    out[3] = g_prof_joins.load(std::memory_order_relaxed);
    out[4] = g_prof_join_ns.load(std::memory_order_relaxed);
    dataplane_profile(&out[5], &out[6]);
}

bool engine_progress_once() {
    const uint64_t p0 = mono_ns();
    if (!g_seg) return false;
    bool any = pump_tickets();
    const uint64_t p1 = mono_ns();
    if (any) g_prof_pump_ns.fetch_add(p1 - p0, std::memory_order_relaxed);
    int active = 0;
    // every registered schedule, by id (a schedule deleted meanwhile is freed only two
    // epochs after its entry was cleared, so one read here stays valid for this pass)
    const int end = g_id_end.load(std::memory_order_acquire);
    for (int id = 0; id < end; ++id) {
        if (quiet(id)) continue;
        Sched *s = g_by_id[id].load(std::memory_order_acquire);
        if (!s) continue;
        while (step(*s)) any = true;   // run a schedule until it has to wait
        // in flight, or posted and waiting for its activation (majority: the drawn
        // activator's post; solo: a sync round's last poster): the join is imminent and
        // its latency adds to the round, so the thread keeps polling instead of sleeping
        if (s->stage != ST_IDLE || s->awaiting) ++active;
    }
    g_active.store(active, std::memory_order_relaxed);
    g_epoch.fetch_add(1, std::memory_order_acq_rel);
    if (any) {   // idle passes are not counted: they only poll
        g_prof_passes.fetch_add(1, std::memory_order_relaxed);
        g_prof_pass_ns.fetch_add(mono_ns() - p0, std::memory_order_relaxed);
    }
    return any;
}

}  // namespace esgd
