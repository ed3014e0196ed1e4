// engine.h — persistent partial-allreduce schedules and the progress thread.
//
// Observable contract restated from fflib2 (paths under
// /root/reference/eager-SGD-modules/fflib2/src):
//   * A schedule is created collectively and reused every round
//     (colls/ffsolo_allreduce.c:20-95, colls/ffrand_allreduce.c:27-75).
//   * Solo: post() of round t goes through the limiter (colls/ffsolo_limiter.c:4-35):
//     rounds 1..async are asynchronous, round async+1 is synchronous, then repeat.
//     An asynchronous round is activated by the FIRST rank that posts it; the
//     activation floods to every rank (colls/ffactivation.c:11-106), and each rank joins
//     with whatever its send buffer holds at that moment (the `move` of
//     colls/ffallreduce.c:126-130).  A synchronous round is joined by each rank when it
//     posts (no activation).
//   * Majority: round t is activated by rank rand_r(&seed) % P, the same draw on every
//     rank (colls/ffrand_allreduce.c:83-103); the others only count passive rounds.
//   * Plain allreduce: every round synchronous (colls/ffallreduce.c).
//   * wait() returns once the next round not yet waited for has completed locally
//     (ffop.c:143-177 waits for version wait_version+1 of allreduce_ends).
// The fflib2 op-DAG/version machinery that implements this is not rebuilt: a round
// counter per schedule in shared memory plays the role of the op versions.
#pragma once

#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "esgd.h"
#include "shm.h"

namespace esgd {

enum Kind { KIND_ALLREDUCE = 0, KIND_SOLO = 1, KIND_MAJORITY = 2 };

// Schedule creation from the C ABIs (comm_api.cpp): transport by esgd_set_transport /
// ESGD_TRANSPORT; tag as ff.h passes it (or kNoTag).
int create_schedule(int kind, int buf, const void *sb, void *rb, uint64_t count, int dtype, int async,
                    unsigned seed, unsigned flags, int tag, uint64_t *out);

enum Stage {
    ST_IDLE = 0,      // between rounds
    ST_WAIT_TICKET,   // joined; waiting for this round's turn in the node's issue ring
    ST_INFLIGHT,      // the whole round is queued on the GPU (or moving nothing)
};

struct Sched;

// A round's own data (esgd_schedule_post_io): the snapshot reads src / div instead of the
// send bucket, and the result lands in dst instead of rb -- if the round is joined at or
// after that post (fresh).
struct RoundIOSegs {   // esgd_schedule_post_iov: the round's data in pieces (fp32)
    std::vector<const float *> src;
    std::vector<float *> dst;
    std::vector<uint64_t> count;
};
struct RoundIO {
    const void *src;
    void *dst;
    float div;
    std::shared_ptr<const RoundIOSegs> segs = nullptr;   // set: src / dst unused
};

// Data movement of one round.  A round is joined on the host (activation rules,
// buffer re-resolution, host staging: prepare()), then queued on the GPU as a whole
// (launch()), in one node-wide order: every rank launches the rounds of all schedules
// in the same sequence (the issue ring), so the GPU-side waits of one round can never
// wait on a round that a peer queued behind another wait.  query() reports whether the
// launched round has finished (1), is pending (0) or failed (< 0).
struct Transport {
    virtual ~Transport() {}
    virtual const char *name() const = 0;
    // creation, in two voted steps: setup() is local (buffers, streams, publishing
    // this rank's bucket); connect() runs once every rank's setup() succeeded (mapping
    // peers, communicator bring-up).  A failure in either fails the creation on all ranks.
    virtual int setup(Sched &s) = 0;
    virtual int connect(Sched &) { return ESGD_SUCCESS; }
    // a peer could not map this rank's publication (`which`: SchedShm::remap bits): move
    // it to a chunk allocated anew and publish again (creation only, before any round)
    virtual int remap(Sched &, uint32_t) { return ESGD_SUCCESS; }
    virtual int note_producer(Sched &s, uint32_t round, void *stream) = 0;
    // the post of `round` carries its own data (RoundIO); checked here, used at launch
    virtual int note_io(Sched &s, uint32_t round, const RoundIO &io);   // default: refused
    // hold mode: the caller's reads of rb / writes of sb queued on `stream` (after
    // wait()) must finish before the next round's snapshot touches the buckets
    virtual int note_consumer(Sched &, void *) { return ESGD_SUCCESS; }
    virtual int prepare(Sched &s, uint32_t round, bool fresh) = 0;
    virtual int launch(Sched &s, uint32_t round, bool fresh) = 0;
    virtual int query(Sched &s) = 0;
    // host-side work once the copy-out has landed (before wait() returns)
    virtual int complete(Sched &) { return ESGD_SUCCESS; }
    // why a launched round has not finished (timeouts), "" if unknown
    virtual std::string diagnose(Sched &) { return std::string(); }
    virtual void teardown(Sched &s) = 0;
};

struct RoundLog {      // per-round record kept for tests / stats (bounded ring)
    uint32_t round;
    uint8_t fresh;     // this rank had posted the round before it joined
    uint8_t sync;
    int16_t activator; // -1 for synchronous rounds
};

struct Sched {
    int id = -1, kind = KIND_ALLREDUCE, async = 0, dtype = 3;
    unsigned seed = 0;
    uint64_t count = 0;
    size_t esize = 4;
    int rank = 0, world = 1;
    SchedShm *sh = nullptr;
    std::atomic<uint32_t> *activated = nullptr;   // Segment::activated[id]
    uint32_t gen = 0;
    int connect_attempt = 0;   // creation: which connect attempt maps peers now (SchedShm::remap)
    int remaps = 0;            // creation retries this schedule needed (diagnostics)
    Transport *tp = nullptr;
    void *tstate = nullptr;

    // caller buffers (captured at creation, like colls/ffallreduce.c:113-115)
    void *sb = nullptr, *rb = nullptr;
    bool host_mode = false, in_place = false;
    // FFCOLL_BUFFERS: buffers are re-resolved at every post (colls/ffallreduce.c:20-52
    // checks type / size and grows the temporaries); returns an esgd status
    int (*resolve)(Sched &s) = nullptr;
    void *resolve_ctx = nullptr;
    void (*resolve_free)(void *ctx) = nullptr;

    std::mutex mu;
    std::condition_variable cv;
    std::atomic<uint32_t> posted{0};
    // joined and stage change only under mu; atomic so that the progress pass can skip a
    // quiet idle schedule without taking mu (engine_progress_once)
    std::atomic<uint32_t> joined{0};
    uint32_t completed = 0, waited = 0;
    std::atomic<uint32_t> completed_a{0};   // = completed, for wait()'s lock-free spin
    std::atomic<Stage> stage{ST_IDLE};
    uint32_t cur = 0;
    bool cur_fresh = false;
    double stage_t0 = 0;
    int error = 0;
    char errmsg[1024] = {0};
    uint32_t passive = 0;      // majority: passive rounds since the last activation
    std::atomic<bool> awaiting{false};   // posted, waiting for the activation (written under mu)
    uint64_t roctx_round = 0;  // ESGD_ROCTX=1: the open "round" range (join -> completion)
    uint64_t n_fresh = 0, n_auto = 0, n_activated = 0;
    std::vector<RoundLog> log;
    // per-round timeline (CLOCK_MONOTONIC ns, comparable across the node's processes):
    // post, join, launch start, launch queued, completion seen, wait returned
    std::vector<std::array<uint64_t, 12>> tl;   // [6..11]: GPU spans (ESGD_GPU_TRACE=1)
    void mark(uint32_t round, int what);
    std::atomic<bool> live{true};

    // ESGD_SCHED_HOLD: once a round has completed, the next round is not joined before
    // wait() has returned it AND release() -- the caller copies rb out (and drops its late
    // send bucket) before a peer-activated round can overwrite them
    // (opt_esgd_solo...py:309-314 runs those steps synchronously right after the wait).
    // `released`: rounds the caller has released; a round is joined only once every
    // joined round has been (holding from wait() on was not enough: a peer could carry
    // this rank into the next round between the completion and the wait)
    bool hold_mode = false, held = false;
    uint32_t released = 0;
    // ESGD_SCHED_ZERO_SB: the snapshot zeroes the send bucket as it reads it (device
    // buckets): the wrapper's zero-after-use (:311-314) fused into the move
    bool zero_sb = false;
    // ESGD_SCHED_WIRE_BF16 (fp32 buckets, IPC transport): peers read a bf16 copy of the
    // bucket, half the xGMI bytes; the result is the bf16-rounded tree widened to fp32
    bool wire_bf16 = false;
    // ESGD_SCHED_FRESH_ONLY: a round joined before this rank posted it contributes zeros
    // (the snapshot zeroes the bucket instead of reading sb)
    bool fresh_only = false;
    // data-plane settings captured at creation (esgd_set_config / env defaults; part of
    // the creation signature, so every rank runs the schedule the same way)
    uint64_t small_bytes = 0;   // buckets up to this many bytes: one-launch rounds
    int flag_mode = 0;          // pairing flags: 0 host memory, 1 uncached HBM, 2 fine-grained HBM
    bool strict = false;        // one-launch rounds with round 2's strict hand-offs
    // whether this rank had posted each joined round before joining it, for the rounds
    // not yet returned by wait()/test(): a bit ring indexed by round, kFreshWindow rounds
    // deep (allocated at the first join).  Without HOLD, peers' activations can carry the
    // progress thread any number of rounds past the caller's last wait; a round more than
    // kFreshWindow rounds behind the newest join has lost its bit and is reported as not
    // fresh (counted in fresh_lost) -- memory stays bounded however long the caller lags.
    static constexpr uint32_t kFreshWindow = 1u << 16;
    std::vector<uint64_t> fresh_bits;
    uint64_t fresh_lost = 0;
    void fresh_set(uint32_t round, bool f) {
        if (fresh_bits.empty()) fresh_bits.assign(kFreshWindow / 64, 0);
        const uint32_t i = round % kFreshWindow;
        if (f) fresh_bits[i / 64] |= uint64_t(1) << (i % 64);
        else fresh_bits[i / 64] &= ~(uint64_t(1) << (i % 64));
    }
    // the bit of `round` (joined already), consumed by wait()/test()
    bool fresh_take(uint32_t round) {
        if (fresh_bits.empty() || round == 0 || round > joined) return false;
        if (joined - round >= kFreshWindow) { ++fresh_lost; return false; }
        const uint32_t i = round % kFreshWindow;
        return (fresh_bits[i / 64] >> (i % 64)) & 1;
    }
};

// Round kind / activator rules (pure functions of the schedule parameters).
bool round_is_sync(const Sched &s, uint32_t round);

// Engine lifetime: attach to the node segment and start the progress thread.
int engine_init(const char *job, int rank, int world, bool start_progress);
int engine_finalize();
bool engine_ready();
int engine_rank();
int engine_world();
Segment *engine_segment();
int engine_barrier();
double engine_timeout();

// Schedules: creation is collective, in the same order on every rank (checked: kind,
// dtype and, through ff.h, the tag must match); deletion is local.
constexpr int kNoTag = INT32_MIN;   // creation without a tag to check
int sched_create(int kind, int dtype, uint64_t count, void *sb, void *rb, bool host_mode,
                 int async, unsigned seed, Transport *tp, Sched **out, unsigned flags = 0, int tag = kNoTag);
// same, with buffers re-resolved at every post (FFCOLL_BUFFERS); ctx freed by ctx_free
int sched_create_with(int kind, int dtype, uint64_t count, void *sb, void *rb, bool host_mode,
                      int async, unsigned seed, Transport *tp, int (*resolve)(Sched &),
                      void *ctx, void (*ctx_free)(void *), Sched **out, unsigned flags = 0,
                      int tag = kNoTag);
// transport chosen by esgd_set_transport / ESGD_TRANSPORT (comm_api.cpp)
Transport *default_transport(bool control_only);
int sched_post(Sched *s, void *producer_stream, int *role, const RoundIO *io = nullptr);
int sched_wait(Sched *s);
// wait, and say whether this rank had posted the round it returns before joining it
int sched_wait_ex(Sched *s, int *fresh);
// hold mode: the caller is done with the round wait() returned; work it queued on
// `stream` (may be null) is waited for by the next round's snapshot
int sched_release(Sched *s, void *stream);
int sched_test(Sched *s, int *flag);
int sched_delete(Sched *s);
Sched *sched_lookup(uint64_t handle);

// Issue log: (schedule id, round) in the order this rank launched rounds.
int engine_issue_log(uint32_t *sched, uint32_t *round, uint32_t cap, uint32_t *n);

// esgd_comm_profile: passes, ns in passes, ns launching, joins, ns joining, launches,
// ns flushing shared launches
void engine_profile(uint64_t out[7]);
// dataplane.cpp: kernel launches of rounds and ns spent flushing shared launches
void dataplane_profile(uint64_t *launches, uint64_t *flush_ns);
// the pending / unfinished shared launches and seal I/O, for a timed-out wait's message
std::string dataplane_state();

// One polling pass over all schedules (the progress thread calls it in a loop; tests
// without a thread may call it directly).  Returns true if anything advanced.
bool engine_progress_once();

// Data-plane resources shared by all schedules of the process (dataplane.cpp): freed at
// finalize, before the node segment is unmapped.
void dataplane_shutdown();
// launch the rounds appended to the pending shared launch (k_round_batch); the engine calls
// it after every pump of the issue ring, transports before queuing anything else
int dataplane_flush();
// the end of a pump: flush unless a shared launch is still queued (kBatchDepth)
int dataplane_flush_soft();
// esgd_schedule_post_group / _release_group: until the end call, this thread's posts
// (which 0) or releases (1) on `stream` share ONE event recording
int dataplane_group_begin(int which, void *stream);
void dataplane_group_end(int which);
// a finalized job of this process had mapped peers' buckets (no new job with peers then)
bool dataplane_mappings_closed();
// settings new schedules capture (esgd_set_config; ESGD_SMALL_ROUND_BYTES / ESGD_DEVICE_FLAGS)
uint64_t config_small_round_bytes();
int config_device_flags();
bool config_strict_handoffs();
int config_set(const char *key, int64_t value);
int config_get(const char *key, int64_t *value);

}  // namespace esgd
