// round_batch.h — several one-launch rounds in ONE kernel (k_round_batch).
//
// The reference's wrapper issues one allreduce per gradient tensor, back to back
// (opt_esgd_solo_imagenet_imbalance.py:24-44 chains 161 ops per ResNet-50 step; each
// ffsolo_allreduce / ffrand_allreduce post is its own op-DAG run, ffsolo_allreduce.c:103-114).
// Run one kernel launch and two rank pairings per round, that call pattern pays a host
// launch and two flag round trips per bucket.  The data plane instead gathers the
// one-launch rounds that are due in the node's issue order (engine.cpp) into one launch:
// a flag-agent wave publishes each entry's `ready` (once the entry's snapshot has landed)
// and turns peers' flags into device gates, while worker workgroups walk the entries'
// snapshot tiles, phase-1 tiles, then phase-2 tiles, in ring order.  Per-entry semantics are those of k_round_small: the same
// flags, counters, published shard, fin word and tree order -- only the launch is shared.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "esgd.h"
#include "esgd_internal.h"

namespace esgd {

constexpr int kBatchMax = 64;          // rounds per launch: one agent lane each
constexpr uint32_t kBatchWorkers = 64; // worker workgroups at most, by default (k_round_small's grid)
constexpr uint32_t kBatchWorkersMax = 512;   // ... and with ESGD_BATCH_WORKERS (batch_workers_max())
constexpr uint32_t kSnapshotWorkers = 256;   // ... of a launch holding snapshot tiles, by default
// ESGD_BATCH_WORKERS (1..512, default kBatchWorkers): the worker cap of shared launches and
// of a phase's tiles per entry (dataplane.cpp; read once per process)
uint32_t batch_workers_max();
// A phase's tiles of one entry: at most kBatchWorkers (one arrival count each), at least
// 1024 16-B vectors (one pass of a 256-lane workgroup, 4 vectors per lane) per tile -- a
// lone entry gets k_round_small's parallelism, a large one few counts.
inline void batch_tiling(uint64_t nvec, uint32_t max_tiles, uint32_t *tiles, uint32_t *tv) {
    const uint64_t want = std::max<uint64_t>(1, std::min<uint64_t>(max_tiles, (nvec + 1023) / 1024));
    uint64_t per = (nvec + want - 1) / want;
    per = std::max<uint64_t>(1024, (per + 1023) / 1024 * 1024);
    *tv = uint32_t(per);
    *tiles = uint32_t(std::max<uint64_t>(1, (nvec + per - 1) / per));
}

// One schedule's round, as the batch kernel sees it.  Built once per schedule (its
// buckets, peers' mappings and flags never move: FFCOLL_BUFFERS schedules are not batched)
// and kept in device memory, indexed by schedule id.
struct BatchDesc {
    const void *src[ESGD_MAX_FANIN];   // phase 1: shard `rank` of every rank's rb, rank order
    void *out;                         // ... folded into shard `rank` of the local rb
    void *pub;                         // ... and into this rank's published shard
    uint64_t n;                        // elements of the local shard
    const void *gsrc[ESGD_MAX_FANIN];  // phase 2: every other rank's published shard
    void *gdst[ESGD_MAX_FANIN];        // ... and where it lands in the local rb
    uint32_t gvec[ESGD_MAX_FANIN];     // 16-B vectors per segment
    uint32_t gtail[ESGD_MAX_FANIN];    // bytes after the last full vector
    uint32_t tvg[ESGD_MAX_FANIN];      // 16-B vectors per phase-2 tile of segment sg
    uint32_t t2pre[ESGD_MAX_FANIN + 1];   // phase-2 tiles before segment sg (prefix)
    uint32_t nseg;
    uint32_t tv1, t1;                  // phase 1: 16-B vectors per tile, tiles
    uint32_t strict;                   // round 2's hand-offs (ESGD_STRICT_HANDOFFS)
    PairFlags ready, reduced;
    uint32_t *fin, *err;               // SchedShm::fin[rank], gpu_err[rank] (device views)
    uint32_t *ctr;                     // device words: [0] phase-1 arrivals, [1] phase-2
                                       // arrivals, [2] ready gate, [3] reduced gate,
                                       // [4] snapshot arrivals, [5] the round that failed
                                       // here (no reduced / fin is published for it)
    // the snapshot inside the launch (BatchArgs::snap): rb = sb, or rb = 0, whole bucket
    const void *ssrc;                  // sb (nullptr: in place)
    void *sdst;                        // rb
    uint32_t svec, stail;              // 16-B vectors, bytes after them (svec 0 and stail 0:
                                       // not eligible -- the host queues such snapshots)
    // rb itself: `out` and every `gdst` lie in it; a round with its own output
    // (BatchArgs::iout) lands at the same offsets there instead
    void *rbase;
    // this rank's own shard: only this rank reads it (phase 1), so a snapshot with a source
    // (rb = src or src / div) skips it and phase 1 reads src there instead -- (P-1)/P of the
    // snapshot's bytes.  Vectors [own_v0, own_v1) of the bucket, own_tail: the ragged bytes
    // after the last vector are the own shard's; own_off: its byte offset
    uint32_t rank;
    uint32_t own_v0, own_v1, own_tail;
    uint64_t own_off;
};

// The launch's tile bookkeeping: kLaunchSlots slots of kSlotWords device words behind the
// descriptor table, launch n using slot n % kLaunchSlots.  Block 0 of every launch zeroes
// every OTHER slot before any tile is taken, so the next launch on the round stream (which
// starts only once this one has ended) finds its slot at zero whatever happened before --
// a launch that ended on a timeout, a launch the host counted as failed but that ran
// (after such a launch the host also zeroes every slot on the stream, so launches that never
// ran cannot leave a stale slot either; ADVICE r05: a device counter the host had to mirror
// could drift for good).
constexpr uint32_t kLaunchSlots = 4;
constexpr uint32_t kSlotWords = 1024;
constexpr uint32_t kSlotQueue = 0;   // next tile of the list (fetch-add)
constexpr uint32_t kSlotDone = 1;    // tiles finished (the agent block leaves at T)
constexpr uint32_t kSlotTail = 3;    // tiles deferred (each by a worker that gave its slots back)
constexpr uint32_t kSlotRing = 8;    // deferred tiles (tile + 1; 0: being written; ~0: taken)
static_assert(kSlotRing + kBatchWorkersMax <= kSlotWords, "one deferral per worker at most");

// Kernel arguments: the entries of one launch, in issue-ring order.
struct BatchArgs {
    const BatchDesc *table;            // device table, indexed by schedule id
    // Tile assignment: every worker takes the next tile of the launch's list from the slot's
    // counter, in ring order, until the list is done -- a tile is only started after every
    // earlier tile was, so the launch completes with ANY number of its workers resident.
    uint32_t *slots;                   // kLaunchSlots x kSlotWords device words
    uint32_t slot;                     // this launch's
    uint32_t nent;
    // yield (ticks, 0: never): a worker whose tile's gate stays closed this long defers the
    // tile (slot ring) and leaves, giving its wave slots back to the GPU; the agent block
    // takes deferred tiles (any whose gate is open) and, once any were deferred, open tiles
    // of the list itself.
    // Set when ranks share this GPU: a peer's launch that cannot be dispatched beside our
    // spinning workers is what opens their gates ("Forward progress").
    long long yield;
    uint32_t tile1[kBatchMax + 1];     // phase-1 tiles before entry e (prefix)
    uint32_t tile2[kBatchMax + 1];     // phase-2 tiles before entry e (prefix)
    uint16_t sid[kBatchMax];
    uint32_t value[kBatchMax];         // the round of entry e
    long long timeout;                 // wall-clock ticks any flag wait may take
    // snapshots done by the launch's own workers before the phases: entry e's kind (0 none /
    // queued before the launch, 1 rb = sb, 2 rb = 0) and its 1024-vector tiles (prefix); the
    // agent publishes e's ready once they have all landed
    uint32_t tile0[kBatchMax + 1];
    uint8_t snap[kBatchMax];           // 3: rb = isrc / idiv (fp32), the op's copy-in fused
    // the round's own send data and output (esgd_schedule_post_io): phase 0 reads isrc
    // (nullptr: the schedule's send bucket), phases 1 and 2 write iout (nullptr: rb)
    const void *isrc[kBatchMax];
    void *iout[kBatchMax];
    float idiv[kBatchMax];
};
static_assert(sizeof(BatchArgs) <= 4096, "k_round_batch's arguments must fit the kernel-argument segment");


// world: ranks (2..ESGD_MAX_FANIN); grid = workers + 1 (the agent)
int round_batch(int dtype, int world, const BatchArgs &a, unsigned workers, hipStream_t s);
// workgroups of the batch kernel for (dtype, world) resident on this GPU at once
int round_batch_capacity(int dtype, int world);

}  // namespace esgd
