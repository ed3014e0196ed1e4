// shm.h — node-local shared segment that replaces fflib2's MPI control traffic.
//
// fflib2 moves activation tokens and completion through MPI point-to-point messages
// polled by a progress pthread (src/colls/ffactivation.c:11-106,
// src/components/mpi/ffop_mpi_progresser.c:34-104).  All ranks of this build live on
// one MI355X node, so the same information is a handful of atomics in a /dev/shm
// segment: activation counters (the "versions" of ffop.c), per-rank ready/done epochs
// of every round, IPC handles of the registered buckets, and a sense-reversing barrier
// (the reference's MPI_Barrier, opt_esgd_solo_imagenet_imbalance.py:295).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>

namespace esgd {

constexpr int kMaxRanks = 16;     // ranks per node
constexpr int kRemapTries = 3;    // creation retries after a peer's mapping showed other memory
constexpr int kMaxSched = 2048;   // persistent schedules per job (the ResNet-50 wrapper uses 161)
constexpr uint64_t kShmMagic = 0x324d4853444753ull;  // "ESGDSHM2" (round 5: packed activation counters)

// One registered device buffer: the allocation's IPC handle plus the offset of the
// buffer inside it (torch's caching allocator hands out sub-allocations).
struct alignas(64) IpcSlot {
    uint8_t handle[64];
    uint64_t offset;
    uint64_t bytes;
    std::atomic<uint32_t> gen;    // 1 once this rank published its bucket for this id
    std::atomic<uint32_t> ver;    // bumped at every (re)publication (buffers that grow)
    // the exported arena chunk's seal (arena.cpp, ChunkSeal): its usable bytes (the seal
    // sits right behind them), the exporter's VA of the chunk and the seal's nonce -- an
    // importer checks them through its fresh mapping (0: no seal, e.g. flag pages)
    uint64_t chunk_bytes;
    uint64_t chunk_base;
    uint64_t seal_nonce;
};

struct alignas(64) SchedShm {
    // (the highest round activated lives in Segment::activated[id], packed: every progress
    // pass reads it for every schedule, and one cache line there covers 16 schedules where a
    // field here cost a page -- SchedShm is several KiB -- apiece)
    std::atomic<int32_t> last_activator;  // diagnostics only (may lag `activated`)
    // per-round activation record, (round << 32) | (rank + 1), claimed by CAS BEFORE
    // `activated` is raised: whoever sees activated >= t also sees round t's activator
    std::atomic<uint64_t> act_of[256];
    // GPU flags (written by the GPUs through the host-registered segment, system scope):
    alignas(64) std::atomic<uint32_t> ready[kMaxRanks];   // round whose snapshot rank r has made
    alignas(64) std::atomic<uint32_t> reduced[kMaxRanks]; // round whose reduce-scatter is done
    alignas(64) std::atomic<uint32_t> done[kMaxRanks];    // round (chunk, chunked host rounds) whose all-gather
                                                          // is done; one-launch rounds have no done pairing
    alignas(64) std::atomic<uint32_t> gpu_err[kMaxRanks]; // round whose flag wait timed out
    alignas(64) std::atomic<uint32_t> fin[kMaxRanks];     // round a one-launch round finished
    // ESGD_GPU_TRACE=1: wall-clock (entry, exit) of the pairings of the last round
    alignas(64) uint64_t gpu_ts[kMaxRanks][6];
    std::atomic<uint32_t> joined[kMaxRanks];  // diagnostics: last round rank r joined
    std::atomic<uint32_t> activations[kMaxRanks];  // diagnostics: rounds activated by r
    std::atomic<uint32_t> ready_count;   // joins so far, all ranks (issue-ring append)
    std::atomic<uint32_t> setup_err;     // ranks whose setup failed (first creation vote)
    std::atomic<uint32_t> connect_err;   // ranks whose connect failed (the second creation vote)
    std::atomic<uint64_t> sig[kMaxRanks];   // creation signature of rank r: kind, dtype, tag
    IpcSlot slot[kMaxRanks];   // rank r's receive bucket (peers read shard q of it in phase 1)
    IpcSlot pub[kMaxRanks];    // rank r's reduced shard, published for the all-gather
    // A peer's fresh mapping of rank r's publication showed other memory (the chunk seal,
    // dataplane.cpp ipc_open) at connect attempt a: remap[a][r] (bit 1 the bucket, bit 2
    // the published shard) asks rank r to move it to a chunk allocated anew; every rank
    // then re-maps (sched_create_with's retry votes, retry_err)
    std::atomic<uint32_t> remap[kRemapTries + 1][kMaxRanks];
    std::atomic<uint32_t> retry_err[2 * kRemapTries];
};

// Global issue order for transports whose collectives must be issued in the same
// order on every rank (RCCL): the rank that completes a round's readiness appends it.
constexpr int kRing = 4096;
struct alignas(16) TicketSlot {
    std::atomic<uint64_t> tag;   // ticket + 1 once the slot is filled
    uint32_t sched;
    uint32_t round;
};

struct Segment {
    uint64_t magic;
    uint32_t world;
    uint32_t bytes;
    std::atomic<uint32_t> attached;
    std::atomic<uint32_t> bar_count;
    std::atomic<uint32_t> bar_gen;
    std::atomic<uint32_t> aborted;
    // idle progress threads sleep on this word (futex); activations, issue-ring appends
    // and posts bump it, so a peer's activation is seen within a wake-up, not a backoff
    std::atomic<uint32_t> wake_seq;
    std::atomic<uint32_t> sleepers;
    std::atomic<uint32_t> nccl_ready;
    uint8_t nccl_id[128];
    // creator liveness for ranks attaching to a file of this name: rank 0's PID namespace
    // (inode of /proc/self/ns/pid) and a heartbeat (CLOCK_MONOTONIC ns) that every rank
    // waiting in the init barrier keeps fresh -- a creator in another PID namespace (one
    // container per GPU sharing /dev/shm) cannot be probed with kill()
    uint64_t creator_pidns;
    std::atomic<uint64_t> beat_ns;
    std::atomic<int32_t> pid[kMaxRanks];
    std::atomic<int32_t> device[kMaxRanks];
    // the physical GPU of rank r ((PCI domain, bus, device) + 1; 0: none): device ordinals
    // are per process (HIP_VISIBLE_DEVICES may give every rank "device 0")
    std::atomic<uint64_t> gpu_id[kMaxRanks];
    std::atomic<uint64_t> ticket_next;
    // device pairing flags: rank r's flag page of mode m + 1 (1 uncached, 2 fine-grained
    // HBM; dataplane.cpp)
    IpcSlot flagpage[2][kMaxRanks];
    TicketSlot ring[kRing];
    // highest round activated of schedule id (solo async / majority): raised by the
    // activator's CAS (engine.cpp activate), read by every rank's progress pass
    alignas(64) std::atomic<uint32_t> activated[kMaxSched];
    SchedShm sched[kMaxSched];
};

// Attach (rank 0 creates) the segment /dev/shm/esgd-<job>.  Returns nullptr and sets
// the error message on failure / timeout.
Segment *shm_attach(const char *job, int rank, int world, double timeout_s);
void shm_detach(Segment *seg, const char *job, int rank);
void shm_unlink_name(const char *job);

// Sense-reversing barrier over the segment; ESGD_ERROR on timeout or abort.
int shm_barrier(Segment *seg, int world, double timeout_s);

// Wake every progress thread of the node sleeping in seg_idle_wait (cheap when none is).
void seg_wake(Segment *seg);
// Sleep until seg->wake_seq differs from `seen` or `usec` elapsed.
void seg_idle_wait(Segment *seg, uint32_t seen, unsigned usec);

// Seconds since an arbitrary epoch (steady clock).
double now_s();
// Spin-then-yield-then-sleep backoff for polling loops.
void backoff(unsigned &polls);

}  // namespace esgd
