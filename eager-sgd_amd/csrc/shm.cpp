// shm.cpp — creation / attachment of the node-local segment and its barrier.
#include "shm.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>

#include "esgd_internal.h"

namespace esgd {

double now_s() {
    using namespace std::chrono;
    return duration<double>(steady_clock::now().time_since_epoch()).count();
}

void backoff(unsigned &polls) {
    ++polls;
    if (polls < 64) return;                      // tight spin: sub-microsecond hand-offs
    if (polls < 2048) { sched_yield(); return; }
    std::this_thread::sleep_for(std::chrono::microseconds(polls < 16384 ? 5 : 50));
}

// The segment is a MAP_SHARED file mapping, so a (non-private) futex on one of its words
// works across the node's processes.
static long futex(std::atomic<uint32_t> *w, int op, uint32_t val, const struct timespec *ts) {
    return syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), op, val, ts, nullptr, 0);
}

void seg_wake(Segment *seg) {
    if (!seg) return;
    seg->wake_seq.fetch_add(1, std::memory_order_acq_rel);
    if (seg->sleepers.load(std::memory_order_acquire)) futex(&seg->wake_seq, FUTEX_WAKE, INT32_MAX, nullptr);
}

void seg_idle_wait(Segment *seg, uint32_t seen, unsigned usec) {
    seg->sleepers.fetch_add(1, std::memory_order_acq_rel);
    if (seg->wake_seq.load(std::memory_order_acquire) == seen) {
        struct timespec ts = {time_t(usec / 1000000u), long(usec % 1000000u) * 1000L};
        (void)futex(&seg->wake_seq, FUTEX_WAIT, seen, &ts);
    }
    seg->sleepers.fetch_sub(1, std::memory_order_acq_rel);
}

static uint64_t mono_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch()).count());
}

static uint64_t pid_namespace() {
    struct stat st;
    return stat("/proc/self/ns/pid", &st) == 0 ? uint64_t(st.st_ino) : 0;
}

// A segment left behind by a crashed job with the same id: its creator is gone.  In the
// creator's PID namespace kill(pid, 0) says so; from another namespace the pid means
// nothing, and the creator counts as alive while the init barrier's heartbeat is fresh
// (stamped every millisecond by every waiting rank; a dead job's stops).
static bool creator_alive(const Segment *seg) {
    const uint64_t ns = pid_namespace();
    if (ns && seg->creator_pidns == ns) {
        const int32_t pid = seg->pid[0].load();
        return pid > 0 && (kill(pid, 0) == 0 || errno == EPERM);
    }
    const uint64_t beat = seg->beat_ns.load(std::memory_order_acquire);
    return beat && mono_ns() - beat < uint64_t(2000000000);
}

static std::string shm_path(const char *job) {
    std::string p = "/dev/shm/esgd-";
    for (const char *c = job; *c; ++c) p += (isalnum((unsigned char)*c) || *c == '-' || *c == '_') ? *c : '_';
    return p;
}

Segment *shm_attach(const char *job, int rank, int world, double timeout_s) {
    if (!job || !*job) { set_error("shm_attach: empty job id"); return nullptr; }
    if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world) {
        set_error("shm_attach: rank %d / world %d outside [0, %d)", rank, world, kMaxRanks);
        return nullptr;
    }
    const std::string path = shm_path(job);
    const size_t bytes = sizeof(Segment);
    void *mem = MAP_FAILED;
    if (rank == 0) {
        // build under a private name, publish atomically with rename(): a peer can only
        // ever open a fully initialised segment.
        const std::string tmp = path + ".tmp." + std::to_string(getpid());
        int fd = open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
        if (fd < 0) { set_error("shm_attach: open %s failed", tmp.c_str()); return nullptr; }
        if (ftruncate(fd, (off_t)bytes) != 0) {
            close(fd); unlink(tmp.c_str());
            set_error("shm_attach: ftruncate %zu failed", bytes);
            return nullptr;
        }
        mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (mem == MAP_FAILED) { unlink(tmp.c_str()); set_error("shm_attach: mmap failed"); return nullptr; }
        std::memset(mem, 0, bytes);
        Segment *seg = static_cast<Segment *>(mem);
        seg->world = uint32_t(world);
        seg->bytes = uint32_t(bytes);
        seg->pid[0].store(int32_t(getpid()));
        seg->creator_pidns = pid_namespace();
        seg->beat_ns.store(mono_ns());
        std::atomic_thread_fence(std::memory_order_seq_cst);
        seg->magic = kShmMagic;
        if (rename(tmp.c_str(), path.c_str()) != 0) {
            munmap(mem, bytes); unlink(tmp.c_str());
            set_error("shm_attach: rename to %s failed", path.c_str());
            return nullptr;
        }
    } else {
        const double t0 = now_s();
        unsigned polls = 0;
        for (;;) {
            int fd = open(path.c_str(), O_RDWR);
            if (fd >= 0) {
                struct stat st;
                if (fstat(fd, &st) == 0 && size_t(st.st_size) == bytes) {
                    mem = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
                    close(fd);
                    if (mem != MAP_FAILED) {
                        Segment *seg = static_cast<Segment *>(mem);
                        // a stale file of an earlier job with this id (its rank 0 died before
                        // unlinking it) is skipped: rank 0 renames a fresh one over it
                        if (seg->magic == kShmMagic && seg->world == uint32_t(world) && creator_alive(seg))
                            break;
                        munmap(mem, bytes);
                        mem = MAP_FAILED;
                    }
                } else {
                    close(fd);
                }
            }
            if (now_s() - t0 > timeout_s) {
                set_error("shm_attach: rank %d timed out waiting for %s", rank, path.c_str());
                return nullptr;
            }
            backoff(polls);
        }
    }
    Segment *seg = static_cast<Segment *>(mem);
    seg->pid[rank].store(int32_t(getpid()));
    seg->attached.fetch_add(1);
    return seg;
}

void shm_unlink_name(const char *job) { unlink(shm_path(job).c_str()); }

void shm_detach(Segment *seg, const char *job, int rank) {
    if (rank == 0 && job) shm_unlink_name(job);
    if (seg) munmap(seg, sizeof(Segment));
}

int shm_barrier(Segment *seg, int world, double timeout_s) {
    if (world <= 1) return ESGD_SUCCESS;
    const uint32_t gen = seg->bar_gen.load(std::memory_order_acquire);
    if (seg->bar_count.fetch_add(1, std::memory_order_acq_rel) + 1 == uint32_t(world)) {
        seg->bar_count.store(0, std::memory_order_relaxed);
        seg->bar_gen.fetch_add(1, std::memory_order_acq_rel);
        return ESGD_SUCCESS;
    }
    const double t0 = now_s();
    unsigned polls = 0;
    uint64_t beat = 0;
    while (seg->bar_gen.load(std::memory_order_acquire) == gen) {
        const uint64_t t = mono_ns();
        if (t - beat > 1000000) {   // the creator-liveness heartbeat (creator_alive)
            seg->beat_ns.store(t, std::memory_order_release);
            beat = t;
        }
        if (seg->aborted.load(std::memory_order_relaxed)) {
            set_error("barrier: job aborted by a peer");
            return ESGD_ERROR;
        }
        if (now_s() - t0 > timeout_s) {
            set_error("barrier: timed out after %.0f s", timeout_s);
            return ESGD_ERROR;
        }
        backoff(polls);
    }
    return ESGD_SUCCESS;
}

}  // namespace esgd
