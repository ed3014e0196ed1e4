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

#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "engine.h"
#include "esgd_internal.h"

namespace esgd {

int reduce_remote(int dtype, int k, const void *const *inputs, void *out, uint64_t count,
                  float scale, hipStream_t s);
int gather_remote(int n, const void *const *src, void *const *dst, const uint64_t *bytes,
                  hipStream_t s);

// ---- IPC mapping cache: one hipIpcOpenMemHandle per (peer, allocation) ----
struct IpcKey {
    int peer;
    uint8_t h[64];
    bool operator<(const IpcKey &o) const {
        if (peer != o.peer) return peer < o.peer;
        return std::memcmp(h, o.h, 64) < 0;
    }
};
struct IpcEntry { void *base; int refs; };
static std::mutex g_ipc_mu;
static std::map<IpcKey, IpcEntry> g_ipc;

static int ipc_open(int peer, const uint8_t *h, void **base) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    IpcKey k;
    k.peer = peer;
    std::memcpy(k.h, h, 64);
    auto it = g_ipc.find(k);
    if (it != g_ipc.end()) { ++it->second.refs; *base = it->second.base; return ESGD_SUCCESS; }
    hipIpcMemHandle_t hh;
    std::memcpy(&hh, h, sizeof(hh));
    void *p = nullptr;
    ESGD_HIP(hipIpcOpenMemHandle(&p, hh, hipIpcMemLazyEnablePeerAccess));
    g_ipc[k] = {p, 1};
    *base = p;
    return ESGD_SUCCESS;
}

static void ipc_close(void *base) {
    std::lock_guard<std::mutex> lk(g_ipc_mu);
    for (auto it = g_ipc.begin(); it != g_ipc.end(); ++it) {
        if (it->second.base == base) {
            if (--it->second.refs == 0) {
                (void)hipIpcCloseMemHandle(base);
                g_ipc.erase(it);
            }
            return;
        }
    }
}

struct IpcState {
    hipStream_t stream = nullptr;
    hipEvent_t ev = nullptr;
    char *rb_dev = nullptr;
    bool owns_rb = false, reg_sb = false, reg_rb = false;
    char *peer[kMaxRanks] = {};
    void *peer_base[kMaxRanks] = {};
    uint64_t off[kMaxRanks] = {}, len[kMaxRanks] = {};   // elements
    std::map<uint32_t, hipEvent_t> producer;
    std::vector<hipEvent_t> spare;
};

// shard j = [off_j, off_j + len_j): equal shards rounded up to 1 KiB so every shard
// (and the 16-B vectors the kernels move) starts aligned; the last one is ragged.
static void layout(Sched &s, IpcState &st) {
    const uint64_t align = 1024 / s.esize;
    uint64_t per = (s.count + uint64_t(s.world) - 1) / uint64_t(s.world);
    per = (per + align - 1) / align * align;
    for (int j = 0; j < s.world; ++j) {
        const uint64_t o = std::min<uint64_t>(s.count, per * uint64_t(j));
        st.off[j] = o;
        st.len[j] = std::min<uint64_t>(per, s.count - o);
    }
}

struct IpcTransport final : Transport {
    const char *name() const override { return "ipc"; }

    static IpcState &S(Sched &s) { return *static_cast<IpcState *>(s.tstate); }

    int setup(Sched &s) override {
        if (s.esize == 0) { set_error("schedule: unsupported dtype %d", s.dtype); return ESGD_INVALID_ARG; }
        if (int rc = require_device()) return rc;
        auto *st = new IpcState();
        s.tstate = st;
        const size_t bytes = s.count * s.esize;
        ESGD_HIP(hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking));
        ESGD_HIP(hipEventCreateWithFlags(&st->ev, hipEventDisableTiming));
        if (s.host_mode) {
            ESGD_HIP(hipMalloc(reinterpret_cast<void **>(&st->rb_dev), bytes ? bytes : 256));
            st->owns_rb = true;
            // pin the caller's persistent host buckets so the move / copy-out are DMA
            if (bytes && s.rb && hipHostRegister(s.rb, bytes, hipHostRegisterDefault) == hipSuccess)
                st->reg_rb = true;
            if (bytes && s.sb && s.sb != s.rb &&
                hipHostRegister(s.sb, bytes, hipHostRegisterDefault) == hipSuccess)
                st->reg_sb = true;
            (void)hipGetLastError();   // "already registered" is fine
        } else {
            if (!s.rb) { set_error("schedule: null receive buffer"); return ESGD_INVALID_ARG; }
            if (reinterpret_cast<uintptr_t>(s.rb) & 15) {
                set_error("schedule: device receive buffer must be 16-B aligned");
                return ESGD_INVALID_ARG;
            }
            st->rb_dev = static_cast<char *>(s.rb);
        }
        layout(s, *st);
        st->peer[s.rank] = st->rb_dev;
        if (s.world == 1) return ESGD_SUCCESS;
        // publish this rank's rb, then map every peer's
        void *base = nullptr;
        size_t size = 0;
        ESGD_HIP(hipMemGetAddressRange(&base, &size, st->rb_dev));
        hipIpcMemHandle_t h;
        ESGD_HIP(hipIpcGetMemHandle(&h, base));
        IpcSlot &mine = s.sh->slot[s.rank];
        std::memcpy(mine.handle, &h, sizeof(h));
        mine.offset = uint64_t(st->rb_dev - static_cast<char *>(base));
        mine.bytes = bytes;
        mine.gen.store(s.gen, std::memory_order_release);
        if (int rc = engine_barrier()) return rc;
        for (int q = 0; q < s.world; ++q) {
            if (q == s.rank) continue;
            IpcSlot &ps = s.sh->slot[q];
            if (ps.gen.load(std::memory_order_acquire) != s.gen) {
                set_error("schedule %d: rank %d did not publish its buffer", s.id, q);
                return ESGD_ERROR;
            }
            if (ps.bytes != bytes) {
                set_error("schedule %d: rank %d has %llu bytes, this rank %zu", s.id, q,
                          (unsigned long long)ps.bytes, bytes);
                return ESGD_INVALID_ARG;
            }
            void *pb = nullptr;
            if (int rc = ipc_open(q, ps.handle, &pb)) return rc;
            st->peer_base[q] = pb;
            st->peer[q] = static_cast<char *>(pb) + ps.offset;
        }
        return ESGD_SUCCESS;
    }

    int note_producer(Sched &s, uint32_t round, void *stream) override {
        IpcState &st = S(s);
        hipEvent_t e;
        if (!st.spare.empty()) { e = st.spare.back(); st.spare.pop_back(); }
        else ESGD_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ESGD_HIP(hipEventRecord(e, static_cast<hipStream_t>(stream)));
        st.producer[round] = e;
        return ESGD_SUCCESS;
    }

    int snapshot(Sched &s, uint32_t round, bool fresh) override {
        IpcState &st = S(s);
        // gradient producer of this round (posted before the join) must have finished
        for (auto it = st.producer.begin(); it != st.producer.end();) {
            if (it->first == round && fresh) ESGD_HIP(hipStreamWaitEvent(st.stream, it->second, 0));
            if (it->first <= round) { st.spare.push_back(it->second); it = st.producer.erase(it); }
            else ++it;
        }
        const size_t bytes = s.count * s.esize;
        if (bytes) {
            if (s.host_mode) {   // the move of ffallreduce.c:126-130, host -> HBM
                const void *src = s.sb ? s.sb : s.rb;
                ESGD_HIP(hipMemcpyAsync(st.rb_dev, src, bytes, hipMemcpyHostToDevice, st.stream));
            } else if (!s.in_place) {
                ESGD_HIP(hipMemcpyAsync(st.rb_dev, s.sb, bytes, hipMemcpyDeviceToDevice, st.stream));
            }
        }
        ESGD_HIP(hipEventRecord(st.ev, st.stream));
        return ESGD_SUCCESS;
    }

    int reduce_scatter(Sched &s) override {
        IpcState &st = S(s);
        const uint64_t n = st.len[s.rank];
        if (s.world > 1 && n) {
            const void *in[kMaxRanks];
            for (int j = 0; j < s.world; ++j) in[j] = st.peer[j] + st.off[s.rank] * s.esize;
            if (int rc = reduce_remote(s.dtype, s.world, in, st.rb_dev + st.off[s.rank] * s.esize, n,
                                       1.0f, st.stream))
                return rc;
        }
        ESGD_HIP(hipEventRecord(st.ev, st.stream));
        return ESGD_SUCCESS;
    }

    int all_gather(Sched &s) override {
        IpcState &st = S(s);
        if (s.world > 1) {
            const void *src[kMaxRanks];
            void *dst[kMaxRanks];
            uint64_t bytes[kMaxRanks];
            int n = 0;
            for (int j = 0; j < s.world; ++j) {
                if (j == s.rank || st.len[j] == 0) continue;
                src[n] = st.peer[j] + st.off[j] * s.esize;
                dst[n] = st.rb_dev + st.off[j] * s.esize;
                bytes[n] = st.len[j] * s.esize;
                ++n;
            }
            if (int rc = gather_remote(n, src, dst, bytes, st.stream)) return rc;
        }
        ESGD_HIP(hipEventRecord(st.ev, st.stream));
        return ESGD_SUCCESS;
    }

    int finish(Sched &s) override {
        IpcState &st = S(s);
        const size_t bytes = s.count * s.esize;
        if (s.host_mode && bytes)
            ESGD_HIP(hipMemcpyAsync(s.rb, st.rb_dev, bytes, hipMemcpyDeviceToHost, st.stream));
        ESGD_HIP(hipEventRecord(st.ev, st.stream));
        return ESGD_SUCCESS;
    }

    int query(Sched &s) override {
        hipError_t e = hipEventQuery(S(s).ev);
        if (e == hipSuccess) return 1;
        if (e == hipErrorNotReady) return 0;
        return hip_fail(e, "hipEventQuery", __FILE__, __LINE__);
    }

    void teardown(Sched &s) override {
        IpcState *st = static_cast<IpcState *>(s.tstate);
        if (!st) return;
        if (st->stream) (void)hipStreamSynchronize(st->stream);
        for (int q = 0; q < kMaxRanks; ++q)
            if (st->peer_base[q]) ipc_close(st->peer_base[q]);
        if (st->owns_rb) (void)hipFree(st->rb_dev);
        if (st->reg_rb) (void)hipHostUnregister(s.rb);
        if (st->reg_sb) (void)hipHostUnregister(s.sb);
        for (auto &kv : st->producer) (void)hipEventDestroy(kv.second);
        for (hipEvent_t e : st->spare) (void)hipEventDestroy(e);
        if (st->ev) (void)hipEventDestroy(st->ev);
        if (st->stream) (void)hipStreamDestroy(st->stream);
        delete st;
        s.tstate = nullptr;
    }
};

struct NullTransport final : Transport {
    const char *name() const override { return "none"; }
    int setup(Sched &) override { return ESGD_SUCCESS; }
    int note_producer(Sched &, uint32_t, void *) override { return ESGD_SUCCESS; }
    int snapshot(Sched &, uint32_t, bool) override { return ESGD_SUCCESS; }
    int reduce_scatter(Sched &) override { return ESGD_SUCCESS; }
    int all_gather(Sched &) override { return ESGD_SUCCESS; }
    int finish(Sched &) override { return ESGD_SUCCESS; }
    int query(Sched &) override { return 1; }
    void teardown(Sched &) override {}
};

Transport *ipc_transport() {
    static IpcTransport t;
    return &t;
}

Transport *null_transport() {
    static NullTransport t;
    return &t;
}

hipStream_t sched_stream(Sched &s) {
    if (!s.tstate || s.tp != ipc_transport()) return nullptr;
    return static_cast<IpcState *>(s.tstate)->stream;
}

}  // namespace esgd
