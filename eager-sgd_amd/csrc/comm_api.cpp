// comm_api.cpp — C ABI of the node communicator and the persistent schedules (esgd.h).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "engine.h"
#include "esgd_internal.h"

namespace esgd {
Transport *ipc_transport();
Transport *rccl_transport();
Transport *null_transport(bool ordered);
hipStream_t sched_stream(Sched &s);
}  // namespace esgd

static std::string g_transport;   // "" -> env ESGD_TRANSPORT -> "ipc"

static const char *transport_name() {
    if (!g_transport.empty()) return g_transport.c_str();
    const char *e = getenv("ESGD_TRANSPORT");
    return (e && *e) ? e : "ipc";
}

namespace esgd {
Transport *default_transport(bool control_only) {
    const bool rccl = !std::strcmp(transport_name(), "rccl");
    if (control_only) return null_transport(rccl);
    return rccl ? rccl_transport() : ipc_transport();
}
}  // namespace esgd

namespace esgd {
int create_schedule(int kind, int buf, const void *sb, void *rb, uint64_t count, int dtype, int async,
                    unsigned seed, unsigned flags, int tag, uint64_t *out) {
    ESGD_ARG(out, "esgd_schedule_create: null output");
    ESGD_ARG((flags & ~unsigned(ESGD_SCHED_HOLD | ESGD_SCHED_ZERO_SB | ESGD_SCHED_WIRE_BF16 |
                                ESGD_SCHED_FRESH_ONLY)) == 0,
             "esgd_schedule_create: unknown flags 0x%x", flags);
    ESGD_ARG(!(flags & ESGD_SCHED_WIRE_BF16) || dtype == ESGD_FLOAT,
             "esgd_schedule_create: ESGD_SCHED_WIRE_BF16 needs FLOAT buckets (dtype %d)", dtype);
    ESGD_ARG(buf == ESGD_BUF_DEVICE || buf == ESGD_BUF_HOST || buf == ESGD_BUF_NONE,
             "esgd_schedule_create: bad buffer kind %d", buf);
    ESGD_ARG(esgd_dtype_size(dtype) > 0, "esgd_schedule_create: unsupported dtype %d", dtype);
    ESGD_ARG(buf == ESGD_BUF_NONE || rb || count == 0, "esgd_schedule_create: null receive buffer");
    const bool rccl = !std::strcmp(transport_name(), "rccl");
    ESGD_ARG(rccl || !std::strcmp(transport_name(), "ipc"), "unknown transport '%s'", transport_name());
    Transport *tp = default_transport(buf == ESGD_BUF_NONE);
    Sched *s = nullptr;
    int rc = sched_create(kind, dtype, count, const_cast<void *>(sb), rb, buf == ESGD_BUF_HOST,
                          async, seed, tp, &s, flags, tag);
    if (rc) return rc;
    *out = reinterpret_cast<uint64_t>(s);
    return ESGD_SUCCESS;
}
}  // namespace esgd

using namespace esgd;

static Sched *handle_to_sched(esgd_sched_h h) {
    Sched *s = sched_lookup(h);
    if (!s) set_error("unknown or deleted schedule handle 0x%llx", (unsigned long long)h);
    return s;
}

extern "C" {

int esgd_comm_init(const char *job_id, int rank, int world) {
    ESGD_ARG(job_id && *job_id, "esgd_comm_init: empty job id");
    return engine_init(job_id, rank, world, true);
}

int esgd_comm_finalize(void) {
    return engine_finalize();   // frees the data plane (dataplane_shutdown) too
}

int esgd_set_transport(const char *name) {
    ESGD_ARG(name && (!std::strcmp(name, "ipc") || !std::strcmp(name, "rccl")),
             "esgd_set_transport: 'ipc' or 'rccl'");
    g_transport = name;
    return ESGD_SUCCESS;
}

int esgd_set_config(const char *key, int64_t value) { return config_set(key, value); }

int esgd_get_config(const char *key, int64_t *value) { return config_get(key, value); }

int esgd_comm_issue_log(uint32_t *sched, uint32_t *round, uint32_t cap, uint32_t *n) {
    return engine_issue_log(sched, round, cap, n);
}

int esgd_comm_profile(uint64_t *out, int n) {
    ESGD_ARG(out || n <= 0, "esgd_comm_profile: null output");
    uint64_t v[ESGD_PROFILE_WORDS];
    engine_profile(v);
    for (int i = 0; i < n && i < ESGD_PROFILE_WORDS; ++i) out[i] = v[i];
    return ESGD_SUCCESS;
}

int esgd_comm_rank(int *rank) {
    ESGD_ARG(rank, "esgd_comm_rank: null pointer");
    *rank = engine_rank();
    return ESGD_SUCCESS;
}

int esgd_comm_size(int *size) {
    ESGD_ARG(size, "esgd_comm_size: null pointer");
    *size = engine_ready() ? engine_world() : 1;
    return ESGD_SUCCESS;
}

int esgd_barrier(void) { return engine_barrier(); }

int esgd_schedule_create(int kind, int buf, const void *sb, void *rb, uint64_t count, int dtype,
                         int async, unsigned seed, esgd_sched_h *out) {
    return esgd_schedule_create_ex(kind, buf, sb, rb, count, dtype, async, seed, 0, out);
}

int esgd_schedule_create_ex(int kind, int buf, const void *sb, void *rb, uint64_t count, int dtype,
                            int async, unsigned seed, unsigned flags, esgd_sched_h *out) {
    return esgd::create_schedule(kind, buf, sb, rb, count, dtype, async, seed, flags, esgd::kNoTag, out);
}

int esgd_schedule_post(esgd_sched_h h, void *producer_stream, int *role) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    return sched_post(s, producer_stream, role);
}

int esgd_schedule_post_group(const esgd_sched_h *hs, int n, void *producer_stream, int *roles) {
    ESGD_ARG(n >= 0 && (n == 0 || hs), "esgd_schedule_post_group: bad arguments");
    dataplane_group_begin(0, producer_stream);
    int rc = ESGD_SUCCESS;
    for (int i = 0; i < n && !rc; ++i) {
        Sched *s = handle_to_sched(hs[i]);
        rc = s ? sched_post(s, producer_stream, roles ? &roles[i] : nullptr) : ESGD_INVALID_ARG;
    }
    dataplane_group_end(0);
    return rc;
}

int esgd_schedule_post_io(esgd_sched_h h, const void *src, void *dst, float divisor, void *producer_stream,
                          int *role) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    const RoundIO io{src, dst, divisor};
    return sched_post(s, producer_stream, role, &io);
}

int esgd_schedule_post_iov(esgd_sched_h h, int n, const float *const *srcs, float *const *dsts,
                           const uint64_t *counts, float divisor, void *producer_stream, int *role) {
    ESGD_ARG(n >= 0 && (n == 0 || (srcs && dsts && counts)), "esgd_schedule_post_iov: bad arguments");
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    auto g = std::make_shared<RoundIOSegs>();
    g->src.assign(srcs, srcs + n);
    g->dst.assign(dsts, dsts + n);
    g->count.assign(counts, counts + n);
    RoundIO io{nullptr, nullptr, divisor};
    io.segs = std::move(g);
    return sched_post(s, producer_stream, role, &io);
}

int esgd_schedule_post_group_io(const esgd_sched_h *hs, int n, const void *const *srcs, void *const *dsts,
                                float divisor, void *producer_stream, int *roles) {
    ESGD_ARG(n >= 0 && (n == 0 || (hs && srcs && dsts)), "esgd_schedule_post_group_io: bad arguments");
    dataplane_group_begin(0, producer_stream);
    int rc = ESGD_SUCCESS;
    for (int i = 0; i < n && !rc; ++i) {
        Sched *s = handle_to_sched(hs[i]);
        const RoundIO io{srcs[i], dsts[i], divisor};
        rc = s ? sched_post(s, producer_stream, roles ? &roles[i] : nullptr, &io) : ESGD_INVALID_ARG;
    }
    dataplane_group_end(0);
    return rc;
}

int esgd_schedule_release_group(const esgd_sched_h *hs, int n, void *stream) {
    ESGD_ARG(n >= 0 && (n == 0 || hs), "esgd_schedule_release_group: bad arguments");
    dataplane_group_begin(1, stream);
    int rc = ESGD_SUCCESS;
    for (int i = 0; i < n && !rc; ++i) {
        Sched *s = handle_to_sched(hs[i]);
        rc = s ? sched_release(s, stream) : ESGD_INVALID_ARG;
    }
    dataplane_group_end(1);
    return rc;
}

int esgd_schedule_wait(esgd_sched_h h) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    return sched_wait(s);
}

int esgd_schedule_wait_ex(esgd_sched_h h, int *fresh) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    return sched_wait_ex(s, fresh);
}


int esgd_schedule_release(esgd_sched_h h, void *stream) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    return sched_release(s, stream);   // ESGD_STREAM_NULL: the legacy default stream
}

int esgd_schedule_test(esgd_sched_h h, int *flag) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    return sched_test(s, flag);
}

int esgd_schedule_delete(esgd_sched_h h) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    return sched_delete(s);
}

int esgd_schedule_stats(esgd_sched_h h, esgd_sched_stats_t *out) {
    ESGD_ARG(out, "esgd_schedule_stats: null output");
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    std::lock_guard<std::mutex> lk(s->mu);
    out->posted = s->posted.load();
    out->joined = s->joined;
    out->completed = s->completed;
    out->waited = s->waited;
    out->activated = s->activated->load();
    out->last_activator = s->sh->last_activator.load();
    out->fresh_rounds = s->n_fresh;
    out->auto_rounds = s->n_auto;
    out->activations = s->n_activated;
    return ESGD_SUCCESS;
}

int esgd_schedule_log(esgd_sched_h h, uint32_t *rounds, uint8_t *fresh, uint8_t *sync,
                      int16_t *activator, uint32_t cap, uint32_t *n) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    std::lock_guard<std::mutex> lk(s->mu);
    const uint32_t total = uint32_t(s->log.size());
    for (uint32_t i = 0; i < total && i < cap; ++i) {
        if (rounds) rounds[i] = s->log[i].round;
        if (fresh) fresh[i] = s->log[i].fresh;
        if (sync) sync[i] = s->log[i].sync;
        if (activator) activator[i] = s->log[i].activator;
    }
    if (n) *n = total;
    return ESGD_SUCCESS;
}

int esgd_schedule_timeline(esgd_sched_h h, uint64_t *t, uint32_t cap, uint32_t *n) {
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    std::lock_guard<std::mutex> lk(s->mu);
    const uint32_t total = std::min<uint32_t>(uint32_t(s->tl.size()), s->completed);
    for (uint32_t i = 0; i < total && i < cap; ++i)
        for (int k = 0; k < 12; ++k) t[12 * i + k] = s->tl[i][k];
    if (n) *n = total;
    return ESGD_SUCCESS;
}

int esgd_schedule_stream(esgd_sched_h h, void **stream) {
    ESGD_ARG(stream, "esgd_schedule_stream: null output");
    Sched *s = handle_to_sched(h);
    if (!s) return ESGD_INVALID_ARG;
    *stream = sched_stream(*s);
    return ESGD_SUCCESS;
}

}  // extern "C"
