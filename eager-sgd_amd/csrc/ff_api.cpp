// ff_api.cpp — fflib2's collective entry points (include/esgd_ff.h) on the esgd engine.
//
// The caller the reference ships (the deep500 op embedded in
// test-models/tf-models-r1.11/official/utils/opt_esgd_solo_imagenet_imbalance.py:277-346)
// calls ffinit once, builds 161 persistent schedules over host buckets, then per step
// post / wait.  Those calls map 1:1 onto esgd schedules with host buffers.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <string>

#include "engine.h"
#include "esgd_ff.h"
#include "esgd_internal.h"

using namespace esgd;

static int env_int(std::initializer_list<const char *> names, int dflt) {
    for (const char *n : names)
        if (const char *v = getenv(n))
            if (*v) return atoi(v);
    return dflt;
}

static bool g_ff_owns_comm = false;

// ---- ffbuffer descriptors (src/ffbuffer.c:10-95 restated) ----
struct FFBuf {
    void *ptr = nullptr;
    uint32_t count = 0;
    int dtype = -1;
    bool selfalloc = false;
};

struct CollBuffers {      // FFCOLL_BUFFERS state of one schedule
    FFBuf *sb = nullptr;  // nullptr: in place
    FFBuf *rb = nullptr;
    int dtype = 0;
};

static int resolve_coll_buffers(Sched &s) {
    auto *cb = static_cast<CollBuffers *>(s.resolve_ctx);
    FFBuf *rb = cb->rb, *sb = cb->sb;
    // colls/ffallreduce.c:32-40: datatype and size must agree
    if (rb->dtype != cb->dtype || (sb && (sb->dtype != rb->dtype || sb->count != rb->count))) {
        set_error("FFCOLL_BUFFERS: datatype / size mismatch between send, receive and schedule");
        return ESGD_INVALID_ARG;
    }
    s.rb = rb->ptr;
    s.sb = sb ? sb->ptr : nullptr;
    s.in_place = (sb == nullptr || sb->ptr == rb->ptr);
    s.count = rb->count;
    return ESGD_SUCCESS;
}

static int make_schedule(int kind, void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h op,
                         ffdatatype_h dt, int options, int async, unsigned seed, ffschedule_h *sched) {
    ESGD_ARG(sched, "fflib: null schedule output");
    ESGD_ARG(count >= 0, "fflib: negative count");
    ESGD_ARG(op == FFSUM, "fflib: only FFSUM is reduced by libesgd (operator %d)", op);
    const bool coll_buffers = (options & FFCOLL_BUFFERS) != 0;
    ESGD_ARG(!(coll_buffers && (options & ESGD_FF_DEVICE_BUFFERS)),
             "fflib: FFCOLL_BUFFERS buckets are host buffers");
    ESGD_ARG(dt == FFINT32 || dt == FFINT64 || dt == FFDOUBLE || dt == FFFLOAT || dt == ESGD_FFBF16,
             "fflib: unsupported datatype %d", dt);
    if (!engine_ready()) {
        if (int rc = ffinit(nullptr, nullptr)) return rc;
    }
    const int buf = (options & ESGD_FF_DEVICE_BUFFERS) ? ESGD_BUF_DEVICE : ESGD_BUF_HOST;
    esgd_sched_h h = 0;
    if (coll_buffers) {
        // colls/ffallreduce.c:104-110: the arguments point at ffbuffer_h handles
        ESGD_ARG(rcvbuff, "fflib: null receive buffer handle");
        auto *cb = new CollBuffers();
        cb->rb = reinterpret_cast<FFBuf *>(*static_cast<ffbuffer_h *>(rcvbuff));
        cb->sb = sndbuff == FFINPLACE ? nullptr : reinterpret_cast<FFBuf *>(*static_cast<ffbuffer_h *>(sndbuff));
        cb->dtype = dt;
        Sched *s = nullptr;
        int rc = sched_create_with(kind, dt, uint64_t(cb->rb->count), cb->sb ? cb->sb->ptr : nullptr,
                                   cb->rb->ptr, true, async, seed, default_transport(false),
                                   resolve_coll_buffers, cb,
                                   [](void *p) { delete static_cast<CollBuffers *>(p); }, &s, 0, tag);
        if (rc) { delete cb; return rc; }
        *sched = reinterpret_cast<ffschedule_h>(s);
        return FFSUCCESS;
    }
    void *sb = sndbuff == FFINPLACE ? nullptr : sndbuff;
    // the tag is checked across ranks at creation (schedules match by creation order;
    // the reference matches MPI messages by tag, src/components/mpi/ffop_mpi_send.c:30)
    int rc = create_schedule(kind, buf, sb, rcvbuff, uint64_t(count), dt, async, seed, 0, tag, &h);
    if (rc) return rc;
    *sched = h;
    return FFSUCCESS;
}

extern "C" {

int ffbuffer_create(void *addr, uint32_t count, ffdatatype_h datatype, int, ffbuffer_h *out) {
    ESGD_ARG(out, "ffbuffer_create: null output");
    auto *b = new FFBuf();
    b->selfalloc = addr == nullptr;
    if (int rc = ffbuffer_resize(reinterpret_cast<ffbuffer_h>(b), addr, count, datatype)) {
        delete b;
        return rc;
    }
    *out = reinterpret_cast<ffbuffer_h>(b);
    return FFSUCCESS;
}

int ffbuffer_resize(ffbuffer_h h, void *addr, uint32_t new_count, ffdatatype_h dt) {
    auto *b = reinterpret_cast<FFBuf *>(h);
    ESGD_ARG(b, "ffbuffer_resize: null handle");
    const size_t es = esgd_dtype_size(dt), old = b->dtype >= 0 ? esgd_dtype_size(b->dtype) : 0;
    ESGD_ARG(es > 0, "ffbuffer_resize: unsupported datatype %d", dt);
    if (!addr) {   // library-owned: grow with realloc (src/ffbuffer.c:79-84)
        if (!b->ptr || size_t(new_count) * es > size_t(b->count) * old) {
            void *p = realloc(b->selfalloc ? b->ptr : nullptr, size_t(new_count) * es);
            if (!p) return FFENOMEM;
            b->ptr = p;
            b->selfalloc = true;
        }
    } else {
        if (b->selfalloc) free(b->ptr);
        b->ptr = addr;
        b->selfalloc = false;
    }
    b->count = new_count;
    b->dtype = dt;
    return FFSUCCESS;
}

int ffbuffer_delete(ffbuffer_h h) {
    auto *b = reinterpret_cast<FFBuf *>(h);
    ESGD_ARG(b, "ffbuffer_delete: null handle");
    if (b->selfalloc) free(b->ptr);
    delete b;
    return FFSUCCESS;
}

int ffbuffer_get_size(ffbuffer_h h, uint32_t *count, ffdatatype_h *datatype) {
    auto *b = reinterpret_cast<FFBuf *>(h);
    ESGD_ARG(b && count && datatype, "ffbuffer_get_size: null argument");
    *count = b->count;
    *datatype = b->dtype;
    return FFSUCCESS;
}

int ffbuffer_get_data(ffbuffer_h h, void **mem) {
    auto *b = reinterpret_cast<FFBuf *>(h);
    ESGD_ARG(b && mem, "ffbuffer_get_data: null argument");
    *mem = b->ptr;
    return FFSUCCESS;
}

int ffinit(int *, char ***) {
    if (engine_ready()) return FFSUCCESS;   // already joined (esgd_comm_init / earlier ffinit)
    // the launcher's own variables (torch.distributed.run, Open MPI, PMI, Slurm)
    const int rank = env_int({"RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK", "SLURM_PROCID"}, 0);
    const int world = env_int({"WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE", "SLURM_NTASKS"}, 1);
    const int local = env_int({"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "SLURM_LOCALID"}, rank);
    std::string job;
    if (const char *j = getenv("ESGD_JOB_ID")) job = j;
    else if (const char *t = getenv("TORCHELASTIC_RUN_ID")) job = std::string(t) + "-" + (getenv("MASTER_PORT") ? getenv("MASTER_PORT") : "0");
    else if (const char *p = getenv("MASTER_PORT")) job = std::string("port-") + p;
    else if (world == 1) job = "single-" + std::to_string(getpid());
    else {
        set_error("ffinit: %d ranks but no job id (set ESGD_JOB_ID or run under torch.distributed.run)", world);
        return FFINVALID_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0) {
        ESGD_HIP(hipSetDevice(local % ndev));
    }
    int rc = engine_init(job.c_str(), rank, world, true);
    if (!rc) g_ff_owns_comm = true;
    return rc;
}

int fffinalize(void) {
    g_ff_owns_comm = false;
    return esgd_comm_finalize();
}

int ffrank(int *rank) { return esgd_comm_rank(rank); }
int ffsize(int *size) { return esgd_comm_size(size); }

int ffallreduce(void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h op,
                ffdatatype_h datatype, int options, ffschedule_h *sched) {
    return make_schedule(KIND_ALLREDUCE, sndbuff, rcvbuff, count, tag, op, datatype, options, 0, 0, sched);
}

int ffsolo_allreduce(void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h op,
                     ffdatatype_h datatype, int options, int async, ffschedule_h *sched) {
    return make_schedule(KIND_SOLO, sndbuff, rcvbuff, count, tag, op, datatype, options, async, 0, sched);
}

int ffrand_allreduce(void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h op,
                     ffdatatype_h datatype, int options, int seed, int async, ffschedule_h *sched) {
    return make_schedule(KIND_MAJORITY, sndbuff, rcvbuff, count, tag, op, datatype, options, async,
                         unsigned(seed), sched);
}

// The reference posts the auto-activator here so activation receives are armed
// (colls/ffsolo_allreduce.c:97-101); the progress thread is always armed.
int ffschedule_start(ffschedule_h sched) {
    return sched_lookup(sched) ? FFSUCCESS : FFINVALID_ARG;
}

int ffschedule_post(ffschedule_h sched) { return esgd_schedule_post(sched, nullptr, nullptr); }
int ffschedule_post_stream(ffschedule_h sched, void *stream) { return esgd_schedule_post(sched, stream, nullptr); }
int ffschedule_wait(ffschedule_h sched) { return esgd_schedule_wait(sched); }
int ffschedule_test(ffschedule_h sched, int *flag) { return esgd_schedule_test(sched, flag); }
int ffschedule_delete(ffschedule_h sched) { return esgd_schedule_delete(sched); }

}  // extern "C"

// ---- single computations: ffcomp (src/ffcomp.c:7-38) -----------------------------------
// The reference's direct handle on its reduction kernel: an op that, when posted, runs
// ffop_gcomp_execute once -- size = MIN of the three buffers' counts, c = a + b (FFSUM,
// ffop_gcomp_operator.c:33-58, operand a first) or c = a (FFIDENTITY, the move, :61-72) --
// and completes (ffop_gcomp.c:29-64).  Here the post queues the tree kernel (k = 2, the
// same operand order as esgd_vsum) on the library stream: host buffers through
// esgd_reduce_host (the reference's buffers are host memory), device buffers with
// ESGD_FF_DEVICE_BUFFERS; an event marks completion for ffop_wait / ffop_test.
namespace {
struct FFComp {
    void *a = nullptr, *b = nullptr, *c = nullptr;   // addresses (ffcomp)
    FFBuf *ba = nullptr, *bb = nullptr, *bc = nullptr;   // descriptors (ffcomp_b)
    int count = 0, dtype = 0, op = FFSUM;
    // a user operator's function, captured when the comp is made: the reference copies the
    // operator descriptor into the op (ffop_gcomp.c:9, ffop_gcomp_operator_get), so deleting
    // or re-creating the handle afterwards changes nothing for this comp
    ffoperator_fun_t fun = nullptr;
    bool device = false;
    hipEvent_t ev = nullptr;
    bool posted = false;
    bool host_done = false;   // a user operator's post ran its function already
};

// user operators (ffcomp_operator_create): handle FFCUSTOM + slot, as the reference numbers
// them (ffop_gcomp_operator.c:124-141); a deleted slot is reused
constexpr int kMaxCustomOps = 64;
std::mutex g_custom_mu;
ffoperator_fun_t g_custom[kMaxCustomOps] = {};

ffoperator_fun_t custom_fun(int op) {
    if (op < FFCUSTOM || op >= FFCUSTOM + kMaxCustomOps) return nullptr;
    std::lock_guard<std::mutex> lk(g_custom_mu);
    return g_custom[op - FFCUSTOM];
}

int comp_make(FFComp *o, ffop_h *out) {
    o->fun = custom_fun(o->op);
    const bool custom = o->fun != nullptr;
    ESGD_ARG(o->op == FFSUM || o->op == FFIDENTITY || custom,
             "ffcomp: operator %d -- FFSUM, FFIDENTITY or a handle from ffcomp_operator_create", o->op);
    ESGD_ARG(!custom || !o->device,
             "ffcomp: a user operator is a host function: host buffers only (not ESGD_FF_DEVICE_BUFFERS)");
    ESGD_ARG(esgd_dtype_size(o->dtype) > 0, "ffcomp: unsupported datatype %d", o->dtype);
    *out = reinterpret_cast<ffop_h>(o);
    return FFSUCCESS;
}
}  // namespace

extern "C" {

int ffcomp(void *addr1, void *addr2, int count, ffdatatype_h datatype, ffoperator_h op, int options,
           void *addr3, ffop_h *out) {
    ESGD_ARG(out && addr1 && addr3 && count >= 0, "ffcomp: null buffer or output, or negative count");
    ESGD_ARG(op == FFIDENTITY || addr2, "ffcomp: FFSUM needs two inputs");
    auto *o = new FFComp();
    o->a = addr1; o->b = addr2; o->c = addr3;
    o->count = count; o->dtype = datatype; o->op = op;
    o->device = (options & ESGD_FF_DEVICE_BUFFERS) != 0;
    if (int rc = comp_make(o, out)) { delete o; return rc; }
    return FFSUCCESS;
}

int ffcomp_b(ffbuffer_h b1, ffbuffer_h b2, ffoperator_h op, int options, ffbuffer_h b3, ffop_h *out) {
    ESGD_ARG(out && b1 && b3, "ffcomp_b: null buffer or output");
    ESGD_ARG(op == FFIDENTITY || b2, "ffcomp_b: FFSUM needs two inputs");
    auto *o = new FFComp();
    o->ba = reinterpret_cast<FFBuf *>(b1);
    o->bb = reinterpret_cast<FFBuf *>(b2);
    o->bc = reinterpret_cast<FFBuf *>(b3);
    o->dtype = o->ba->dtype;   // "they are the same" (ffop_gcomp.c:53)
    o->op = op;
    o->device = (options & ESGD_FF_DEVICE_BUFFERS) != 0;
    if (int rc = comp_make(o, out)) { delete o; return rc; }
    return FFSUCCESS;
}

int ffcomp_operator_create(ffoperator_fun_t fun, int, ffoperator_h *handle) {
    ESGD_ARG(fun && handle, "ffcomp_operator_create: null function or handle");
    std::lock_guard<std::mutex> lk(g_custom_mu);
    for (int i = 0; i < kMaxCustomOps; ++i)
        if (!g_custom[i]) {
            g_custom[i] = fun;
            *handle = FFCUSTOM + i;
            return FFSUCCESS;
        }
    esgd::set_error("ffcomp_operator_create: more than %d user operators", kMaxCustomOps);
    return FFENOMEM;
}

int ffcomp_operator_delete(ffoperator_h handle) {
    std::lock_guard<std::mutex> lk(g_custom_mu);
    ESGD_ARG(handle >= FFCUSTOM && handle < FFCUSTOM + kMaxCustomOps && g_custom[handle - FFCUSTOM],
             "ffcomp_operator_delete: %d is not a user operator", handle);
    g_custom[handle - FFCUSTOM] = nullptr;
    return FFSUCCESS;
}

int ffop_post(ffop_h h) {
    auto *o = reinterpret_cast<FFComp *>(h);
    ESGD_ARG(o, "ffop_post: null op");
    // buffers re-read at every post, size = MIN of the counts (ffop_gcomp.c:32-52)
    void *a = o->ba ? o->ba->ptr : o->a, *b = o->bb ? o->bb->ptr : o->b, *c = o->bc ? o->bc->ptr : o->c;
    int64_t n = o->ba ? int64_t(o->ba->count) : int64_t(o->count);
    if (o->bb) n = std::min<int64_t>(n, o->bb->count);
    if (o->bc) n = std::min<int64_t>(n, o->bc->count);
    if (const ffoperator_fun_t fun = o->fun) {
        // the user's host function over the host buffers, now (ffop_gcomp.c:52-55): the op
        // is complete when the post returns, and the function's status is the post's
        const int rc = fun(a, b, c, uint32_t(std::max<int64_t>(n, 0)), o->dtype);
        if (rc != FFSUCCESS) return rc;
        o->posted = true;
        o->host_done = true;
        return FFSUCCESS;
    }
    o->host_done = false;
    // never a user operator's handle through the sum (comp_make admitted only these two)
    ESGD_ARG(o->op == FFSUM || o->op == FFIDENTITY, "ffop_post: operator %d is not FFSUM / FFIDENTITY", o->op);
    if (!o->ev) ESGD_HIP(hipEventCreateWithFlags(&o->ev, hipEventDisableTiming));
    hipStream_t s = default_stream();
    if (n > 0) {
        if (o->op == FFIDENTITY) {
            ESGD_HIP(hipMemcpyAsync(c, a, size_t(n) * esgd_dtype_size(o->dtype), hipMemcpyDefault, s));
        } else {
            const void *in[2] = {b, a};   // tree order x1 + x0 = a + b, as esgd_vsum
            const int rc = o->device ? esgd_reduce(o->dtype, 2, in, c, uint64_t(n), s)
                                     : esgd_reduce_host(o->dtype, 2, in, c, uint64_t(n), s);
            if (rc) return rc;
        }
    }
    ESGD_HIP(hipEventRecord(o->ev, s));
    o->posted = true;
    return FFSUCCESS;
}

int ffop_wait(ffop_h h) {
    auto *o = reinterpret_cast<FFComp *>(h);
    ESGD_ARG(o && o->posted, "ffop_wait: op not posted");
    if (!o->host_done) ESGD_HIP(hipEventSynchronize(o->ev));
    o->posted = false;
    return FFSUCCESS;
}

int ffop_test(ffop_h h, int *flag) {
    auto *o = reinterpret_cast<FFComp *>(h);
    ESGD_ARG(o && flag, "ffop_test: null argument");
    if (!o->posted || o->host_done) { *flag = 1; o->posted = false; return FFSUCCESS; }
    const hipError_t e = hipEventQuery(o->ev);
    if (e == hipErrorNotReady) { *flag = 0; return FFSUCCESS; }
    if (e != hipSuccess) return hip_fail(e, "ffop_test", __FILE__, __LINE__);
    *flag = 1;
    o->posted = false;
    return FFSUCCESS;
}

int ffop_free(ffop_h h) {
    auto *o = reinterpret_cast<FFComp *>(h);
    if (!o) return FFSUCCESS;
    if (o->ev) {
        hip_ignore(hipEventSynchronize(o->ev));
        hip_ignore(hipEventDestroy(o->ev));
    }
    delete o;
    return FFSUCCESS;
}

}  // extern "C"
