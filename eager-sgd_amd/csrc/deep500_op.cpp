// deep500_op.cpp — the eager-SGD gradient operator behind deep500's custom-op C ABI.
//
// Restates allreducef (opt_esgd_solo_imagenet_imbalance.py:255-346 and its majority
// twin) on the esgd engine.  Per op instance and training step:
//   copy the gradient into the op's persistent send bucket      (:301)
//   post the partial allreduce, wait for its round              (:304-307)
//   copy the reduced bucket out, zero the send bucket           (:309-314)
// Differences, all deliberate:
//   * each op instance owns its bucket (the reference indexes 161 hard-coded ResNet-50
//     buckets by call order, :85-248 / :301 — identical under its fixed call order,
//     and not tied to one model);
//   * buckets are pinned host memory (host path) or HBM (forward_cuda), and the
//     schedule is created at the instance's first forward (collective: the training
//     graph calls ops in the same order on every rank, which the reference relies on
//     for its 161 creations at :288-293);
//   * report() returns the bytes reduced (the reference always returns 0, :273-275);
//   * the schedule holds from each round's completion (ESGD_SCHED_HOLD) until the copy-out
//     is queued, so a round a peer activates next cannot overwrite rb under the copy-out
//     -- the reference gets the same ordering by doing it synchronously right after its
//     wait (:309-314);
//   * a round a peer's activation carries this rank through before its post contributes
//     zeros (ESGD_SCHED_FRESH_ONLY): the late gradient is dropped, as the reference's
//     zeroing after use intends, but never read half-written -- the reference's move can
//     read the bucket while :301 is still copying into it.  The device path therefore
//     needs no zeroing pass at all, and the wrapper's division by the comm size (:40) is
//     fused into the copy-in (allreducef_forward_cuda_div);
//   * the extension entry points return a status instead of aborting the process; the
//     deep500-shaped void ones abort by default (their ABI has no error channel) or, with
//     esgd_op_on_error(ESGD_OP_ON_ERROR_LOCAL), carry on with this rank's own gradient.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <mutex>
#include <string>

#include "engine.h"
#include "esgd_deep500.h"
#include "esgd_ff.h"
#include "esgd_internal.h"

using namespace esgd;

namespace {

struct OpConfig {
    int mode = -1;
    int async = 32;       // LIMITER, opt_esgd_solo_imagenet_imbalance.py:82
    unsigned seed = 6545343;   // opt_esgd_majority_imagenet_imbalance.py:252
    int wire = ESGD_FLOAT;     // ESGD_BF16: device ops exchange bf16 copies (ESGD_SCHED_WIRE_BF16)
};

std::mutex g_op_mu;
OpConfig g_cfg;

OpConfig current_config() {
    std::lock_guard<std::mutex> lk(g_op_mu);
    OpConfig c = g_cfg;
    if (c.mode < 0) {
        const char *m = getenv("ESGD_OP_MODE");
        c.mode = ESGD_OP_SOLO;
        if (m && !strcmp(m, "majority")) c.mode = ESGD_OP_MAJORITY;
        if (m && !strcmp(m, "allreduce")) c.mode = ESGD_OP_ALLREDUCE;
        if (const char *a = getenv("ESGD_OP_ASYNC")) c.async = atoi(a);
        if (const char *s = getenv("ESGD_OP_SEED")) c.seed = unsigned(strtoul(s, nullptr, 10));
    }
    return c;
}

[[noreturn]] void die(const char *where) {
    fprintf(stderr, "[esgd] %s failed: %s\n", where, esgd_last_error());
    std::abort();
}

// what the void entry points do on a failed round (esgd_op_on_error / ESGD_OP_ON_ERROR)
std::atomic<int> g_on_error{-1};

int on_error_policy() {
    const int v = g_on_error.load();
    if (v >= 0) return v;
    const char *e = getenv("ESGD_OP_ON_ERROR");
    return (e && !strcmp(e, "local")) ? ESGD_OP_ON_ERROR_LOCAL : ESGD_OP_ON_ERROR_ABORT;
}

// The op's stream argument names the framework's stream; NULL is the legacy default
// stream (stream 0: torch's default stream, a TF kernel without a device context), never
// the library's own stream -- work queued for the caller (copy-in, copy-out, the producer
// and consumer events) must be ordered with the caller's work on that stream.
void *caller_stream(hipStream_t s) { return s ? static_cast<void *>(s) : ESGD_STREAM_NULL; }

struct AllreduceOp {
    uint64_t len = 0;
    OpConfig cfg;
    esgd_sched_h sched = 0;
    bool device = false;
    float *sb = nullptr, *rb = nullptr;   // persistent buckets (host pinned or HBM)
    int64_t bytes = 0;
    int status = 0;                       // first failure of a void entry point (ESGD_OP_ON_ERROR_LOCAL)
    bool warned = false;
    bool pending = false;                 // a split round posted and not yet waited
    // the pending round was posted with its own data (esgd_schedule_post_io): the gradient
    // is read by the round itself and, if the round takes it, the result lands in io_out
    bool io_posted = false;
    float *io_out = nullptr;
    // a split packed round (allreducef_forward_cuda_packed_post): the pieces' outputs and
    // counts, for the copy-out of a round that did not take them
    std::vector<float *> pk_out;
    std::vector<uint64_t> pk_count;

    // the fused path fits: device op, fp32 wire, 16-B aligned tensors
    bool io_ok(const float *in, const float *out) const {
        return device && cfg.wire != ESGD_BF16 &&
               ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    }

    // Lazy creation of the buckets and the schedule (:288-298); an esgd status (the void
    // entry points abort on failure, the status-returning ones pass it on).
    int ensure(bool dev) {
        if (sched) {
            if (dev != device) {
                esgd::set_error("op used with both host and device buffers");
                return ESGD_INVALID_ARG;
            }
            return ESGD_SUCCESS;
        }
        device = dev;
        const size_t nbytes = size_t(len) * sizeof(float);
        if (dev) {
            // arena buckets: exported to the peers as they are (no shadow copies)
            if (esgd::arena_alloc(nbytes ? nbytes : 256, reinterpret_cast<void **>(&sb), true) ||
                esgd::arena_alloc(nbytes ? nbytes : 256, reinterpret_cast<void **>(&rb), true) ||
                hipMemset(sb, 0, nbytes) != hipSuccess || hipMemset(rb, 0, nbytes) != hipSuccess) {
                (void)hipGetLastError();   // reported here, not by the next launch check
                if (sb) esgd::arena_free(sb);
                if (rb) esgd::arena_free(rb);
                sb = rb = nullptr;
                esgd::set_error("device bucket allocation of %zu bytes", nbytes);
                return ESGD_ENOMEM;
            }
        } else {
            if (hipHostMalloc(reinterpret_cast<void **>(&sb), nbytes ? nbytes : 256, hipHostMallocDefault) != hipSuccess ||
                hipHostMalloc(reinterpret_cast<void **>(&rb), nbytes ? nbytes : 256, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                if (sb) hip_ignore(hipHostFree(sb));
                if (rb) hip_ignore(hipHostFree(rb));
                sb = rb = nullptr;
                esgd::set_error("pinned bucket allocation of %zu bytes", nbytes);
                return ESGD_ENOMEM;
            }
            std::memset(sb, 0, nbytes);   // calloc in the reference (:290-291)
            std::memset(rb, 0, nbytes);
        }
        const int kind = cfg.mode == ESGD_OP_MAJORITY ? ESGD_SCHED_MAJORITY
                         : cfg.mode == ESGD_OP_ALLREDUCE ? ESGD_SCHED_ALLREDUCE : ESGD_SCHED_SOLO;
        const unsigned flags = ESGD_SCHED_HOLD | ESGD_SCHED_FRESH_ONLY |
                               (dev && cfg.wire == ESGD_BF16 ? ESGD_SCHED_WIRE_BF16 : 0u);
        return esgd_schedule_create_ex(kind, dev ? ESGD_BUF_DEVICE : ESGD_BUF_HOST, sb, rb, len,
                                       ESGD_FLOAT, cfg.async, cfg.seed, flags, &sched);
    }

    // Device round: the gradient is already in sb (queued on s).  post -> wait -> drop a
    // late gradient -> `out` consumes rb on s -> release.  Returns an esgd status.  The
    // split entry points run the same steps as post_round() and finish_round().
    int post_round(hipStream_t s) {
        // the snapshot of this round waits for the copy-in just queued on the caller's
        // stream (the data plane's streams are non-blocking: the NULL stream is named)
        void *ps = caller_stream(s);
        // a round a peer's activation carried this rank through before this post took
        // zeros, not the gradient (FRESH_ONLY): the gradient is dropped, and the next
        // copy-in overwrites the send bucket before it is read again
        return esgd_schedule_post(sched, ps, nullptr);
    }

    template <class Out>
    int finish_round(hipStream_t s, Out &&out) {
        void *ps = caller_stream(s);
        if (int rc = esgd_schedule_wait(sched)) return rc;
        if (int rc = out()) return rc;
        if (int rc = esgd_schedule_release(sched, ps)) return rc;
        bytes += int64_t(len) * int64_t(sizeof(float));
        return ESGD_SUCCESS;
    }

    template <class Out>
    int device_round(hipStream_t s, Out &&out) {
        if (int rc = post_round(s)) return rc;
        return finish_round(s, out);
    }
};

constexpr float kNoDivide = 1.0f;


// copy-in of a device round, on s: a plain copy, or the wrapper's division (:40) fused
int cuda_copy_in(AllreduceOp *op, const float *input, float divisor, hipStream_t s) {
    const size_t nbytes = size_t(op->len) * sizeof(float);
    const uint64_t n = op->len;
    if (divisor == kNoDivide) {
        if (const hipError_t e = hipMemcpyAsync(op->sb, input, nbytes, hipMemcpyDeviceToDevice, s)) {
            (void)hip_fail(e, "allreducef: copy-in", __FILE__, __LINE__);
            return ESGD_ERROR;
        }
        return ESGD_SUCCESS;
    }
    return esgd_pack_div(1, &input, &n, op->sb, divisor, caller_stream(s));
}

int cuda_copy_out(AllreduceOp *op, float *output, hipStream_t s) {
    if (const hipError_t e = hipMemcpyAsync(output, op->rb, size_t(op->len) * sizeof(float),
                                            hipMemcpyDeviceToDevice, s)) {
        (void)hip_fail(e, "allreducef: copy-out", __FILE__, __LINE__);
        return ESGD_ERROR;
    }
    return ESGD_SUCCESS;
}

// The round reads the gradient itself (rb = input / divisor in its snapshot) and writes the
// result into output (esgd_schedule_post_io): no copy-in or copy-out on the caller's stream.
// A round a peer's activation carried this rank through before the post (not fresh) ran
// without the gradient (FRESH_ONLY zeros) and left its result in rb: copied out as before.
int forward_cuda_io(AllreduceOp *op, const float *input, float *output, float divisor, hipStream_t s) {
    void *ps = caller_stream(s);
    if (int rc = esgd_schedule_post_io(op->sched, input, output, divisor, ps, nullptr)) return rc;
    int fresh = 0;
    if (int rc = esgd_schedule_wait_ex(op->sched, &fresh)) return rc;
    if (!fresh)
        if (int rc = cuda_copy_out(op, output, s)) return rc;
    if (int rc = esgd_schedule_release(op->sched, fresh ? nullptr : ps)) return rc;
    op->bytes += int64_t(op->len) * int64_t(sizeof(float));
    return ESGD_SUCCESS;
}

int forward_cuda_impl(AllreduceOp *op, const float *input, float *output, float divisor, hipStream_t s) {
    ESGD_ARG(op, "allreducef: null handle");
    ESGD_ARG(!op->pending, "allreducef: a split round is posted and not yet waited");
    if (int rc = op->ensure(true)) return rc;
    if (op->io_ok(input, output)) return forward_cuda_io(op, input, output, divisor, s);
    if (int rc = cuda_copy_in(op, input, divisor, s)) return rc;
    return op->device_round(s, [&]() -> int { return cuda_copy_out(op, output, s); });
}

// Host round, the wrapper's steps (:301-316): copy in -> post -> wait -> copy out ->
// zero the send bucket -> release.
int forward_host_impl(AllreduceOp *op, const float *input, float *output) {
    ESGD_ARG(op && (op->len == 0 || (input && output)), "allreducef_forward: null handle or buffer");
    if (int rc = op->ensure(false)) return rc;
    const size_t nbytes = size_t(op->len) * sizeof(float);
    std::memcpy(op->sb, input, nbytes);
    if (int rc = esgd_schedule_post(op->sched, nullptr, nullptr)) return rc;
    if (int rc = esgd_schedule_wait(op->sched)) return rc;
    std::memcpy(output, op->rb, nbytes);
    std::memset(op->sb, 0, nbytes);
    if (int rc = esgd_schedule_release(op->sched, nullptr)) return rc;
    op->bytes += int64_t(nbytes);
    return ESGD_SUCCESS;
}

// A void entry point's round failed: abort (the default), or keep the job going with
// this rank's own contribution as the step's gradient -- what a round that only this
// rank's fresh gradient reached would give (its peers' shares zero, rsgd.c:87,100) --
// and remember the status for esgd_op_status().
void fail_void(AllreduceOp *op, int rc, const char *where, const float *input, float *output, bool dev,
               hipStream_t s) {
    if (!op || on_error_policy() != ESGD_OP_ON_ERROR_LOCAL) die(where);
    if (!op->status) op->status = rc;
    if (!op->warned) {
        fprintf(stderr, "[esgd] %s failed: %s -- continuing with this rank's own gradient "
                "(ESGD_OP_ON_ERROR_LOCAL; later failures of this op are not printed)\n", where, esgd_last_error());
        op->warned = true;
    }
    const size_t nbytes = size_t(op->len) * sizeof(float);
    if (!nbytes || input == output || !input || !output) return;
    if (dev) {
        if (hipMemcpyAsync(output, input, nbytes, hipMemcpyDeviceToDevice, s) != hipSuccess) die(where);
    } else {
        std::memcpy(output, input, nbytes);
    }
}

}  // namespace

extern "C" {

int esgd_op_on_error(int policy) {
    ESGD_ARG(policy == ESGD_OP_ON_ERROR_ABORT || policy == ESGD_OP_ON_ERROR_LOCAL || policy == -1,
             "esgd_op_on_error: ESGD_OP_ON_ERROR_ABORT, ESGD_OP_ON_ERROR_LOCAL or -1 (the default)");
    g_on_error.store(policy);
    return ESGD_SUCCESS;
}

int esgd_op_status(void *handle) {
    return handle ? static_cast<AllreduceOp *>(handle)->status : ESGD_INVALID_ARG;
}

uint64_t esgd_op_schedule(void *handle) { return handle ? static_cast<AllreduceOp *>(handle)->sched : 0; }

int esgd_op_configure(int mode, int async, unsigned seed) {
    ESGD_ARG(mode == ESGD_OP_SOLO || mode == ESGD_OP_MAJORITY || mode == ESGD_OP_ALLREDUCE,
             "esgd_op_configure: bad mode %d", mode);
    std::lock_guard<std::mutex> lk(g_op_mu);
    g_cfg.mode = mode;
    g_cfg.async = async;
    g_cfg.seed = seed;
    return ESGD_SUCCESS;
}

int esgd_op_configure_wire(int wire_dtype) {
    ESGD_ARG(wire_dtype == ESGD_FLOAT || wire_dtype == ESGD_BF16,
             "esgd_op_configure_wire: FLOAT or BF16, not %d", wire_dtype);
    std::lock_guard<std::mutex> lk(g_op_mu);
    g_cfg.wire = wire_dtype;
    return ESGD_SUCCESS;
}

void *create_new_op(esgd_d5_tensor_t *in, int num_inputs, esgd_d5_tensor_t *, int) {
    if (!in || num_inputs < 1) {
        esgd::set_error("create_new_op: no input descriptor");
        return nullptr;
    }
    if (!engine_ready() && ffinit(nullptr, nullptr) != FFSUCCESS) die("ffinit");   // :335-339
    auto *op = new AllreduceOp();
    uint64_t total = 1;
    for (int i = 0; i < in[0].dims; ++i) total *= in[0].sizes[i];       // :341-343
    op->len = total;
    op->cfg = current_config();
    return op;
}

void allreducef_forward(void *handle, const float *input, const float *, float *output) {
    auto *op = static_cast<AllreduceOp *>(handle);
    if (int rc = forward_host_impl(op, input, output)) fail_void(op, rc, "allreducef_forward", input, output, false, nullptr);
}

int allreducef_forward_host(void *handle, const float *input, float *output) {
    return forward_host_impl(static_cast<AllreduceOp *>(handle), input, output);
}

void allreducef_forward_cuda(void *handle, const float *input, const float *, float *output,
                             void *stream) {
    auto *op = static_cast<AllreduceOp *>(handle);
    if (int rc = forward_cuda_impl(op, input, output, kNoDivide, static_cast<hipStream_t>(stream)))
        fail_void(op, rc, "allreducef_forward_cuda", input, output, true, static_cast<hipStream_t>(stream));
}

int allreducef_forward_cuda_div(void *handle, const float *input, float *output, float divisor,
                                void *stream) {
    ESGD_ARG(divisor == divisor && divisor != 0.0f, "allreducef_forward_cuda_div: bad divisor");
    return forward_cuda_impl(static_cast<AllreduceOp *>(handle), input, output, divisor,
                             static_cast<hipStream_t>(stream));
}

int allreducef_forward_cuda_packed(void *handle, int n, const float *const *grads, const uint64_t *counts,
                                   float *const *outs, float divisor, void *stream) {
    auto *op = static_cast<AllreduceOp *>(handle);
    ESGD_ARG(op && n >= 0 && (n == 0 || (grads && counts && outs)), "allreducef_forward_cuda_packed: bad arguments");
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) total += counts[i];
    ESGD_ARG(total == op->len, "allreducef_forward_cuda_packed: %llu elements for a %llu-element op",
             (unsigned long long)total, (unsigned long long)op->len);
    ESGD_ARG(!op->pending, "allreducef_forward_cuda_packed: a split round is posted and not yet waited");
    if (int rc = op->ensure(true)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (op->io_ok(nullptr, nullptr)) {
        // the pack (/ divisor) and the unpack are the round's own copy-in and copy-out
        // (esgd_schedule_post_iov, on the round stream): no send bucket, no kernels on s
        void *ps = caller_stream(s);
        if (int rc = esgd_schedule_post_iov(op->sched, n, grads, outs, counts, divisor, ps, nullptr)) return rc;
        int fresh = 0;
        if (int rc = esgd_schedule_wait_ex(op->sched, &fresh)) return rc;
        // a round a peer carried this rank through before the post left its result in rb
        if (!fresh)
            if (int rc = esgd_unpack(n, outs, counts, op->rb, ps)) return rc;
        if (int rc = esgd_schedule_release(op->sched, fresh ? nullptr : ps)) return rc;
        op->bytes += int64_t(op->len) * int64_t(sizeof(float));
        return ESGD_SUCCESS;
    }
    if (int rc = esgd_pack_div(n, grads, counts, op->sb, divisor, caller_stream(s))) return rc;
    return op->device_round(s, [&]() -> int { return esgd_unpack(n, outs, counts, op->rb, caller_stream(s)); });
}

int allreducef_forward_cuda_packed_post(void *handle, int n, const float *const *grads, const uint64_t *counts,
                                        float *const *outs, float divisor, void *stream) {
    auto *op = static_cast<AllreduceOp *>(handle);
    ESGD_ARG(op && n >= 0 && (n == 0 || (grads && counts && outs)), "allreducef_forward_cuda_packed_post: bad arguments");
    ESGD_ARG(divisor == divisor && divisor != 0.0f, "allreducef_forward_cuda_packed_post: bad divisor");
    ESGD_ARG(!op->pending, "allreducef_forward_cuda_packed_post: the previous round was not waited");
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) total += counts[i];
    ESGD_ARG(total == op->len, "allreducef_forward_cuda_packed_post: %llu elements for a %llu-element op",
             (unsigned long long)total, (unsigned long long)op->len);
    if (int rc = op->ensure(true)) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    void *ps = caller_stream(s);
    op->pk_out.assign(outs, outs + n);
    op->pk_count.assign(counts, counts + n);
    if (op->io_ok(nullptr, nullptr)) {   // the round packs and unpacks the pieces itself
        if (int rc = esgd_schedule_post_iov(op->sched, n, grads, outs, counts, divisor, ps, nullptr)) return rc;
        op->io_posted = true;
    } else {                             // bf16 wire: packed into the send bucket first
        if (int rc = esgd_pack_div(n, grads, counts, op->sb, divisor, ps)) return rc;
        if (int rc = op->post_round(s)) return rc;
        op->io_posted = false;
    }
    op->pending = true;
    return ESGD_SUCCESS;
}

int allreducef_forward_cuda_packed_wait(void *handle, void *stream) {
    auto *op = static_cast<AllreduceOp *>(handle);
    ESGD_ARG(op && op->pending, "allreducef_forward_cuda_packed_wait: no round posted");
    op->pending = false;
    void *ps = caller_stream(static_cast<hipStream_t>(stream));
    int fresh = 0;
    if (int rc = esgd_schedule_wait_ex(op->sched, &fresh)) return rc;
    const bool in_place = op->io_posted && fresh;   // the round unpacked into the outputs itself
    op->io_posted = false;
    int rc = ESGD_SUCCESS;
    if (!in_place)
        rc = esgd_unpack(int(op->pk_out.size()), op->pk_out.data(), op->pk_count.data(), op->rb, ps);
    const int rr = esgd_schedule_release(op->sched, in_place ? nullptr : ps);   // released even after a failure
    if (!rc) rc = rr;
    if (!rc) op->bytes += int64_t(op->len) * int64_t(sizeof(float));
    return rc;
}

// the copy-in way of post_many_io: every op's copy-in (inputs[i] / divisor into its send
// bucket; one launch per 48 ops) on stream, then the n rounds posted in order with ONE
// producer event (the fallback for a group the fused round I/O cannot take)
static int post_many_copy_in(void *const *handles, int n, const float *const *inputs, float divisor,
                             void *stream) {
    ESGD_ARG(n >= 0 && (n == 0 || (handles && inputs)), "allreducef_forward_cuda_post_many_io: bad arguments");
    ESGD_ARG(divisor == divisor && divisor != 0.0f, "allreducef_forward_cuda_post_many_io: bad divisor");
    if (n == 0) return ESGD_SUCCESS;
    std::vector<AllreduceOp *> ops(static_cast<size_t>(n));
    std::vector<float *> sbs(static_cast<size_t>(n));
    std::vector<uint64_t> counts(static_cast<size_t>(n));
    std::vector<esgd_sched_h> hs(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) {
        AllreduceOp *op = ops[i] = static_cast<AllreduceOp *>(handles[i]);
        ESGD_ARG(op, "allreducef_forward_cuda_post_many_io: op %d is null", i);
        ESGD_ARG(!op->pending, "allreducef_forward_cuda_post_many_io: op %d's previous round was not waited", i);
        if (int rc = op->ensure(true)) return rc;   // collective, in the callers' common order
        sbs[i] = op->sb;
        counts[i] = op->len;
        hs[i] = op->sched;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    void *ps = caller_stream(s);
    if (int rc = esgd::pack_scatter(n, inputs, sbs.data(), counts.data(), divisor, ps)) return rc;
    std::vector<int> roles(static_cast<size_t>(n), -1);
    const int rc = esgd_schedule_post_group(hs.data(), n, ps, roles.data());
    for (int i = 0; i < n; ++i) ops[i]->pending = roles[i] >= 0;   // posted (a role was written)
    return rc;
}

int allreducef_forward_cuda_post_many_io(void *const *handles, int n, const float *const *inputs,
                                         float *const *outputs, float divisor, void *stream) {
    ESGD_ARG(n >= 0 && (n == 0 || (handles && inputs && outputs)),
             "allreducef_forward_cuda_post_many_io: bad arguments");
    ESGD_ARG(divisor == divisor && divisor != 0.0f, "allreducef_forward_cuda_post_many_io: bad divisor");
    if (n == 0) return ESGD_SUCCESS;
    std::vector<AllreduceOp *> ops(static_cast<size_t>(n));
    std::vector<esgd_sched_h> hs(static_cast<size_t>(n));
    bool fits = true;
    for (int i = 0; i < n; ++i) {
        AllreduceOp *op = ops[i] = static_cast<AllreduceOp *>(handles[i]);
        ESGD_ARG(op, "allreducef_forward_cuda_post_many_io: op %d is null", i);
        ESGD_ARG(!op->pending, "allreducef_forward_cuda_post_many_io: op %d's previous round was not waited", i);
        if (int rc = op->ensure(true)) return rc;   // collective, in the callers' common order
        fits = fits && op->io_ok(inputs[i], outputs[i]);
        hs[i] = op->sched;
    }
    // a tensor the fused path cannot take (unaligned, bf16 wire): the whole group goes the
    // copy-in way, and wait_many copies out
    if (!fits) return post_many_copy_in(handles, n, inputs, divisor, stream);
    void *ps = caller_stream(static_cast<hipStream_t>(stream));
    std::vector<int> roles(static_cast<size_t>(n), -1);
    const int rc = esgd_schedule_post_group_io(hs.data(), n, reinterpret_cast<const void *const *>(inputs),
                                               reinterpret_cast<void *const *>(outputs), divisor, ps, roles.data());
    for (int i = 0; i < n; ++i) {
        ops[i]->pending = roles[i] >= 0;   // posted (a role was written)
        ops[i]->io_posted = ops[i]->pending;
        ops[i]->io_out = outputs[i];
    }
    return rc;
}

}  // extern "C"

namespace {

int wait_many_impl(void *const *handles, int n, float *const *outputs, void *stream) {
    ESGD_ARG(n >= 0 && (n == 0 || (handles && outputs)), "allreducef_forward_cuda_wait_many: bad arguments");
    void *ps = caller_stream(static_cast<hipStream_t>(stream));
    std::vector<float *> outs, rbs;
    std::vector<uint64_t> counts;
    std::vector<esgd_sched_h> hs, hs_io;   // copied out from rb / results already in place
    std::vector<AllreduceOp *> done, done_io;
    int first = ESGD_SUCCESS;
    for (int i = 0; i < n; ++i) {
        AllreduceOp *op = static_cast<AllreduceOp *>(handles[i]);
        if (!op || !op->pending) continue;
        op->pending = false;
        const bool io = op->io_posted;
        op->io_posted = false;
        int fresh = 0;
        if (int rc = esgd_schedule_wait_ex(op->sched, &fresh)) {
            if (!first) first = rc;
            continue;
        }
        // a round that took the gradient wrote its result into io_out itself; one a peer
        // carried this rank through before the post left it in rb
        const bool in_place = io && fresh;
        outs.push_back(outputs[i]);
        rbs.push_back(in_place ? op->io_out : op->rb);
        counts.push_back(op->len);
        if (in_place && outputs[i] == op->io_out) {
            outs.pop_back(); rbs.pop_back(); counts.pop_back();   // nothing to move
            hs_io.push_back(op->sched);
            done_io.push_back(op);
        } else {
            hs.push_back(op->sched);
            done.push_back(op);
        }
    }
    if (!done_io.empty()) {   // the caller read nothing of rb: no consumer event
        const int rc = esgd_schedule_release_group(hs_io.data(), int(hs_io.size()), nullptr);
        if (rc && !first) first = rc;
        if (!rc)
            for (AllreduceOp *op : done_io) op->bytes += int64_t(op->len) * int64_t(sizeof(float));
    }
    if (!done.empty()) {
        int rc = esgd::unpack_gather(int(outs.size()), outs.data(), rbs.data(), counts.data(), ps);
        // released even when the copy-out could not be queued: no round stays held
        const int rr = esgd_schedule_release_group(hs.data(), int(hs.size()), ps);
        if (!rc) rc = rr;
        if (rc && !first) first = rc;
        if (!rc)
            for (AllreduceOp *op : done) op->bytes += int64_t(op->len) * int64_t(sizeof(float));
    }
    return first;
}

}  // namespace

extern "C" {

int allreducef_forward_cuda_wait_many(void *const *handles, int n, float *const *outputs, void *stream) {
    return wait_many_impl(handles, n, outputs, stream);
}

bool is_cuda_supported(void *) { return true; }

int64_t report(void *handle, void *) {
    return handle ? static_cast<AllreduceOp *>(handle)->bytes : 0;
}

// The schedule and its buckets stay alive: peers may still activate rounds that read
// them (the reference never deletes its schedules either).  They go at fffinalize.
void delete_op(void *handle) {
    auto *op = static_cast<AllreduceOp *>(handle);
    if (op && !op->sched) delete op;
}

}  // extern "C"
