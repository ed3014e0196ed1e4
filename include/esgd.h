/*
 * esgd.h — C ABI of libesgd.so, the MI355X-native gradient-bucket reduction
 * behind eager-SGD's partial allreduce.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and returns an
 * int status with the reference's error numbering (src/ff.h:4-10 in
 * /root/reference/eager-SGD-modules/fflib2): 0 success, -1 error, -2 invalid
 * argument, -4 out of memory.  esgd_last_error() gives the message of the calling
 * thread's last failure.  Streams and events are opaque `void *` (hipStream_t /
 * hipEvent_t); NULL means the library's default stream for the current device.
 *
 * The reference-shaped entry points (ffinit, ffallreduce, ffsolo_allreduce,
 * ffrand_allreduce, ffschedule_*) live in esgd_ff.h; the deep500 operator ABI in
 * esgd_deep500.h.  This header holds the device-resident hot path those build on.
 */
#ifndef ESGD_H
#define ESGD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (src/ff.h:4-10) ---- */
#define ESGD_SUCCESS 0
#define ESGD_ERROR -1
#define ESGD_INVALID_ARG -2
#define ESGD_ENOMEM -4
#define ESGD_NO_DEVICE -6 /* extension: no usable gfx950 device / HIP runtime error */

/* ---- element types: numbering of src/ff.h:21-31, plus bf16 (extension) ---- */
#define ESGD_INT32 0
#define ESGD_INT64 1
#define ESGD_DOUBLE 2
#define ESGD_FLOAT 3
#define ESGD_BF16 16 /* not in the reference (parity unpinned): fp32 accumulate, one RNE */

/* largest fan-in of one local-reduction launch */
#define ESGD_MAX_FANIN 8

const char *esgd_last_error(void);
int esgd_version(void);                 /* 100 * major + minor */
size_t esgd_dtype_size(int dtype);      /* 0 for unsupported */

/* ---- device plumbing (replaces the reference's host buffers; no reference
 *      equivalent — fflib2 is CPU-only) ---- */
int esgd_device_count(int *n);
int esgd_set_device(int dev);
int esgd_get_device(int *dev);
int esgd_device_arch(int dev, char *name, size_t len); /* e.g. "gfx950:sramecc+:xnack-" */
/* Device buckets come from the library's IPC arena (exportable to the node's other
 * processes, never handed back to the driver while a peer may map them).  esgd_free keeps
 * hipFree's contract: the memory is reused only after the work already queued on its
 * device has finished. */
int esgd_malloc(void **ptr, size_t bytes);
int esgd_free(void *ptr);
/* arena footprint: bytes reserved from the driver, handed out and not freed, and
 * reserved in chunks exported over IPC (those stay reserved until the process exits) */
int esgd_memory_stats(uint64_t *reserved, uint64_t *in_use, uint64_t *exported);
int esgd_host_alloc(void **ptr, size_t bytes);           /* pinned host memory */
int esgd_host_free(void *ptr);
int esgd_host_register(void *ptr, size_t bytes);         /* pin caller-owned memory */
int esgd_host_unregister(void *ptr);
/* kind: 0 host->device, 1 device->host, 2 device->device, 3 inferred */
int esgd_memcpy_async(void *dst, const void *src, size_t bytes, int kind, void *stream);
int esgd_memset_async(void *dst, int value, size_t bytes, void *stream);
int esgd_stream_create(void **stream);
int esgd_stream_destroy(void *stream);
int esgd_stream_synchronize(void *stream);
int esgd_device_synchronize(void);
int esgd_event_create(void **event);                     /* timing-enabled */
int esgd_event_destroy(void *event);
int esgd_event_record(void *event, void *stream);
int esgd_event_synchronize(void *event);
int esgd_event_elapsed_ms(void *start, void *stop, float *ms);
int esgd_stream_wait_event(void *stream, void *event);

/* ---- the hot path: element-wise bucket reduction (device pointers) ----
 *
 * esgd_reduce: out[i] = tree(x_0[i], ..., x_{k-1}[i]) for i < count, where tree is
 * the hypercube order of fflib2's recursive doubling as rank 0 sees it
 * (src/colls/ffallreduce.c:138-171): ((x0+x1)+(x2+x3))+((x4+x5)+(x6+x7)).
 * For power-of-two k that is bit-identical to what every rank of the reference
 * holds after ffallreduce; for other k it is rank 0's (complete) result.
 * `inputs` is a HOST array of k device pointers; `out` may alias any input.
 * dtype: ESGD_FLOAT / ESGD_DOUBLE / ESGD_INT32 / ESGD_INT64 (wrapping) / ESGD_BF16.
 * Stream-ordered; returns after the launch is queued. */
int esgd_reduce(int dtype, int k, const void *const *inputs, void *out,
                uint64_t count, void *stream);

/* The same reduction on the reference's contract -- fflib2 sums host buffers on the CPU
 * (src/components/gcomp/ffop_gcomp_operator.c:33-58, buckets calloc'd by the wrapper,
 * opt_esgd_solo_imagenet_imbalance.py:288-298): `inputs` (k HOST pointers) and `out`
 * are host buckets.  Pinned, mapped buckets are reduced in place by the tree kernel
 * through their device views (zero-copy, PCIe both ways at once); others (pageable, or
 * ESGD_HOST_REDUCE_MODE=dma) run in chunks (ESGD_HOST_REDUCE_CHUNK bytes per input,
 * default 16 MiB) through HBM staging: chunk c's H2D, chunk c-1's tree kernel and chunk
 * c-2's D2H overlap (PCIe is full duplex).  Same bits as esgd_reduce.  Stream-ordered: starts after the work
 * queued on `stream` (NULL: the library stream; ESGD_STREAM_NULL: the legacy default
 * stream) and `stream` waits for its last copy; buckets must stay valid until then. */
int esgd_reduce_host(int dtype, int k, const void *const *inputs, void *out,
                     uint64_t count, void *stream);

/* c = a + b element-wise: the reference's FFSUM operator
 * (src/components/gcomp/ffop_gcomp_operator.c:33-58) on device memory. */
int esgd_vsum(int dtype, const void *a, const void *b, void *c, uint64_t count,
              void *stream);

/* Scaled variant used by the optimizer wrapper: out = tree(x) * scale, the
 * division by comm size of opt_esgd_solo_imagenet_imbalance.py:40 fused into the
 * sum (FLOAT / BF16 only).  scale == 1 is exactly esgd_reduce. */
int esgd_reduce_scaled(int dtype, int k, const void *const *inputs, void *out,
                       uint64_t count, float scale, void *stream);

/* Bucket packing for fused rounds (fp32): dst = concat_i(src_i / divisor) in order,
 * each src_i of count_i elements; divisor == 1 copies.  The division is IEEE fp32
 * (correctly rounded), the wrapper's grad / comm_size of
 * opt_esgd_solo_imagenet_imbalance.py:40 fused into the pack.  esgd_unpack is the
 * inverse copy (dst_i may alias the tensors that were packed).  n <= 4096. */
int esgd_pack_div(int n, const float *const *src, const uint64_t *count, float *dst,
                  float divisor, void *stream);
int esgd_unpack(int n, float *const *dst, const uint64_t *count, const float *src,
                void *stream);

/* Synthetic gradient generator shared with the oracle: x[i] = 2*u - 1 with
 * u = (splitmix64(seed ^ (rank << 40) ^ i) >> 40) / 2^24  (SURVEY.md §8d). */
int esgd_fill_uniform_f32(uint64_t seed, int rank, float *out, uint64_t n, void *stream);
int esgd_fill_uniform_bf16(uint64_t seed, int rank, uint16_t *out, uint64_t n, void *stream);

/* ---- node communicator (replaces MPI_Init / MPI_Barrier of the reference:
 *      src/components/mpi/ffmpi.c:11-31, opt_esgd_solo_imagenet_imbalance.py:295) ----
 * Collective over the `world` processes of one node that pass the same job id; each
 * process drives the HIP device current at the call.  A node-local shared segment
 * carries activations, round epochs and IPC handles; a progress thread drives rounds. */
int esgd_comm_init(const char *job_id, int rank, int world);
int esgd_comm_finalize(void);
int esgd_comm_rank(int *rank);
int esgd_comm_size(int *size);
int esgd_barrier(void);

/* Data plane of schedules created afterwards: "ipc" (default: pull over IPC-mapped peer
 * HBM, two kernels per round) or "rccl" (grouped ncclSend/ncclRecv + the tree kernel on
 * a side stream; one GPU per rank).  Env ESGD_TRANSPORT sets the default. */
int esgd_set_transport(const char *name);
/* Data-plane settings that schedules created afterwards capture (every rank must use the
 * same values for the same creation: they are part of the creation signature).
 *   "small_round_bytes"  buckets up to this many bytes run each round as ONE kernel
 *                        launch (k_round_small); larger ones as pairing + reduce-scatter +
 *                        pairing + all-gather + pairing launches.  Default 4 MiB (env
 *                        ESGD_SMALL_ROUND_BYTES); 0 = never.
 *   "device_flags"       where the rank-pairing flags live: 0 pinned host memory (default,
 *                        env ESGD_DEVICE_FLAGS), 1 uncached HBM pages, 2 fine-grained HBM
 *                        pages (peers' pages written over xGMI).
 *   "strict_handoffs"    1: one-launch rounds use acq_rel arrival counts, release gates
 *                        and an L2 write-back before the reduced flag; 0 (default, env
 *                        ESGD_STRICT_HANDOFFS): the relaxed hand-offs of DESIGN.md §5.
 * value -1 restores the default.  Unknown keys / values -> ESGD_INVALID_ARG. */
int esgd_set_config(const char *key, int64_t value);
int esgd_get_config(const char *key, int64_t *value);
/* ordered transports (rccl): (schedule id, round) pairs in the order this rank issued
 * them — identical on every rank by construction (tests). */
int esgd_comm_issue_log(uint32_t *sched, uint32_t *round, uint32_t cap, uint32_t *n);
/* Host-side profile of this process's progress thread since init (monotonic counters;
 * take differences): out[0] passes, [1] ns inside passes, [2] ns launching rounds
 * (issue-ring pumps, shared launches included), [3] rounds joined, [4] ns joining,
 * [5] kernel launches of rounds, [6] ns in those launches' flushes (k_round_batch).
 * Fills min(n, 7) values. */
#define ESGD_PROFILE_WORDS 7
int esgd_comm_profile(uint64_t *out, int n);

/* ---- persistent partial-allreduce schedules ----
 * kind: ESGD_SCHED_ALLREDUCE (every round synchronous, src/colls/ffallreduce.c),
 *       ESGD_SCHED_SOLO (first poster activates; every (async+1)-th round synchronous,
 *                        src/colls/ffsolo_allreduce.c + ffsolo_limiter.c),
 *       ESGD_SCHED_MAJORITY (activator rand_r(&seed) % P, src/colls/ffrand_allreduce.c).
 * buf:  ESGD_BUF_DEVICE (sb/rb are device pointers, rb 16-B aligned),
 *       ESGD_BUF_HOST (sb/rb are host pointers, staged through HBM: the reference's
 *                      host-memory contract), ESGD_BUF_NONE (control plane only: no data
 *                      moves; for multi-process tests of the round protocol).
 * sb == NULL or sb == rb: in place (FFINPLACE).  Buffers are captured at creation and
 * must stay valid until esgd_schedule_delete (src/colls/ffallreduce.c:113-115).
 * Creation is collective, in the same order on every rank (kind and dtype are checked
 * across ranks); deletion is local, like ffschedule_delete. */
#define ESGD_SCHED_ALLREDUCE 0
#define ESGD_SCHED_SOLO 1
#define ESGD_SCHED_MAJORITY 2
#define ESGD_BUF_DEVICE 0
#define ESGD_BUF_HOST 1
#define ESGD_BUF_NONE 2

typedef uint64_t esgd_sched_h;

typedef struct {
    uint32_t posted, joined, completed, waited; /* round counters of this rank */
    uint32_t activated;                         /* highest round activated (shared) */
    int32_t last_activator;                     /* rank that activated it, -1 if none */
    uint64_t fresh_rounds;                      /* joined after posting them */
    uint64_t auto_rounds;                       /* joined on a peer's activation */
    uint64_t activations;                       /* rounds this rank activated */
} esgd_sched_stats_t;

int esgd_schedule_create(int kind, int buf, const void *sb, void *rb, uint64_t count,
                         int dtype, int async, unsigned seed, esgd_sched_h *out);
/* flags (extension, 0 = esgd_schedule_create):
 *   ESGD_SCHED_HOLD    once a round has completed, this rank joins no further round of
 *                      the schedule until wait/test has returned that round and
 *                      esgd_schedule_release() has been called: the caller copies rb out
 *                      and drops a late send bucket first, as the reference wrapper does
 *                      synchronously right after its wait
 *                      (opt_esgd_solo_imagenet_imbalance.py:309-314);
 *   ESGD_SCHED_ZERO_SB the snapshot (move sb -> rb) zeroes sb as it reads it (device
 *                      buckets, not in place): the wrapper's zero-after-use (:311-314)
 *                      fused into the move, one HBM pass fewer;
 *   ESGD_SCHED_WIRE_BF16 FLOAT buckets, ipc or rccl transport: peers exchange a bf16 copy of the
 *                      bucket (half the xGMI bytes).  Every rank's
 *                      bucket is rounded to bf16 (RNE), each shard is folded in fp32 in the
 *                      tree order and rounded once, and every rank receives that bf16 result
 *                      widened to fp32 (identical on all ranks).  Not in the reference (no
 *                      bf16 in ff.h): parity unpinned, checked against the oracle's
 *                      convention (ffref_tree_sum_bf16 of the rounded inputs). */
/*   ESGD_SCHED_FRESH_ONLY a round this rank joins before posting it (a peer's activation
 *                      carried it through) contributes zeros: its send bucket is not read.
 *                      The reference's wrapper means the same by zeroing the send bucket
 *                      after use (opt_esgd_solo_imagenet_imbalance.py:311-314), but its
 *                      move can read a bucket the caller is still writing (:301); here a
 *                      late gradient never enters a round, whole or torn, and the send
 *                      bucket needs no zeroing (the deep500 op uses HOLD | FRESH_ONLY). */
#define ESGD_SCHED_HOLD 0x1
#define ESGD_SCHED_ZERO_SB 0x2
#define ESGD_SCHED_WIRE_BF16 0x4
#define ESGD_SCHED_FRESH_ONLY 0x8
int esgd_schedule_create_ex(int kind, int buf, const void *sb, void *rb, uint64_t count,
                            int dtype, int async, unsigned seed, unsigned flags,
                            esgd_sched_h *out);
/* post: start round `posted+1`.  producer_stream: stream that writes sb; the snapshot of
 * a round this rank posted waits for the work queued on it so far.  NULL = no producer;
 * ESGD_STREAM_NULL = the legacy default (NULL) stream, e.g. torch's default stream --
 * accepted by every entry point that takes a stream (NULL there: the library stream). */
#define ESGD_STREAM_NULL ((void *)1)
/*
 * role (may be NULL): 1 activated the round, 0 passive, 2 synchronous round. */
int esgd_schedule_post(esgd_sched_h h, void *producer_stream, int *role);
int esgd_schedule_wait(esgd_sched_h h);
/* wait, and report whether this rank had posted the returned round before it joined it
 * (0: a peer's activation carried this rank through the round with whatever its send
 * bucket held -- the caller's late gradient did not take part) */
int esgd_schedule_wait_ex(esgd_sched_h h, int *fresh);
/* ESGD_SCHED_HOLD schedules: done with the round wait returned.  Work queued on
 * `stream` so far (copy-out of rb, zeroing sb; NULL = nothing queued) is waited for by
 * the next round's snapshot on the GPU. */
int esgd_schedule_release(esgd_sched_h h, void *stream);
/* n posts (releases) in this order with ONE event recorded on the stream for all of them
 * -- the per-tensor call pattern (opt_esgd_solo_imagenet_imbalance.py:24-44, one op per
 * gradient) in one call: the same rounds, draws and activations as n single calls.
 * roles may be NULL.  Stops at the first failure and returns its status. */
int esgd_schedule_post_group(const esgd_sched_h *h, int n, void *producer_stream, int *roles);
int esgd_schedule_release_group(const esgd_sched_h *h, int n, void *stream);
/* A post whose round carries its own data (device schedules, ipc or rccl transport, not
 * WIRE_BF16 / FFCOLL_BUFFERS): instead of moving the send bucket, the round's snapshot
 * reads src / divisor (divisor 1: src as it is; any other divisor: FLOAT only, IEEE
 * division as the wrapper's grad / comm_size, opt_esgd_solo_imagenet_imbalance.py:40),
 * and the result is written to dst (may be src) instead of rb -- the deep500 op's copy-in
 * and copy-out fused into the round.  src and dst: count elements, 16-B aligned, untouched
 * by the caller until wait returns.  Only a round this rank joins at or after this post
 * (wait_ex's fresh = 1) takes src and writes dst; a round a peer's activation carried this
 * rank through before the post (fresh = 0) ran with the send bucket as usual (zeros with
 * ESGD_SCHED_FRESH_ONLY) and left its result in rb.  producer_stream: as for post (the
 * work that writes src).  The group form posts n schedules with ONE producer event. */
int esgd_schedule_post_io(esgd_sched_h h, const void *src, void *dst, float divisor, void *producer_stream,
                          int *role);
int esgd_schedule_post_group_io(const esgd_sched_h *h, int n, const void *const *srcs, void *const *dsts,
                                float divisor, void *producer_stream, int *roles);
/* post_io with the round's data in n fp32 pieces (FLOAT device schedules; counts summing to
 * the schedule's count; any alignment): a round this rank joins at or after the post packs
 * srcs[i] / divisor into its bucket in order and, finished, unpacks the result into
 * dsts[i] (may be srcs[i]) -- the fused optimizer's pack and unpack as part of the round,
 * on the round stream, with no send bucket in between.  Otherwise as post_io. */
int esgd_schedule_post_iov(esgd_sched_h h, int n, const float *const *srcs, float *const *dsts,
                           const uint64_t *counts, float divisor, void *producer_stream, int *role);
int esgd_schedule_test(esgd_sched_h h, int *flag);
int esgd_schedule_delete(esgd_sched_h h);
int esgd_schedule_stats(esgd_sched_h h, esgd_sched_stats_t *out);
/* per-round log of this rank: round number, fresh (posted before joining), sync,
 * activator (-1 for synchronous rounds).  Writes up to cap entries, *n = total. */
int esgd_schedule_log(esgd_sched_h h, uint32_t *rounds, uint8_t *fresh, uint8_t *sync,
                      int16_t *activator, uint32_t cap, uint32_t *n);
/* per-round timeline of this rank (tracing): 12 values per completed round -- 6
 * CLOCK_MONOTONIC ns stamps: post, join, launch start, launch queued, completion seen,
 * wait returned (0 = did not happen, e.g. no post for a round joined on activation);
 * then, with ESGD_GPU_TRACE=1 and P > 1, 6 GPU spans in ns: wait at the ready pairing,
 * reduce-scatter, wait at the reduced pairing, all-gather, wait at the done pairing,
 * first pairing to last.  Writes up to cap rounds (12*cap values), *n = rounds available. */
int esgd_schedule_timeline(esgd_sched_h h, uint64_t *t, uint32_t cap, uint32_t *n);
/* the stream rounds run on (consumers of rb may wait on it) */
int esgd_schedule_stream(esgd_sched_h h, void **stream);

#ifdef __cplusplus
}
#endif
#endif /* ESGD_H */
