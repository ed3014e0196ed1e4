/*
 * esgd_deep500.h — the deep500 custom-operator C ABI of the eager-SGD gradient op,
 * prebuilt in libesgd.so (the reference compiles it at run time from a C++ string,
 * test-models/tf-models-r1.11/official/utils/opt_esgd_solo_imagenet_imbalance.py:46-347,
 * against eager-SGD-modules/deep500/deep500/lv0/operators/include/deep500/deep500.h).
 *
 * Entry points and the reference symbol each replaces:
 *   create_new_op      D500_EXPORTED create_new_op (opt_esgd_solo...py:331-346)
 *   allreducef_forward _op_forward -> allreducef::forward (deep500.h:95-104; :277-318)
 *                      host buffers, the contract of the CPU-registered TF kernel
 *                      (deep500/frameworks/tensorflow/custom_operators/tf.py:80)
 *   allreducef_forward_cuda  device buffers + stream (deep500.h "forward_cuda")
 *   is_cuda_supported / report / delete_op   tf.tmpl.cpp:20-32
 * The template-based _op_forward of deep500.h cannot cross a C ABI; a framework bridge
 * binds allreducef_forward instead.
 */
#ifndef ESGD_DEEP500_H
#define ESGD_DEEP500_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* deep500::tensor_t (deep500.h:43-49; ctypes layout utils/tensor_desc.py:6-11) */
typedef struct {
    int type;        /* deep500::tensortype_t, TT_FLOAT = 10 */
    int order;       /* deep500::tensororder_t */
    uint8_t dims;
    uint32_t *sizes;
} esgd_d5_tensor_t;

#define ESGD_OP_SOLO 1       /* opt_esgd_solo_imagenet_imbalance.py (LIMITER 32) */
#define ESGD_OP_MAJORITY 2   /* opt_esgd_majority_imagenet_imbalance.py (seed 6545343) */
#define ESGD_OP_ALLREDUCE 0  /* opt_sgd_mpi.py's synchronous baseline */

/* Mode of the ops created afterwards (defaults: env ESGD_OP_MODE=solo|majority|allreduce,
 * ESGD_OP_ASYNC=32, ESGD_OP_SEED=6545343, ESGD_OP_DEVICE=0|1). */
int esgd_op_configure(int mode, int async, unsigned seed);
/* Extension: what device ops created afterwards exchange between ranks -- ESGD_FLOAT (the
 * reference's fp32, default) or ESGD_BF16 (fp32 buckets, bf16 copies on the wire:
 * ESGD_SCHED_WIRE_BF16 in esgd.h; parity unpinned).  Host-buffer ops stay fp32. */
int esgd_op_configure_wire(int wire_dtype);

void *create_new_op(esgd_d5_tensor_t *input_descriptors, int num_inputs,
                    esgd_d5_tensor_t *output_descriptors, int num_outputs);
/* input: this rank's gradient (already divided by the comm size, :40), last: the unused
 * false-dependency input, output: the partially reduced gradient. */
void allreducef_forward(void *handle, const float *input, const float *last, float *output);
/* stream (every device entry point below): the framework's stream the op's copy-in and
 * copy-out are ordered with; NULL is the legacy default stream (stream 0, e.g. torch's
 * default stream), not the library's own stream. */
void allreducef_forward_cuda(void *handle, const float *input, const float *last, float *output,
                             void *stream);
/* Extensions (device path, return an esgd status instead of aborting):
 *   allreducef_forward_cuda_div: output = partial allreduce of (input / divisor), the
 *     wrapper's grad / comm_size (opt_esgd_solo_imagenet_imbalance.py:40) fused into the
 *     copy-in (IEEE fp32 division, the same bits as dividing first); output may alias input;
 *   allreducef_forward_cuda_packed: n gradient tensors (counts summing to the op's size)
 *     packed in order into the op's bucket (divided as above), one round, unpacked into
 *     outs[i] (may alias grads[i]): the bucket fusion of one round per step instead of
 *     one per tensor. */
/* Extension: allreducef_forward (host buffers) returning an esgd status instead of
 * aborting -- a peer timeout or an allocation failure reaches the framework as an error. */
int allreducef_forward_host(void *handle, const float *input, float *output);
int allreducef_forward_cuda_div(void *handle, const float *input, float *output, float divisor,
                                void *stream);
int allreducef_forward_cuda_packed(void *handle, int n, const float *const *grads,
                                   const uint64_t *counts, float *const *outs, float divisor,
                                   void *stream);
/* Extension: the per-tensor step of EagerSGDOptimizer in one call each way.  The
 * reference's ops block one after another (opt_esgd_solo_imagenet_imbalance.py:304-307);
 * here a caller posts the rounds of many ops (one per gradient tensor) before waiting for
 * the first -- the same rounds, operands and sums, the host round trips overlapped.
 * _post_many_io posts the n rounds in this order with ONE producer event; each round reads
 * inputs[i] / divisor itself in its snapshot and writes its result into outputs[i] (may
 * alias inputs[i]; esgd_schedule_post_io) -- no copy-in or copy-out launch on stream.
 * Tensors that are not 16-B aligned, or ops with a bf16 wire, make the group go the copy-in
 * way (inputs[i] / divisor into the op's bucket, one launch per 48 ops).  It stops at the
 * first failure (its status); the ops before it stay posted.  _wait_many waits for the
 * rounds of the ops that are posted, in order, copies out only what a round did not write
 * itself (a peer's activation carried this rank through before the post, or the copy-in
 * way; one launch per 48 ops) and releases the rounds with ONE consumer event; ops not
 * posted are skipped; the first failure's status is returned after every round was waited
 * for.  One round per op in flight; every rank posts its ops in the same order. */
int allreducef_forward_cuda_post_many_io(void *const *handles, int n, const float *const *inputs,
                                         float *const *outputs, float divisor, void *stream);
int allreducef_forward_cuda_wait_many(void *const *handles, int n, float *const *outputs, void *stream);
/* Extension: allreducef_forward_cuda_packed split in two (posting a fused bucket while
 * backward still runs): _packed_post hands the n pieces to the round (esgd_schedule_post_iov:
 * packed / divisor into the op's bucket and unpacked into outs by the round; bf16 wire:
 * packed into the send bucket on stream), _packed_wait waits for it and copies out a round
 * that did not take them (a peer carried this rank through first).  One round in flight per
 * op; the pieces and outputs must stay valid until _packed_wait. */
int allreducef_forward_cuda_packed_post(void *handle, int n, const float *const *grads, const uint64_t *counts,
                                        float *const *outs, float divisor, void *stream);
int allreducef_forward_cuda_packed_wait(void *handle, void *stream);
/* Extension: what the void entry points above (allreducef_forward, allreducef_forward_cuda)
 * do when their round fails (a peer timeout, an allocation failure).  ESGD_OP_ON_ERROR_ABORT
 * (default; env ESGD_OP_ON_ERROR=abort): print the error and abort the process, as their
 * ABI has no error channel.  ESGD_OP_ON_ERROR_LOCAL (env ESGD_OP_ON_ERROR=local): print it
 * once per op, write this rank's own contribution (input) to output and return, so the
 * training step goes on with the local gradient; esgd_op_status(handle) then returns the
 * first failure's status (0 while none).  -1 restores the default. */
#define ESGD_OP_ON_ERROR_ABORT 0
#define ESGD_OP_ON_ERROR_LOCAL 1
int esgd_op_on_error(int policy);
int esgd_op_status(void *handle);
/* extension: the op's schedule (an esgd_sched_h of esgd.h, e.g. for esgd_schedule_timeline);
 * 0 before its first device or host round created it */
uint64_t esgd_op_schedule(void *handle);
bool is_cuda_supported(void *handle);
int64_t report(void *handle, void *data);   /* bytes of gradient reduced so far */
void delete_op(void *handle);

#ifdef __cplusplus
}
#endif
#endif /* ESGD_DEEP500_H */
