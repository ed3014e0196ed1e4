/*
 * ffref.h — CPU ORACLE (test infrastructure only; never linked into the product).
 *
 * A plain-C restatement of the reference fflib2 reduction path, used by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.  Every
 * function cites the reference file:line whose behaviour it restates
 * (paths relative to /root/reference/eager-SGD-modules/fflib2/).
 *
 * Parity status: pinned by the reference's own known-answer tests (evaluation/ programs'
 * formulas, see tests/test_oracle.py) and by a libc rand_r golden sequence.  The
 * reference binaries themselves may not be executed in this pipeline,
 * so no oracle/_ref build exists.
 */
#ifndef FFREF_H
#define FFREF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* datatype codes: same numbering as the reference src/ff.h:21-31 */
enum { FFREF_INT32 = 0, FFREF_INT64 = 1, FFREF_DOUBLE = 2, FFREF_FLOAT = 3 };

/* element size, 0 on unsupported type (src/ffdatatype.c:4-32) */
size_t ffref_dtype_size(int dtype);

/* c[i] = a[i] + b[i], strip-mined in blocks of 1024
 * (src/components/gcomp/ffop_gcomp_operator.c:8-25, 33-58). Returns 0 / -2. */
int ffref_vsum(int dtype, const void *a, const void *b, void *c, uint32_t n);

/* memcpy "move" (src/components/gcomp/ffop_gcomp_operator.c:61-72) */
int ffref_copy(int dtype, const void *a, void *c, uint32_t n);

/* A computation with a user operator (FFCUSTOM: ffcomp_operator_create, src/ffcomp.c:40-42;
 * ff.h:134): the gcomp backend calls the operator once over size = MIN(count1, count2,
 * count3) elements (src/components/gcomp/ffop_gcomp.c:29-56) and the op completes when it
 * returns FFSUCCESS (0).  Returns the operator's status. */
typedef int (*ffref_operator_fun_t)(void *a, void *b, void *c, uint32_t count, int dtype);
int ffref_comp_custom(ffref_operator_fun_t fun, int dtype, void *a, uint32_t na, void *b, uint32_t nb,
                      void *c, uint32_t nc);
/* the user operator of evaluation/custom_computation.c:12-24: c[i] = a[i] + b[i] + 1 over
 * int32 (two's complement wrap, as gcc compiles the reference's int arithmetic) */
int ffref_op_plus_one(void *a, void *b, void *c, uint32_t count, int dtype);

/* Recursive-doubling allreduce simulated for all P ranks in one process
 * (src/colls/ffallreduce.c:74-177, hot loop :138-171):
 *   rb[r] = sb[r]                       (move, :126-130; skipped when sb == NULL -> in place)
 *   for mask = 1, 2, 4 ... < P:         (:138)
 *      dst = r ^ mask; if dst < P:      (:139-140)
 *         tmp  = rb[dst] as sent at the start of the round   (send :145, recv :152)
 *         rb[r] = tmp + rb[r]           (comp_b(tmp, rb -> rb), :155)
 * `scratch` must hold P*count elements.  Non-power-of-two P reproduces the
 * reference's partial results (partners >= P are skipped). */
int ffref_allreduce_rd(int dtype, int P, uint32_t count, const void *const *sb,
                       void *const *rb, void *scratch);

/* Same algorithm with one pthread per rank (ranks run concurrently, round barriers
 * stand in for the matched MPI send/recv).  Used only as the CPU baseline timing. */
int ffref_allreduce_rd_threads(int dtype, int P, uint32_t count,
                               const void *const *sb, void *const *rb,
                               void *const *tmp);

/* Closed form of rank 0's recursive-doubling result: the pairwise hypercube tree
 * ((x0+x1)+(x2+x3))+... with absent partners skipped.  For power-of-two k this is
 * bit-identical on every rank (IEEE add is commutative). */
int ffref_tree_sum(int dtype, int k, const void *const *x, void *out, uint32_t n);

/* bf16 extension (NOT in the reference: src/ff.h:21-31 has no half types ->
 * parity unpinned): bf16 in, fp32 accumulate in the same tree order, one
 * round-to-nearest-even at the end (NaN stays NaN). */
int ffref_tree_sum_bf16(int k, const uint16_t *const *x, uint16_t *out, uint32_t n);
uint16_t ffref_f32_to_bf16(float f);
float ffref_bf16_to_f32(uint16_t h);

/* glibc rand_r restated (the majority activator draw,
 * src/colls/ffrand_allreduce.c:88: rand_r(&seed) % comm_size). */
int ffref_rand_r(unsigned int *seed);

/* Deterministic synthetic gradients: x_r[i] = u(splitmix64(seed ^ (r << 40) ^ i))
 * mapped to [-1, 1).  Same generator runs on the GPU. */
uint64_t ffref_splitmix64(uint64_t x);
void ffref_fill_uniform_f32(uint64_t seed, int rank, float *out, uint64_t n);
void ffref_fill_uniform_f32_at(uint64_t seed, int rank, uint64_t start, float *out, uint64_t n);

/* One reduction step's wall time on this host for the CPU baseline leg:
 * allreduce of P simulated ranks with `threads` (1 => sequential ranks,
 * P => one pthread per rank).  Returns seconds per allreduce (best of reps). */
double ffref_time_allreduce(int P, uint32_t count, int threads, int reps);

/* C1-shaped CPU baseline (BASELINE.json configs[0]): P ranks, each a main thread and a
 * progress thread (src/ff.c:72), reducing one `count`-element fp32 bucket per step the
 * way the wrapper drives fflib2 (opt_esgd_solo_imagenet_imbalance.py:301-316): copy the
 * gradient into the send bucket, post, spin-wait (ffop.c:156-163), copy the result out,
 * zero the send bucket; the progress thread runs the move and the recursive-doubling
 * rounds (ffallreduce.c:126-171), exchanging rb through shared memory in place of MPI.
 * Returns the median per-step seconds over `reps` steps (after one warm-up step); *ok = 1
 * if every rank's last result equals the oracle tree of the P buckets. */
double ffref_time_c1(int P, uint32_t count, int reps, int *ok);
/* the same with rank r's progress / main thread pinned to cpus[2r] / cpus[2r + 1] */
double ffref_time_c1_pinned(int P, uint32_t count, int reps, const int *cpus, int ncpus, int *ok);

#ifdef __cplusplus
}
#endif
#endif
