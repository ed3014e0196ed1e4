/*
 * ffref.c — CPU ORACLE for the eager-SGD gradient-bucket reduction.
 *
 * TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / baseline.  The product library
 * (eager-sgd_amd/csrc, libesgd.so) never links or calls this file.
 *
 * Restates (does not copy) fflib2's arithmetic; citations are relative to
 * /root/reference/eager-SGD-modules/fflib2/.  Built with -O3 -ftree-vectorize and
 * WITHOUT -ffast-math / FMA contraction, matching the reference's flags
 * (CMakeLists.txt:80-81), so float results are the IEEE results of the
 * reference's element order.
 */
#define _GNU_SOURCE
#include "ffref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

size_t ffref_dtype_size(int dtype) {
    switch (dtype) {              /* src/ffdatatype.c:7-20 */
    case FFREF_INT32: return 4;
    case FFREF_INT64: return 8;
    case FFREF_DOUBLE: return 8;
    case FFREF_FLOAT: return 4;
    default: return 0;
    }
}

/* The reference walks the arrays in 1024-element strips and then the remainder
 * (ffop_gcomp_operator.c:17-25).  The strip walk does not change any element's
 * operands, so one loop per strip is an exact restatement. */
#define FFREF_STRIP 1024u
#define FFREF_ADD_STRIPS(T)                                                   \
    do {                                                                      \
        const T *pa = (const T *)a; const T *pb = (const T *)b; T *pc = (T *)c; \
        uint32_t done = 0;                                                    \
        while (n - done >= FFREF_STRIP) {                                     \
            for (uint32_t i = 0; i < FFREF_STRIP; ++i)                        \
                pc[done + i] = pa[done + i] + pb[done + i];                   \
            done += FFREF_STRIP;                                              \
        }                                                                     \
        for (uint32_t i = done; i < n; ++i) pc[i] = pa[i] + pb[i];            \
    } while (0)

int ffref_vsum(int dtype, const void *a, const void *b, void *c, uint32_t n) {
    switch (dtype) {              /* ffop_gcomp_operator.c:33-58 */
    case FFREF_INT32: {
        /* int32 add in the reference is signed C arithmetic; wrap explicitly
         * (two's complement) so overflow cases are defined here. */
        const uint32_t *pa = (const uint32_t *)a, *pb = (const uint32_t *)b;
        uint32_t *pc = (uint32_t *)c;
        for (uint32_t i = 0; i < n; ++i) pc[i] = pa[i] + pb[i];
        return 0;
    }
    case FFREF_INT64: {
        const uint64_t *pa = (const uint64_t *)a, *pb = (const uint64_t *)b;
        uint64_t *pc = (uint64_t *)c;
        for (uint32_t i = 0; i < n; ++i) pc[i] = pa[i] + pb[i];
        return 0;
    }
    case FFREF_DOUBLE: FFREF_ADD_STRIPS(double); return 0;
    case FFREF_FLOAT: FFREF_ADD_STRIPS(float); return 0;
    default: return -2;           /* FFINVALID_ARG, :52-54 */
    }
}

int ffref_copy(int dtype, const void *a, void *c, uint32_t n) {
    size_t es = ffref_dtype_size(dtype);   /* ffop_gcomp_operator.c:61-72 */
    if (!es) return -2;
    memmove(c, a, (size_t)n * es);
    return 0;
}

int ffref_comp_custom(ffref_operator_fun_t fun, int dtype, void *a, uint32_t na, void *b, uint32_t nb,
                      void *c, uint32_t nc) {
    if (!fun) return -2;
    uint32_t size = na;                        /* ffop_gcomp.c:52: MIN of the three counts */
    if (b && nb < size) size = nb;             /* :36-42: buffer 2 is optional */
    if (nc < size) size = nc;
    return fun(a, b, c, size, dtype);          /* :56 */
}

int ffref_op_plus_one(void *a, void *b, void *c, uint32_t count, int dtype) {
    (void)dtype;                               /* custom_computation.c:14-20: int32 only */
    const uint32_t *ia = (const uint32_t *)a, *ib = (const uint32_t *)b;
    uint32_t *ic = (uint32_t *)c;
    for (uint32_t i = 0; i < count; ++i) ic[i] = ia[i] + ib[i] + 1u;
    return 0;                                  /* FFSUCCESS */
}

int ffref_allreduce_rd(int dtype, int P, uint32_t count, const void *const *sb,
                       void *const *rb, void *scratch) {
    size_t es = ffref_dtype_size(dtype);
    if (!es || P < 1) return -2;
    size_t bytes = (size_t)count * es;
    char *snap = (char *)scratch;   /* P snapshots = the in-flight messages */
    if (sb)                         /* move sb -> rb (ffallreduce.c:126-130) */
        for (int r = 0; r < P; ++r) ffref_copy(dtype, sb[r], rb[r], count);
    for (int mask = 1; mask < P; mask <<= 1) {          /* :138 */
        /* every rank sends its current rb (:145) before anyone combines */
        for (int r = 0; r < P; ++r) memcpy(snap + (size_t)r * bytes, rb[r], bytes);
        for (int r = 0; r < P; ++r) {
            int dst = r ^ mask;                          /* :139 */
            if (dst >= P) continue;                      /* :140 (power-of-two only) */
            /* comp_b(tmp[r], rb, SUM -> rb): tmp is operand a (:155) */
            ffref_vsum(dtype, snap + (size_t)dst * bytes, rb[r], rb[r], count);
        }
    }
    return 0;
}

/* ---- pthread variant: one thread per rank, used for the CPU baseline ---- */
typedef struct {
    int dtype, P, rank;
    uint32_t count;
    const void *const *sb;
    void *const *rb;
    void *const *tmp;
    pthread_barrier_t *bar;
} ffref_rank_arg;

static void *ffref_rank_main(void *p) {
    ffref_rank_arg *a = (ffref_rank_arg *)p;
    size_t bytes = (size_t)a->count * ffref_dtype_size(a->dtype);
    if (a->sb) ffref_copy(a->dtype, a->sb[a->rank], a->rb[a->rank], a->count);
    int round = 0;
    for (int mask = 1; mask < a->P; mask <<= 1, ++round) {
        int dst = a->rank ^ mask;
        pthread_barrier_wait(a->bar);      /* partner's rb is final for this round */
        if (dst < a->P) memcpy(a->tmp[a->rank], a->rb[dst], bytes);   /* recv */
        pthread_barrier_wait(a->bar);      /* everyone received before anyone combines */
        if (dst < a->P)
            ffref_vsum(a->dtype, a->tmp[a->rank], a->rb[a->rank], a->rb[a->rank], a->count);
    }
    return NULL;
}

int ffref_allreduce_rd_threads(int dtype, int P, uint32_t count,
                               const void *const *sb, void *const *rb,
                               void *const *tmp) {
    if (!ffref_dtype_size(dtype) || P < 1 || P > 1024) return -2;
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)P);
    pthread_t th[1024];
    ffref_rank_arg args[1024];
    for (int r = 0; r < P; ++r) {
        args[r] = (ffref_rank_arg){dtype, P, r, count, sb, rb, tmp, &bar};
        pthread_create(&th[r], NULL, ffref_rank_main, &args[r]);
    }
    for (int r = 0; r < P; ++r) pthread_join(th[r], NULL);
    pthread_barrier_destroy(&bar);
    return 0;
}

/* Rank 0's hypercube tree, evaluated bottom-up in place in `out` + scratch-free
 * form: level by level, lane j at stride s adds lane j+s when it exists. */
int ffref_tree_sum(int dtype, int k, const void *const *x, void *out, uint32_t n) {
    size_t es = ffref_dtype_size(dtype);
    if (!es || k < 1 || k > 64) return -2;
    /* work[j] holds the partial sum of block starting at j */
    void **work = (void **)malloc(sizeof(void *) * (size_t)k);
    for (int j = 0; j < k; ++j) {
        work[j] = malloc((size_t)n * es);
        memcpy(work[j], x[j], (size_t)n * es);
    }
    for (int s = 1; s < k; s <<= 1)
        for (int j = 0; j + s < k; j += 2 * s)
            /* partner block (j+s) arrives as operand a, like tmp in ffallreduce.c:155 */
            ffref_vsum(dtype, work[j + s], work[j], work[j], n);
    memcpy(out, work[0], (size_t)n * es);
    for (int j = 0; j < k; ++j) free(work[j]);
    free(work);
    return 0;
}

float ffref_bf16_to_f32(uint16_t h) {
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

uint16_t ffref_f32_to_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu))
        return (uint16_t)((u >> 16) | 0x0040u);          /* quiet NaN, sign kept */
    u += 0x7fffu + ((u >> 16) & 1u);                     /* round to nearest even */
    return (uint16_t)(u >> 16);
}

int ffref_tree_sum_bf16(int k, const uint16_t *const *x, uint16_t *out, uint32_t n) {
    if (k < 1 || k > 64) return -2;
    float *acc = (float *)malloc(sizeof(float) * (size_t)k);
    for (uint32_t i = 0; i < n; ++i) {
        for (int j = 0; j < k; ++j) acc[j] = ffref_bf16_to_f32(x[j][i]);
        for (int s = 1; s < k; s <<= 1)
            for (int j = 0; j + s < k; j += 2 * s) acc[j] = acc[j + s] + acc[j];
        out[i] = ffref_f32_to_bf16(acc[0]);
    }
    free(acc);
    return 0;
}

/* glibc's reentrant generator: three LCG steps, 11 + 10 + 10 output bits. */
int ffref_rand_r(unsigned int *seed) {
    unsigned int s = *seed;
    unsigned int r;
    s = s * 1103515245u + 12345u;
    r = (s >> 16) & 0x7ffu;
    s = s * 1103515245u + 12345u;
    r = (r << 10) ^ ((s >> 16) & 0x3ffu);
    s = s * 1103515245u + 12345u;
    r = (r << 10) ^ ((s >> 16) & 0x3ffu);
    *seed = s;
    return (int)r;
}

uint64_t ffref_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

void ffref_fill_uniform_f32(uint64_t seed, int rank, float *out, uint64_t n) {
    ffref_fill_uniform_f32_at(seed, rank, 0, out, n);
}

void ffref_fill_uniform_f32_at(uint64_t seed, int rank, uint64_t start, float *out, uint64_t n) {
    uint64_t base = seed ^ ((uint64_t)(uint32_t)rank << 40);
    for (uint64_t j = 0; j < n; ++j) {
        uint64_t i = start + j;
        /* top 24 bits -> [0,1) exactly representable, then to [-1, 1) */
        uint64_t h = ffref_splitmix64(base ^ i);
        float u = (float)(h >> 40) * (1.0f / 16777216.0f);
        out[j] = 2.0f * u - 1.0f;
    }
}

static double ffref_now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double ffref_time_allreduce(int P, uint32_t count, int threads, int reps) {
    size_t bytes = (size_t)count * 4;
    void **sb = (void **)malloc(sizeof(void *) * (size_t)P);
    void **rb = (void **)malloc(sizeof(void *) * (size_t)P);
    void **tmp = (void **)malloc(sizeof(void *) * (size_t)P);
    for (int r = 0; r < P; ++r) {
        sb[r] = malloc(bytes); rb[r] = malloc(bytes); tmp[r] = malloc(bytes);
        ffref_fill_uniform_f32(0x5EEDE56Dull, r, (float *)sb[r], count);
        memset(rb[r], 0, bytes); memset(tmp[r], 0, bytes);
    }
    void *scratch = threads > 1 ? NULL : malloc(bytes * (size_t)P);
    double best = 1e30;
    for (int it = 0; it < reps; ++it) {
        double t0 = ffref_now();
        if (threads > 1)
            ffref_allreduce_rd_threads(FFREF_FLOAT, P, count, (const void *const *)sb, rb, tmp);
        else
            ffref_allreduce_rd(FFREF_FLOAT, P, count, (const void *const *)sb, rb, scratch);
        double dt = ffref_now() - t0;
        if (dt < best) best = dt;
    }
    for (int r = 0; r < P; ++r) { free(sb[r]); free(rb[r]); free(tmp[r]); }
    free(sb); free(rb); free(tmp); free(scratch);
    return best;
}

/* ---- C1 baseline: P ranks x (main + progress thread), shared-memory "MPI" ---- */
typedef struct {
    int P, rank, reps;
    uint32_t count;
    float **sb, **rb, **tmp, **in, **out;
    volatile int *posted, *done;       /* per rank: step numbers */
    volatile int *ready, *taken;       /* per rank: (step * 64 + round) sequence */
    pthread_barrier_t *bar;            /* the main threads' MPI_Barrier */
    volatile int *stop;
} ffref_c1_arg;

static void ffref_spin_until(volatile int *w, int v) {
    int polls = 0;
    while (__atomic_load_n(w, __ATOMIC_ACQUIRE) < v)
        if (++polls % 5 == 0) sched_yield();    /* ffop.c:156-163 */
}

static void *ffref_c1_progress(void *p) {
    ffref_c1_arg *a = (ffref_c1_arg *)p;
    const int r = a->rank;
    for (int step = 1; step <= a->reps + 1; ++step) {
        ffref_spin_until(&a->posted[r], step);
        ffref_copy(FFREF_FLOAT, a->sb[r], a->rb[r], a->count);      /* move, :126-130 */
        int round = 0;
        for (int mask = 1; mask < a->P; mask <<= 1, ++round) {
            const int dst = r ^ mask, seq = step * 64 + round + 1;
            __atomic_store_n(&a->ready[r], seq, __ATOMIC_RELEASE);  /* send(rb), :145 */
            if (dst >= a->P) { __atomic_store_n(&a->taken[r], seq, __ATOMIC_RELEASE); continue; }
            ffref_spin_until(&a->ready[dst], seq);                   /* recv(tmp), :152 */
            memcpy(a->tmp[r], a->rb[dst], (size_t)a->count * 4);
            __atomic_store_n(&a->taken[r], seq, __ATOMIC_RELEASE);
            ffref_spin_until(&a->taken[dst], seq);                   /* partner has our rb */
            ffref_vsum(FFREF_FLOAT, a->tmp[r], a->rb[r], a->rb[r], a->count);   /* :155 */
        }
        __atomic_store_n(&a->done[r], step, __ATOMIC_RELEASE);
    }
    return NULL;
}

static double ffref_c1_median;

static int ffref_cmp_double(const void *a, const void *b) {
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static void *ffref_c1_main(void *p) {
    ffref_c1_arg *a = (ffref_c1_arg *)p;
    const int r = a->rank;
    const size_t bytes = (size_t)a->count * 4;
    double *dts = r == 0 ? (double *)malloc(sizeof(double) * (size_t)a->reps) : NULL;
    for (int step = 1; step <= a->reps + 1; ++step) {
        pthread_barrier_wait(a->bar);
        double t0 = ffref_now();
        memcpy(a->sb[r], a->in[r], bytes);                           /* :301 */
        __atomic_store_n(&a->posted[r], step, __ATOMIC_RELEASE);     /* post, :304 */
        ffref_spin_until(&a->done[r], step);                         /* wait, :307 */
        memcpy(a->out[r], a->rb[r], bytes);                          /* :309 */
        memset(a->sb[r], 0, bytes);                                  /* :311-314 */
        double dt = ffref_now() - t0;
        pthread_barrier_wait(a->bar);
        if (r == 0 && step > 1) dts[step - 2] = dt;
    }
    if (r == 0) {   /* median over the timed steps (step 1 is the warm-up) */
        qsort(dts, (size_t)a->reps, sizeof(double), ffref_cmp_double);
        ffref_c1_median = dts[a->reps / 2];
        free(dts);
    }
    return NULL;
}

/* Each simulated rank on cores of its own (2 cores per rank; the
 * reference's ff.c:72 starts one progress pthread beside each MPI rank): rank r's progress
 * thread on cpus[2r], its main thread on cpus[2r + 1] (cpus NULL or ncpus < 2P: unpinned,
 * the scheduler's choice -- round 5's figures moved 1.7x between boxes that way). */
static void ffref_start(pthread_t *t, void *(*fn)(void *), void *arg, const int *cpus, int i) {
    pthread_attr_t at;
    pthread_attr_init(&at);
    if (cpus) {   /* pinned from its first instruction, not after the create */
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpus[i], &set);
        (void)pthread_attr_setaffinity_np(&at, sizeof(set), &set);
    }
    pthread_create(t, &at, fn, arg);
    pthread_attr_destroy(&at);
}

double ffref_time_c1_pinned(int P, uint32_t count, int reps, const int *cpus, int ncpus, int *ok) {
    if (P < 1 || P > 64 || reps < 1) return -1.0;
    if (ncpus < 2 * P) cpus = NULL;
    const size_t bytes = (size_t)count * 4;
    /* the buffers are allocated and first touched (Linux places a page on the NUMA node of
     * the CPU that first writes it) by this thread pinned to the ranks' cores for the while,
     * so they sit on those cores' node, not on whichever node the caller happened to run */
    cpu_set_t caller, ranks;
    const int repin = cpus && pthread_getaffinity_np(pthread_self(), sizeof(caller), &caller) == 0;
    if (repin) {
        CPU_ZERO(&ranks);
        for (int i = 0; i < 2 * P; ++i) CPU_SET(cpus[i], &ranks);
        (void)pthread_setaffinity_np(pthread_self(), sizeof(ranks), &ranks);
    }
    float *bufs[5][64];
    for (int k = 0; k < 5; ++k)
        for (int r = 0; r < P; ++r) { bufs[k][r] = (float *)malloc(bytes ? bytes : 4); memset(bufs[k][r], 0, bytes); }
    for (int r = 0; r < P; ++r) ffref_fill_uniform_f32(0x5EEDE56Dull, r, bufs[3][r], count);
    if (repin) (void)pthread_setaffinity_np(pthread_self(), sizeof(caller), &caller);
    volatile int posted[64] = {0}, done[64] = {0}, ready[64] = {0}, taken[64] = {0}, stop = 0;
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)P);
    ffref_c1_arg args[64];
    pthread_t th[128];
    for (int r = 0; r < P; ++r) {
        args[r] = (ffref_c1_arg){P, r, reps, count, bufs[0], bufs[1], bufs[2], bufs[3], bufs[4],
                                 posted, done, ready, taken, &bar, &stop};
        ffref_start(&th[2 * r], ffref_c1_progress, &args[r], cpus, 2 * r);
        ffref_start(&th[2 * r + 1], ffref_c1_main, &args[r], cpus, 2 * r + 1);
    }
    for (int i = 0; i < 2 * P; ++i) pthread_join(th[i], NULL);
    pthread_barrier_destroy(&bar);
    /* every rank's last result vs the tree */
    float *want = (float *)malloc(bytes ? bytes : 4);
    ffref_tree_sum(FFREF_FLOAT, P, (const void *const *)bufs[3], want, count);
    int good = 1;
    for (int r = 0; r < P; ++r) good &= memcmp(bufs[4][r], want, bytes) == 0;
    if (ok) *ok = good;
    free(want);
    for (int k = 0; k < 5; ++k)
        for (int r = 0; r < P; ++r) free(bufs[k][r]);
    return ffref_c1_median;
}

double ffref_time_c1(int P, uint32_t count, int reps, int *ok) {
    return ffref_time_c1_pinned(P, count, reps, NULL, 0, ok);
}
