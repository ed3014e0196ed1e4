/*
 * A plain C caller of the fflib2 API (include/ff.h -> libesgd.so), written the way the
 * reference's evaluation programs use fflib2, with their known answers:
 *   - ffallreduce of to_reduce[j] = i + j gives (i + j) * size
 *     (eager-SGD-modules/fflib2/evaluation/allreduce.c:49-63), fresh schedule per i;
 *   - ffsolo_allreduce / ffrand_allreduce with every rank posting behind a barrier give
 *     the plain allreduce of the running inputs
 *     (evaluation/solo_allreduce_correctness.c:76-97, rand_allreduce_correctness.c:78-98);
 *   - FFCOLL_BUFFERS: one schedule, buckets that move and change size every round, one
 *     user-managed and one library-managed (evaluation/allreduce_buffers_user_managed.c,
 *     allreduce_buffers_fflib_managed.c), same (i + j) * size answer;
 *   - FFCOLL_BUFFERS under ffsolo_allreduce with a late rank (posts of rounds a peer
 *     already ran are accepted);
 *   - single computations: ffcomp(a, b, FFSUM) -> c == a + b for rand() int32 inputs
 *     (evaluation/simple_computation.c:48-75), the same in fp32 against C's own IEEE add,
 *     FFIDENTITY, ffcomp_b over descriptors of different counts (MIN of the counts,
 *     ffop_gcomp.c:52), and ffcomp_operator_create refused (no host compute path).
 * Ranks come from RANK / WORLD_SIZE / ESGD_JOB_ID (no MPI).  Exit status 0 = passed.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "ff.h"

static int check_int(const int32_t *got, const int32_t *want, int n, const char *what, int it) {
    for (int j = 0; j < n; ++j)
        if (got[j] != want[j]) {
            int rank;
            ffrank(&rank);
            int bad = 0, zero = 0;
            for (int k = 0; k < n; ++k) { bad += got[k] != want[k]; zero += got[k] == 0; }
            fprintf(stderr, "[rank %d] %s iteration %d: element %d = %d, expected %d "
                    "(%d of %d wrong, %d zero; got[1..3] = %d %d %d)\n", rank, what, it, j, got[j],
                    want[j], bad, n, zero, n > 1 ? got[1] : 0, n > 2 ? got[2] : 0, n > 3 ? got[3] : 0);
            return 1;
        }
    return 0;
}

/* simple_computation.c on the GPU kernel, every rank on its own */
/* custom_computation.c:12-24 */
static int plus_one(void *a, void *b, void *c, uint32_t count, ffdatatype_h type) {
    const int32_t *ia = (const int32_t *)a, *ib = (const int32_t *)b;
    int32_t *ic = (int32_t *)c;
    (void)type;
    for (uint32_t i = 0; i < count; ++i) ic[i] = (int32_t)((uint32_t)ia[i] + (uint32_t)ib[i] + 1u);   /* wraps */
    return FFSUCCESS;
}

static int single_computations(int count) {
    int32_t *a = malloc(count * sizeof(int32_t)), *b = malloc(count * sizeof(int32_t)),
            *c = calloc(count, sizeof(int32_t)), *w = malloc(count * sizeof(int32_t));
    float *fa = malloc(count * sizeof(float)), *fb = malloc(count * sizeof(float)), *fc = calloc(count, sizeof(float));
    srand(12345);
    for (int i = 0; i < count; ++i) {
        a[i] = rand(); b[i] = rand();
        w[i] = (int32_t)((uint32_t)a[i] + (uint32_t)b[i]);   /* the reference's int add, wrapped */
        fa[i] = (float)rand() / RAND_MAX - 0.5f; fb[i] = (float)rand() / RAND_MAX * 1e-3f;
    }
    ffop_h op;
    if (ffcomp(a, b, count, FFINT32, FFSUM, 0, c, &op) != FFSUCCESS || ffop_post(op) != FFSUCCESS ||
        ffop_wait(op) != FFSUCCESS) {
        fprintf(stderr, "ffcomp int32: %s\n", esgd_last_error());
        return 1;
    }
    ffop_free(op);
    if (check_int(c, w, count, "ffcomp FFSUM int32", 0)) return 1;
    if (ffcomp(fa, fb, count, FFFLOAT, FFSUM, 0, fc, &op) != FFSUCCESS || ffop_post(op) != FFSUCCESS) return 1;
    int flag = 0;
    while (!flag)
        if (ffop_test(op, &flag) != FFSUCCESS) return 1;
    ffop_free(op);
    for (int i = 0; i < count; ++i)
        if (fc[i] != fa[i] + fb[i]) { fprintf(stderr, "ffcomp FFSUM fp32: element %d\n", i); return 1; }
    /* FFIDENTITY: the move */
    if (ffcomp(a, NULL, count, FFINT32, FFIDENTITY, 0, c, &op) != FFSUCCESS || ffop_post(op) != FFSUCCESS ||
        ffop_wait(op) != FFSUCCESS) return 1;
    ffop_free(op);
    if (check_int(c, a, count, "ffcomp FFIDENTITY", 0)) return 1;
    /* descriptors of different counts: size = MIN(counts), the rest of c untouched */
    ffbuffer_h ba, bb, bc;
    for (int i = 0; i < count; ++i) c[i] = -7;
    const int m = count / 2;
    ffbuffer_create(a, count, FFINT32, 0, &ba);
    ffbuffer_create(b, m, FFINT32, 0, &bb);
    ffbuffer_create(c, count, FFINT32, 0, &bc);
    if (ffcomp_b(ba, bb, FFSUM, 0, bc, &op) != FFSUCCESS || ffop_post(op) != FFSUCCESS || ffop_wait(op) != FFSUCCESS)
        return 1;
    ffop_free(op);
    if (check_int(c, w, m, "ffcomp_b MIN(counts)", 0)) return 1;
    for (int i = m; i < count; ++i) if (c[i] != -7) { fprintf(stderr, "ffcomp_b wrote past MIN(counts)\n"); return 1; }
    ffbuffer_delete(ba); ffbuffer_delete(bb); ffbuffer_delete(bc);
    /* evaluation/custom_computation.c: a user operator c = a + b + 1, run on the host
     * buffers once per post; a null function is refused */
    ffoperator_h custom;
    if (ffcomp_operator_create(NULL, 1, &custom) != FFINVALID_ARG) return 1;
    if (ffcomp_operator_create(plus_one, 1, &custom) != FFSUCCESS || custom < FFCUSTOM) return 1;
    if (ffcomp(a, b, count, FFINT32, custom, 0, c, &op) != FFSUCCESS || ffop_post(op) != FFSUCCESS ||
        ffop_wait(op) != FFSUCCESS) return 1;
    ffop_free(op);
    for (int i = 0; i < count; ++i)
        if (c[i] != (int32_t)((uint32_t)a[i] + (uint32_t)b[i] + 1u)) {
            fprintf(stderr, "custom operator: c[%d] = %d\n", i, c[i]);
            return 1;
        }
    if (ffcomp_operator_delete(custom) != FFSUCCESS) return 1;
    free(a); free(b); free(c); free(w); free(fa); free(fb); free(fc);
    return 0;
}

int main(int argc, char **argv) {
    const int count = argc > 1 ? atoi(argv[1]) : 10007;
    const int iters = argc > 2 ? atoi(argv[2]) : 4;
    if (ffinit(&argc, &argv) != FFSUCCESS) { fprintf(stderr, "ffinit: %s\n", esgd_last_error()); return 2; }
    int rank, size, failed = 0;
    ffrank(&rank);
    ffsize(&size);
    if (single_computations(count)) { fprintf(stderr, "[rank %d] single computations failed\n", rank); return 1; }
    int32_t *to_reduce = calloc(count, sizeof(int32_t));
    int32_t *reduced = calloc(count, sizeof(int32_t));
    int32_t *want = calloc(count, sizeof(int32_t));

    /* allreduce.c: a fresh schedule per iteration */
    int16_t tag = 0;
    for (int i = 0; i < iters && !failed; ++i) {
        for (int j = 0; j < count; ++j) { to_reduce[j] = i + j; reduced[j] = 0; want[j] = (i + j) * size; }
        ffschedule_h ar;
        if (ffallreduce(to_reduce, reduced, count, tag++, FFSUM, FFINT32, 0, &ar) != FFSUCCESS) {
            fprintf(stderr, "ffallreduce: %s\n", esgd_last_error());
            return 2;
        }
        if (ffschedule_post(ar) != FFSUCCESS || ffschedule_wait(ar) != FFSUCCESS) {
            fprintf(stderr, "[rank %d] allreduce: %s\n", rank, esgd_last_error());
            return 2;
        }
        failed |= check_int(reduced, want, count, "allreduce", i);
        ffschedule_delete(ar);
    }

    /* solo / majority correctness: running inputs, every rank posts behind a barrier */
    for (int kind = 0; kind < 2 && !failed; ++kind) {
        for (int j = 0; j < count; ++j) to_reduce[j] = 0;
        ffschedule_h s;
        int rc = kind == 0 ? ffsolo_allreduce(to_reduce, reduced, count, 0, FFSUM, FFINT32, 0, 20, &s)
                           : ffrand_allreduce(to_reduce, reduced, count, 0, FFSUM, FFINT32, 0, 34495645, 20, &s);
        if (rc != FFSUCCESS) { fprintf(stderr, "schedule: %s\n", esgd_last_error()); return 2; }
        ffschedule_start(s);
        for (int i = 0; i < iters && !failed; ++i) {
            for (int j = 0; j < count; ++j) { to_reduce[j]++; want[j] = to_reduce[j] * size; }
            esgd_barrier();            /* MPI_Barrier in the reference test */
            if (ffschedule_post(s) != FFSUCCESS || ffschedule_wait(s) != FFSUCCESS) {
                fprintf(stderr, "[rank %d] schedule: %s\n", rank, esgd_last_error());
                return 2;
            }
            esgd_barrier();
            failed |= check_int(reduced, want, count, kind == 0 ? "solo" : "majority", i);
        }
        ffschedule_delete(s);
    }
    /* FFCOLL_BUFFERS: relocating / resizing buckets under one persistent schedule */
    if (!failed) {
        const int initial = 1000, max_count = 3 * count;
        int32_t *sbuf = calloc(initial, sizeof(int32_t));
        ffbuffer_h sbh, rbh;
        ffbuffer_create(sbuf, initial, FFINT32, 0, &sbh);     /* user managed */
        ffbuffer_create(NULL, initial, FFINT32, 0, &rbh);     /* library managed */
        ffschedule_h s;
        if (ffallreduce(&sbh, &rbh, initial, 0, FFSUM, FFINT32, FFCOLL_BUFFERS, &s) != FFSUCCESS) {
            fprintf(stderr, "ffallreduce(FFCOLL_BUFFERS): %s\n", esgd_last_error());
            return 2;
        }
        /* same sizes on every rank: a private LCG seeded like the reference (SEED 439634);
         * libc rand() is not usable here, the HIP runtime draws from it too */
        uint32_t lcg = 439634u;
        for (int i = 0; i < iters + 2 && !failed; ++i) {
            lcg = lcg * 1103515245u + 12345u;
            const int c = (int)((lcg >> 8) % (uint32_t)max_count) + 1;
            free(sbuf);
            sbuf = malloc(sizeof(int32_t) * c);
            ffbuffer_resize(sbh, sbuf, c, FFINT32);
            ffbuffer_resize(rbh, NULL, c, FFINT32);
            int32_t *rbuf;
            ffbuffer_get_data(rbh, (void **)&rbuf);
            int32_t *w = malloc(sizeof(int32_t) * c);
            for (int j = 0; j < c; ++j) { sbuf[j] = i + j; rbuf[j] = 0; w[j] = (i + j) * size; }
            if (ffschedule_post(s) != FFSUCCESS || ffschedule_wait(s) != FFSUCCESS) {
                fprintf(stderr, "[rank %d] FFCOLL_BUFFERS round %d: %s\n", rank, i, esgd_last_error());
                failed = 1;
                free(w);
                break;
            }
            failed |= check_int(rbuf, w, c, "FFCOLL_BUFFERS", i);
            free(w);
        }
        ffschedule_delete(s);
        ffbuffer_delete(sbh);
        ffbuffer_delete(rbh);
        free(sbuf);
    }
    /* FFCOLL_BUFFERS under ffsolo_allreduce with a late rank: peers activate the
     * asynchronous rounds, the late rank is carried through them and its own post of a
     * round that already ran must be accepted (the reference takes options =
     * FFCOLL_BUFFERS for ffsolo_allreduce too, src/colls/ffsolo_allreduce.c:20-95).
     * Every rank's bucket holds 1 before the barrier, so every round reduces to size. */
    if (!failed && size > 1) {
        const int c = count;
        int32_t *sbuf = malloc(sizeof(int32_t) * c);
        ffbuffer_h sbh, rbh;
        ffbuffer_create(sbuf, c, FFINT32, 0, &sbh);
        ffbuffer_create(NULL, c, FFINT32, 0, &rbh);
        ffschedule_h s;
        if (ffsolo_allreduce(&sbh, &rbh, c, 0, FFSUM, FFINT32, FFCOLL_BUFFERS, 3, &s) != FFSUCCESS) {
            fprintf(stderr, "ffsolo_allreduce(FFCOLL_BUFFERS): %s\n", esgd_last_error());
            return 2;
        }
        int32_t *w = malloc(sizeof(int32_t) * c);
        for (int j = 0; j < c; ++j) { sbuf[j] = 1; w[j] = size; }
        for (int i = 0; i < iters + 4 && !failed; ++i) {
            esgd_barrier();
            if (rank == size - 1) {
                struct timespec d = {0, 20 * 1000 * 1000};
                nanosleep(&d, NULL);
            }
            if (ffschedule_post(s) != FFSUCCESS || ffschedule_wait(s) != FFSUCCESS) {
                fprintf(stderr, "[rank %d] solo FFCOLL_BUFFERS round %d: %s\n", rank, i, esgd_last_error());
                failed = 1;
                break;
            }
            esgd_barrier();
            int32_t *rbuf;
            ffbuffer_get_data(rbh, (void **)&rbuf);
            failed |= check_int(rbuf, w, c, "solo FFCOLL_BUFFERS", i);
        }
        free(w);
        ffschedule_delete(s);
        ffbuffer_delete(sbh);
        ffbuffer_delete(rbh);
        free(sbuf);
    }
    if (!failed && rank == 0) printf("Correctness check passed! (%d ranks)\n", size);
    fffinalize();
    free(to_reduce); free(reduced); free(want);
    return failed;
}
