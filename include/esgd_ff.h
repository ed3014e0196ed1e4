/*
 * esgd_ff.h — the subset of fflib2's public API that eager-SGD's callers bind,
 * re-implemented by libesgd.so on MI355X (HIP tree reduction + IPC/xGMI data plane).
 *
 * Each declaration names the reference entry point it replaces
 * (/root/reference/eager-SGD-modules/fflib2/src/ff.h).  Constants keep the reference's
 * values so that existing callers compile unchanged against include/ff.h.
 * Differences (documented in INTEGRATION.md):
 *   - no MPI: ranks are the processes of one node (env RANK / WORLD_SIZE / LOCAL_RANK
 *     as set by torch.distributed.run, or OMPI_ / PMI_ / SLURM_ equivalents), joined
 *     through a node-local shared segment named by ESGD_JOB_ID (or
 *     TORCHELASTIC_RUN_ID + MASTER_PORT);
 *   - operator FFSUM only (the reference's generic comp also has FFIDENTITY, used
 *     internally for the move) ; datatypes FFINT32/FFINT64/FFDOUBLE/FFFLOAT + ESGD_FFBF16;
 *   - FFCOLL_BUFFERS takes host ffbuffer_h buckets (no FFBUFFER_IDX buffers);
 *   - extension option ESGD_FF_DEVICE_BUFFERS: sndbuff/rcvbuff are device pointers.
 */
#ifndef ESGD_FF_H
#define ESGD_FF_H

#include <stdint.h>

#include "esgd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* return codes (src/ff.h:4-10) */
#define FFCOMPLETED 1
#define FFSUCCESS 0
#define FFERROR -1
#define FFINVALID_ARG -2
#define FFTOO_MANY_DEPS -3
#define FFENOMEM -4
#define FFVERSION -5

/* datatypes (src/ff.h:21-31) */
#define FFINT32 0
#define FFINT64 1
#define FFDOUBLE 2
#define FFFLOAT 3
#define ESGD_FFBF16 16   /* extension */

/* operators (src/ff.h:34-40); only FFSUM reduces here */
#define FFSUM 0
#define FFPROD 1
#define FFMAX 2
#define FFMIN 3
#define FFIDENTITY 4
#define FFOPERATOR_SENTINEL 5
#define FFCUSTOM 6                         /* first user operator handle (src/ff.h:41) */

/* options used by collective callers (src/ff.h:43-58) */
#define FFCOLL_BUFFERS (1 << 7)
#define ESGD_FF_DEVICE_BUFFERS (1 << 20)   /* extension: sndbuff/rcvbuff on the device */

#define FFINPLACE ((void *)0x1)            /* src/ff.h:62 */

typedef int ffdatatype_h;
typedef int ffoperator_h;
typedef uint64_t ffschedule_h;
typedef uint64_t ffbuffer_h;
typedef uint64_t ffop_h;
typedef int (*ffoperator_fun_t)(void *, void *, void *, uint32_t, ffdatatype_h);

/* buffer descriptors (src/ffbuffer.c:10-95): addr NULL = library-allocated (grows on
 * resize like the reference's realloc).  With FFCOLL_BUFFERS a collective takes
 * pointers to ffbuffer_h and re-reads address and count at every post, so buckets may
 * move and change size between rounds (evaluation/allreduce_buffers_*.c); every rank
 * must use the same count in a round. */
int ffbuffer_create(void *addr, uint32_t count, ffdatatype_h datatype, int options, ffbuffer_h *buf);
int ffbuffer_delete(ffbuffer_h buf);
int ffbuffer_resize(ffbuffer_h buf, void *addr, uint32_t new_count, ffdatatype_h new_datatype);
int ffbuffer_get_size(ffbuffer_h buf, uint32_t *count, ffdatatype_h *datatype);
int ffbuffer_get_data(ffbuffer_h buf, void **mem);

int ffinit(int *argc, char ***argv);   /* src/ff.c:23-86 (MPI_Init + progress thread) */
int fffinalize(void);                  /* src/ff.c:88- */
int ffrank(int *rank);                 /* src/ff.h:102 */
int ffsize(int *size);                 /* src/ff.h:103 */

/* src/colls/ffallreduce.c:74 — every round synchronous */
int ffallreduce(void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h ffoperator,
                ffdatatype_h datatype, int options, ffschedule_h *sched);
/* src/colls/ffsolo_allreduce.c:20 — solo allreduce with a limiter of `async` */
int ffsolo_allreduce(void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h ffoperator,
                     ffdatatype_h datatype, int options, int async, ffschedule_h *sched);
/* src/colls/ffrand_allreduce.c:27 — majority allreduce, activator rand_r(&seed) % P */
int ffrand_allreduce(void *sndbuff, void *rcvbuff, int count, int16_t tag, ffoperator_h ffoperator,
                     ffdatatype_h datatype, int options, int seed, int async, ffschedule_h *sched);

int ffschedule_start(ffschedule_h sched);              /* src/ffschedule.c (arms receives) */
int ffschedule_post(ffschedule_h sched);               /* src/ffschedule.c:84-88 */
int ffschedule_wait(ffschedule_h sched);
int ffschedule_test(ffschedule_h sched, int *flag);
int ffschedule_delete(ffschedule_h sched);

/* extension: post with the stream that produced sndbuff (device buffers) */
int ffschedule_post_stream(ffschedule_h sched, void *stream);

/* One computation (src/ffcomp.c:7-38, ff.h:132-135): posting it runs the reduction kernel
 * once over MIN(count1, count2, count3) elements (src/components/gcomp/ffop_gcomp.c:29-64):
 * FFSUM c = a + b, FFIDENTITY c = a (b may be NULL).  Host buffers (the reference's); with
 * ESGD_FF_DEVICE_BUFFERS device buffers.  ffcomp_b takes ffbuffer_h descriptors and re-reads
 * them at every post.  User operators (ffcomp_operator_create: a host function, handles
 * FFCUSTOM + i, src/components/gcomp/ffop_gcomp_operator.c:124-141) run as the reference runs
 * them -- the function itself, on the host, over host buffers, once per post
 * (ffop_gcomp.c:52-55; its status is the post's) -- and are refused with device buffers and
 * by the allreduce schedules, whose GPU reductions are FFSUM.  FFPROD / FFMAX
 * / FFMIN have no implementation in the reference either: FFINVALID_ARG. */
int ffcomp(void *addr1, void *addr2, int count, ffdatatype_h datatype, ffoperator_h ffoperator, int options,
           void *addr3, ffop_h *op);
int ffcomp_b(ffbuffer_h buffer1, ffbuffer_h buffer2, ffoperator_h ffoperator, int options, ffbuffer_h buffer3,
             ffop_h *op);
int ffcomp_operator_create(ffoperator_fun_t fun, int commutative, ffoperator_h *handle);
int ffcomp_operator_delete(ffoperator_h handle);
int ffop_post(ffop_h op);              /* src/ffop.c:59-72 */
int ffop_wait(ffop_h op);              /* src/ffop.c:143-177 */
int ffop_test(ffop_h op, int *flag);
int ffop_free(ffop_h op);

#ifdef __cplusplus
}
#endif
#endif /* ESGD_FF_H */
