/*
 * jd_prof.h -- optional per-kernel timing with HIP events recorded on the
 * stream each kernel is launched on (bench.py's live roofline figure).
 * Off by default; when on, two events bracket every kernel launch.
 */
#ifndef JD_PROF_H
#define JD_PROF_H

#include <hip/hip_runtime.h>

enum {
    JDK_CHAINS4 = 0, JDK_CHAINS3, JDK_MATCH, JDK_PARSE, JDK_EMIT, JDK_STORED,
    JDK_SCAN, JDK_COMPACT, JDK_INFLATE, JDK_INFLATE_P1, JDK_INFLATE_P2,
    JDK_PSPEC, JDK_PSYNC, JDK_PJOIN, JDK_CHECKSUM, JDK_INFLATE_MP,
    JDK_FSP_FIND, JDK_FSP_DECODE, JDK_FSP_WINDOW, JDK_FSP_RESOLVE, JDK_INFLATE_RPAR, JDK_PORDER,
    JDK_COUNT
};

#ifdef __cplusplus
extern "C" {
#endif
int jdprof_on(void);
/* returns a pair of pooled events to record around kernel `kid`, or 0 */
int jdprof_begin(int kid, hipStream_t st, int* slot);
void jdprof_end(int slot, hipStream_t st);
#ifdef __cplusplus
}
#endif

#define JDPROF_RUN(kid, st, launch)                                   \
    do {                                                              \
        int slot_ = -1;                                               \
        const int on_ = jdprof_on() && jdprof_begin((kid), (st), &slot_); \
        launch;                                                       \
        if (on_) jdprof_end(slot_, (st));                             \
    } while (0)

#endif
