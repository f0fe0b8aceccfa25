/*
 * jdeflate/deflator.h -- drop-in replacement for the reference encoder API
 * (Jpn666/jdeflate jdeflate/deflator.h).  Same enums, same public struct
 * layout (deflator.h:81-99, 72 bytes on LP64), same exported functions and
 * header inlines.  The implementation (libjdeflate_amd.so) compresses on an
 * MI355X: input is cut into independent 64 KiB blocks, each encoded exactly
 * as a fresh reference deflator with DEFLT_FLUSH (DEFLT_END for the last)
 * would encode it.
 *
 * With DEFLT_SINGLEWINDOW (an extension) the instance instead buffers the
 * input up to each flush and encodes it as one stream whose 32 KiB window
 * runs across the whole input, exactly as the reference deflator does (its
 * own default): the output is byte-identical to the reference's for the same
 * sequence of calls -- input in pieces without a flush, DEFLT_FLUSH (the
 * window, chains and parser state carry on, deflator.c:763-768) and
 * DEFLT_END.  Output is written at the flushes.
 *
 * Usage is unchanged:
 *   do {
 *       deflator_setsrc(state, source, sourcesize);
 *       do {
 *           deflator_settgt(state, target, targetsize);
 *           result = deflator_deflate(state, final ? DEFLT_END : DEFLT_NOFLUSH);
 *       } while (result == DEFLT_TGTEXHSTD);
 *   } while (result == DEFLT_SRCEXHSTD);
 */
#ifndef JDEFLATE_DEFLATOR_H
#define JDEFLATE_DEFLATOR_H

#include <jdeflate/config/config.h>

#ifdef __cplusplus
extern "C" {
#endif

/* deflator.h:48-53 */
typedef enum {
	DEFLT_OK        = 0,
	DEFLT_SRCEXHSTD = 1,
	DEFLT_TGTEXHSTD = 2,
	DEFLT_ERROR     = 3
} eDEFLTResult;

/* deflator.h:57-61 */
typedef enum {
	DEFLT_NOFLUSH = 0,
	DEFLT_END     = 1,
	DEFLT_FLUSH   = 2
} eDEFLTFlush;

/* deflator.h:65-70 */
typedef enum {
	DEFLT_EBADSTATE     = 1,
	DEFLT_EOOM          = 2,
	DEFLT_ELEVEL        = 3,
	DEFLT_EINCORRECTUSE = 4
} eDEFLTError;

/* deflator.h:74-76 */
typedef enum {
	DEFLT_FIXEDCODES   = 0x01,
	DEFLT_SINGLEWINDOW = 0x100    /* extension: see the header comment */
} eDEFLTFlags;

/* deflator.h:81-99 (ABI: state and error first) */
struct TDeflator {
	const uint32 state;
	const uint32 error;
	const uint32 flags;
	const uint32 flush;

	const uint32 status;

	const uint8* source;
	const uint8* sbgn;
	const uint8* send;

	uint8* target;
	uint8* tbgn;
	uint8* tend;
};

typedef struct TDeflator TDeflator;

/* deflator.h:106-153 */
JDEFLATE_API TDeflator* deflator_create(uintxx flags, intxx level, const TAllocator*);
JDEFLATE_API void deflator_destroy(TDeflator*);
CTB_INLINE void deflator_setsrc(TDeflator*, const uint8* source, uintxx size);
CTB_INLINE void deflator_settgt(TDeflator*, uint8* target, uintxx size);
CTB_INLINE uintxx deflator_srcend(TDeflator*);
CTB_INLINE uintxx deflator_tgtend(TDeflator*);
JDEFLATE_API eDEFLTResult deflator_deflate(TDeflator*, eDEFLTFlush flush);
JDEFLATE_API void deflator_setdctnr(TDeflator*, const uint8* dict, uintxx size);
JDEFLATE_API void deflator_reset(TDeflator*);

/* header inlines, deflator.h:159-203 */
CTB_INLINE void
deflator_setsrc(TDeflator* state, const uint8* source, uintxx size)
{
	CTB_ASSERT(state && source && size);

	if (CTB_EXPECT0(state->flush)) {
		if (state->error == 0) {
			struct TStateHeader {
				uint32 state;
				uint32 error;
			}* h = (struct TStateHeader*) state;
			h->error = DEFLT_EINCORRECTUSE;
			h->state = 0xDEADBEEF;
		}
		return;
	}
	state->source = state->sbgn = state->send = source;
	state->send  += size;
}

CTB_INLINE void
deflator_settgt(TDeflator* state, uint8* target, uintxx size)
{
	CTB_ASSERT(state && target && size);
	state->target = state->tbgn = state->tend = target;
	state->tend  += size;
}

CTB_INLINE uintxx
deflator_srcend(TDeflator* state)
{
	CTB_ASSERT(state);
	return (uintxx) (state->source - state->sbgn);
}

CTB_INLINE uintxx
deflator_tgtend(TDeflator* state)
{
	CTB_ASSERT(state);
	return (uintxx) (state->target - state->tbgn);
}

#ifdef __cplusplus
}
#endif

#endif
