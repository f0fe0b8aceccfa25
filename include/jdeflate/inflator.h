/*
 * jdeflate/inflator.h -- drop-in replacement for the reference decoder API
 * (Jpn666/jdeflate jdeflate/inflator.h).  Same enums, same public struct
 * layout (inflator.h:71-89), same exported functions and header inlines.
 * The implementation decodes on an MI355X.
 */
#ifndef JDEFLATE_INFLATOR_H
#define JDEFLATE_INFLATOR_H

#include <jdeflate/config/config.h>

#ifdef __cplusplus
extern "C" {
#endif

/* inflator.h:48-53 */
typedef enum {
	INFLT_OK        = 0,
	INFLT_SRCEXHSTD = 1,
	INFLT_TGTEXHSTD = 2,
	INFLT_ERROR     = 3
} eINFLTResult;

/* inflator.h:57-66 */
typedef enum {
	INFLT_EBADSTATE     = 1,
	INFLT_EBADCODE      = 2,
	INFLT_EBADTREE      = 3,
	INFLT_EFAROFFSET    = 4,
	INFLT_EBADBLOCK     = 5,
	INFLT_EINPUTEND     = 6,
	INFLT_EOOM          = 7,
	INFLT_EINCORRECTUSE = 8
} eINFLTError;

/* inflator.h:71-89 */
struct TInflator {
	const uint32 state;
	const uint32 error;
	const uint32 flags;
	const uint32 finalinput;

	const uint32 status;

	const uint8* source;
	const uint8* sbgn;
	const uint8* send;

	uint8* target;
	uint8* tbgn;
	uint8* tend;
};

typedef struct TInflator TInflator;

/* inflator.h:97-139 */
JDEFLATE_API TInflator* inflator_create(uintxx flags, const TAllocator*);
JDEFLATE_API void inflator_destroy(TInflator*);
CTB_INLINE void inflator_setsrc(TInflator*, const uint8* source, uintxx size);
CTB_INLINE void inflator_settgt(TInflator*, uint8* target, uintxx size);
CTB_INLINE uintxx inflator_srcend(TInflator*);
CTB_INLINE uintxx inflator_tgtend(TInflator*);
JDEFLATE_API eINFLTResult inflator_inflate(TInflator*, uint32 final);
JDEFLATE_API void inflator_setdctnr(TInflator*, const uint8* dict, uintxx size);
JDEFLATE_API void inflator_reset(TInflator*);

/* header inlines, inflator.h:145-189 */
CTB_INLINE void
inflator_setsrc(TInflator* state, const uint8* source, uintxx size)
{
	CTB_ASSERT(state && source && size);

	if (CTB_EXPECT0(state->finalinput)) {
		if (state->error == 0) {
			struct TStateHeader {
				uint32 state;
				uint32 error;
			}* h = (struct TStateHeader*) state;
			h->error = INFLT_EINCORRECTUSE;
			h->state = 0xDEADBEEF;
		}
		return;
	}
	state->source = state->sbgn = state->send = source;
	state->send  += size;
}

CTB_INLINE void
inflator_settgt(TInflator* state, uint8* target, uintxx size)
{
	CTB_ASSERT(state && target && size);
	state->target = state->tbgn = state->tend = target;
	state->tend  += size;
}

CTB_INLINE uintxx
inflator_srcend(TInflator* state)
{
	CTB_ASSERT(state);
	return (uintxx) (state->source - state->sbgn);
}

CTB_INLINE uintxx
inflator_tgtend(TInflator* state)
{
	CTB_ASSERT(state);
	return (uintxx) (state->target - state->tbgn);
}

#ifdef __cplusplus
}
#endif

#endif
