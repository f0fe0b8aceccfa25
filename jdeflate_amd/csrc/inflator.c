/*
 * inflator.c -- drop-in inflator_* API (jdeflate/inflator.h) over the
 * MI355X engine.
 *
 * Result codes, the final-input latch (:770-772), misuse checks (validate
 * :730-762) and poisoning follow inflator.c of the reference, and so does the
 * streaming contract of inflator_inflate (:765-903):
 *
 *  - every call decodes as far as the input given so far allows, with or
 *    without `final`, and delivers those bytes (INFLT_TGTEXHSTD while the
 *    target is too small for them);
 *  - the call in which the final block ends returns INFLT_OK, with `source`
 *    left on the first byte after the stream (bytes that follow the stream
 *    in the caller's buffer are not consumed), whatever `final` says
 *    (:829-833);
 *  - input that runs out mid-stream is INFLT_SRCEXHSTD, or INFLT_ERROR with
 *    INFLT_EINPUTEND once `final` is set (:805-810, :845-848).
 *
 * The decode runs on the GPU through one resumable stream decoder per
 * instance (jdgpu_istream_*): the decoder state -- block mode, the current
 * block's tables, a pending copy, the stored remainder -- and the 32 KiB
 * window stay in device memory between calls, as the reference keeps them in
 * its private state and window ring (decodeblock :1330-1518, copybytes
 * :1214-1290, updatewindow :617-675).  A call hands over exactly its new
 * input and the room left in the target: the output goes straight into the
 * target and stops exactly where the target ends (INFLT_TGTEXHSTD; the input
 * from the first byte not yet used stays with the caller, as `source` shows),
 * and every input bit is decoded once -- only an incomplete token or block
 * header at the end of the input is carried to the next call.  A stream given
 * in one piece is decoded once (its verified FLUSH-joined segments in
 * parallel, the rest by one wave).
 */
#include <jdeflate/inflator.h>
#include <jdeflate/jdgpu.h>

#include "jd_internal.h"

#include <stdlib.h>
#include <string.h>

struct TINFLTPrvt {
	struct TINFLTPblc {
		uint32 state;
		uint32 error;
		uint32 flags;
		uint32 finalinput;
		uint32 status;
		const uint8* source;
		const uint8* sbgn;
		const uint8* send;
		uint8* target;
		uint8* tbgn;
		uint8* tend;
	} public;

	uint32 used;
	uint32 ended;        /* the final block has ended                     */
	JDGPUInflateStream* is;

	uint32* crc;          /* jd_inflator_checksums (zstrm), or NULL      */
	uint32* adler;

	const struct TAllocator* allctr;
};

/* inflator.c:152-154 */
typedef union {
	char a[-1 + (sizeof(struct TInflator) == sizeof(struct TINFLTPblc)) * 2];
} TINFLTStaticAssert;

#define PRVT ((struct TINFLTPrvt*) state)
#define PBLC ((struct TINFLTPblc*) state)

static void* jd_request(uintxx size, void* user) { (void) user; return malloc(size); }
static void jd_dispose(void* p, uintxx size, void* user) { (void) size; (void) user; free(p); }
static const struct TAllocator jd_defaultallocator = { jd_request, jd_dispose, NULL };

TInflator*
inflator_create(uintxx flags, const TAllocator* allctr)
{
	struct TINFLTPrvt* p;

	if (allctr == NULL) {
		allctr = &jd_defaultallocator;
	}
	if (!jdgpu_available()) {
		return NULL;
	}
	p = allctr->request(sizeof(struct TINFLTPrvt), allctr->user);
	if (p == NULL) {
		return NULL;
	}
	memset(p, 0, sizeof(*p));
	p->allctr = allctr;
	p->is = jdgpu_istream_create();
	if (p->is == NULL) {
		allctr->dispose(p, sizeof(struct TINFLTPrvt), allctr->user);
		return NULL;
	}
	inflator_reset((TInflator*) p);
	p->public.flags = (uint32) flags;
	return (TInflator*) p;
}

void
inflator_destroy(TInflator* state)
{
	const struct TAllocator* a;
	if (state == NULL) {
		return;
	}
	a = PRVT->allctr;
	jdgpu_istream_destroy(PRVT->is);
	a->dispose(PRVT, sizeof(struct TINFLTPrvt), a->user);
}

void
inflator_reset(TInflator* state)
{
	CTB_ASSERT(state);
	PBLC->state = 0;
	PBLC->error = 0;
	PBLC->finalinput = 0;
	PBLC->status = 0;
	PBLC->source = NULL;
	PBLC->sbgn = NULL;
	PBLC->send = NULL;
	PBLC->target = NULL;
	PBLC->tbgn = NULL;
	PBLC->tend = NULL;

	PRVT->used = 0;
	PRVT->ended = 0;
	if (jdgpu_istream_reset(PRVT->is, NULL, 0) != 0) {
		PBLC->error = INFLT_EBADSTATE;
		PBLC->state = 0xDEADBEEF;
	}
}

/* inflator_setdctnr :905-925: the dictionary's last 32 KiB are the window
 * the first deflate block may reach into; after use it is misuse */
void
inflator_setdctnr(TInflator* state, const uint8* dict, uintxx size)
{
	CTB_ASSERT(state && dict && size);
	if (PRVT->used) {
		PBLC->error = INFLT_EINCORRECTUSE;
		PBLC->state = 0xDEADBEEF;
		return;
	}
	if (jdgpu_istream_reset(PRVT->is, dict, size) != 0) {
		PBLC->error = INFLT_EBADSTATE;
		PBLC->state = 0xDEADBEEF;
		return;
	}
	PRVT->used = 1;
}

void
jd_inflator_checksums(TInflator* state, uint32* crc, uint32* adler)
{
	PRVT->crc = crc;
	PRVT->adler = adler;
}

/* validate :730-762 */
static int
validate(struct TINFLTPrvt* state)
{
	if (PBLC->source == NULL || PBLC->target == NULL) {
		PBLC->error = INFLT_EINCORRECTUSE;
		return 0;
	}
	switch (PBLC->status) {
		case INFLT_SRCEXHSTD:
			if (PBLC->source == PBLC->send && PBLC->finalinput == 0) {
				PBLC->error = INFLT_EINCORRECTUSE;
				return 0;
			}
			break;
		case INFLT_TGTEXHSTD:
			if (PBLC->target == PBLC->tend) {
				PBLC->error = INFLT_EINCORRECTUSE;
				return 0;
			}
			break;
	}
	return 1;
}

eINFLTResult
inflator_inflate(TInflator* state, uint32 final)
{
	JDGPUInflateStep r;
	uintxx n, room;
	int rc;

	if (PBLC->state == 0xDEADBEEF) {
		return INFLT_ERROR;
	}
	if (PBLC->finalinput == 0 && final) {
		PBLC->finalinput = 1;
	}
	if (validate(PRVT) == 0) {
		PBLC->state = 0xDEADBEEF;
		return INFLT_ERROR;
	}
	PRVT->used = 1;

	n = (uintxx) (PBLC->send - PBLC->source);
	room = (uintxx) (PBLC->tend - PBLC->target);
	rc = jdgpu_istream_inflate(PRVT->is, PBLC->source, n, PBLC->target, room, &r,
	                           PRVT->crc, PRVT->adler);
	if (rc != 0) {
		PBLC->error = rc == JDGPU_EOOM ? INFLT_EOOM : INFLT_EBADSTATE;
		PBLC->state = 0xDEADBEEF;
		return INFLT_ERROR;
	}
	PBLC->source += (uintxx) r.consumed;
	PBLC->target += (uintxx) r.produced;

	switch (r.status) {
		case JDGPU_IS_ENDED:
			/* :829-833: OK, source on the first byte after the stream */
			PRVT->ended = 1;
			PBLC->state = 0xDEADBEEF;
			return (eINFLTResult) (PBLC->status = INFLT_OK);
		case JDGPU_IS_FULL:
			return (eINFLTResult) (PBLC->status = INFLT_TGTEXHSTD);
		case JDGPU_IS_NEEDINPUT:
			if (PBLC->finalinput) {
				/* :805-810, :845-848 */
				PBLC->error = INFLT_EINPUTEND;
				PBLC->state = 0xDEADBEEF;
				return INFLT_ERROR;
			}
			return (eINFLTResult) (PBLC->status = INFLT_SRCEXHSTD);
		default:
			PBLC->error = (uint32) r.error;
			PBLC->state = 0xDEADBEEF;
			return INFLT_ERROR;
	}
}
