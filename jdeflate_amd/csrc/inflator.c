/*
 * inflator.c -- drop-in inflator_* API (jdeflate/inflator.h) over the
 * MI355X engine.
 *
 * Result codes, the final-input latch (:770-772), misuse checks (validate
 * :730-762) and poisoning follow inflator.c of the reference.  The stream is
 * decoded on the GPU once the final input has been supplied: input given
 * without `final` is consumed and buffered (INFLT_SRCEXHSTD), then the
 * whole stream is inflated and the output is delivered across as many
 * INFLT_TGTEXHSTD calls as the caller's target needs.  The decoded bytes are
 * the reference's; on corrupt input the error is reported once, after the
 * bytes decoded before it were delivered.
 */
#include <jdeflate/inflator.h>
#include <jdeflate/jdgpu.h>

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
	uint32 decoded;      /* the GPU pass has run                    */
	int32 pendingerr;    /* error to report after the output        */

	uint8* dict;          /* inflator_setdctnr: the window's first bytes */
	uintxx dictlen;

	uint8* inbuf;
	uintxx incap;
	uintxx inlen;
	uint8* outbuf;
	uintxx outcap;
	uintxx outlen;
	uintxx outpos;

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
	inflator_reset((TInflator*) p);
	p->public.flags = (uint32) flags;
	return (TInflator*) p;
}

static void
release(struct TINFLTPrvt* state)
{
	const struct TAllocator* a = PRVT->allctr;
	if (PRVT->inbuf) {
		a->dispose(PRVT->inbuf, PRVT->incap, a->user);
	}
	if (PRVT->outbuf) {
		a->dispose(PRVT->outbuf, PRVT->outcap, a->user);
	}
	if (PRVT->dict) {
		a->dispose(PRVT->dict, 32768, a->user);
	}
	PRVT->dict = NULL;
	PRVT->inbuf = NULL;
	PRVT->outbuf = NULL;
	PRVT->incap = 0;
	PRVT->outcap = 0;
}

void
inflator_destroy(TInflator* state)
{
	const struct TAllocator* a;
	if (state == NULL) {
		return;
	}
	a = PRVT->allctr;
	release(PRVT);
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
	PRVT->dictlen = 0;
	PRVT->decoded = 0;
	PRVT->pendingerr = 0;
	PRVT->inlen = 0;
	PRVT->outlen = 0;
	PRVT->outpos = 0;
}

/* inflator_setdctnr :905-925: the dictionary's last 32 KiB prime the window
 * (the stream decoder starts after them); after use it is misuse */
void
inflator_setdctnr(TInflator* state, const uint8* dict, uintxx size)
{
	CTB_ASSERT(state && dict && size);
	if (PRVT->used) {
		PBLC->error = INFLT_EINCORRECTUSE;
		PBLC->state = 0xDEADBEEF;
		return;
	}
	if (PRVT->dict == NULL) {
		PRVT->dict = PRVT->allctr->request(32768, PRVT->allctr->user);
		if (PRVT->dict == NULL) {
			PBLC->error = INFLT_EOOM;
			PBLC->state = 0xDEADBEEF;
			return;
		}
	}
	if (size > 32768) {
		dict = (dict + size) - 32768;
		size = 32768;
	}
	memcpy(PRVT->dict, dict, size);
	PRVT->dictlen = size;
	PRVT->used = 1;
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

static int
append(struct TINFLTPrvt* state, const uint8* p, uintxx n)
{
	const struct TAllocator* a = PRVT->allctr;
	if (PRVT->inlen + n > PRVT->incap) {
		uintxx cap = PRVT->incap ? PRVT->incap : 65536;
		uint8* q;
		while (cap < PRVT->inlen + n) {
			cap *= 2;
		}
		q = a->request(cap, a->user);
		if (q == NULL) {
			return 0;
		}
		if (PRVT->inlen) {
			memcpy(q, PRVT->inbuf, PRVT->inlen);
		}
		if (PRVT->inbuf) {
			a->dispose(PRVT->inbuf, PRVT->incap, a->user);
		}
		PRVT->inbuf = q;
		PRVT->incap = cap;
	}
	memcpy(PRVT->inbuf + PRVT->inlen, p, n);
	PRVT->inlen += n;
	return 1;
}

/* run the decoder, growing the output buffer until the stream fits */
static int
decode(struct TINFLTPrvt* state, uintxx* consumed)
{
	const struct TAllocator* a = PRVT->allctr;
	uintxx cap = PRVT->inlen * 4 + 65536;
	uintxx limit = PRVT->inlen * 1032 + 65536;   /* deflate's max ratio */

	for (;;) {
		uint64 produced = 0;
		uint64 used = 0;
		int32 err = 0;
		int r;

		if (PRVT->outcap < cap) {
			if (PRVT->outbuf) {
				a->dispose(PRVT->outbuf, PRVT->outcap, a->user);
			}
			PRVT->outbuf = a->request(cap, a->user);
			PRVT->outcap = PRVT->outbuf ? cap : 0;
			if (PRVT->outbuf == NULL) {
				PBLC->error = INFLT_EOOM;
				return 0;
			}
		}
		if (PRVT->dictlen) {
			r = jdgpu_inflate_stream_dict(PRVT->dict, PRVT->dictlen, PRVT->inbuf,
			                              PRVT->inlen, PRVT->outbuf, PRVT->outcap,
			                              &produced, &used, &err);
		} else {
			r = jdgpu_inflate_stream(PRVT->inbuf, PRVT->inlen, PRVT->outbuf,
			                         PRVT->outcap, &produced, &used, &err);
		}
		if (r < 0) {
			PBLC->error = r == JDGPU_EOOM ? INFLT_EOOM : INFLT_EBADSTATE;
			return 0;
		}
		if (err == JDGPU_EBLOCKOVERFLOW && cap < limit) {
			cap = cap * 4 < limit ? cap * 4 : limit;
			continue;
		}
		PRVT->outlen = (uintxx) produced;
		PRVT->outpos = 0;
		PRVT->pendingerr = err == JDGPU_EBLOCKOVERFLOW ? INFLT_EBADSTATE : err;
		*consumed = (uintxx) used;
		return 1;
	}
}

eINFLTResult
inflator_inflate(TInflator* state, uint32 final)
{
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

	if (!PRVT->decoded) {
		uintxx n = (uintxx) (PBLC->send - PBLC->source);
		uintxx before = PRVT->inlen;
		uintxx consumed = 0;

		if (n && !append(PRVT, PBLC->source, n)) {
			PBLC->error = INFLT_EOOM;
			PBLC->state = 0xDEADBEEF;
			return INFLT_ERROR;
		}
		PBLC->source = PBLC->send;
		if (!PBLC->finalinput) {
			return (eINFLTResult) (PBLC->status = INFLT_SRCEXHSTD);
		}
		if (!decode(PRVT, &consumed)) {
			PBLC->state = 0xDEADBEEF;
			return INFLT_ERROR;
		}
		/* leave unconsumed trailing bytes of this call's buffer */
		if (PRVT->pendingerr == 0 && consumed >= before && consumed < PRVT->inlen) {
			PBLC->source = PBLC->send - (PRVT->inlen - consumed);
		}
		PRVT->decoded = 1;
	}

	{
		uintxx n = PRVT->outlen - PRVT->outpos;
		uintxx room = (uintxx) (PBLC->tend - PBLC->target);
		if (n > room) {
			n = room;
		}
		memcpy(PBLC->target, PRVT->outbuf + PRVT->outpos, n);
		PBLC->target += n;
		PRVT->outpos += n;
		if (PRVT->outpos < PRVT->outlen) {
			return (eINFLTResult) (PBLC->status = INFLT_TGTEXHSTD);
		}
	}
	if (PRVT->pendingerr) {
		PBLC->error = (uint32) PRVT->pendingerr;
		PBLC->state = 0xDEADBEEF;
		return INFLT_ERROR;
	}
	PBLC->state = 0xDEADBEEF;
	return (eINFLTResult) (PBLC->status = INFLT_OK);
}
