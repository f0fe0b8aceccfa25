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
 * The decode runs on the GPU (jdgpu_inflate_resume).  Between calls the
 * state is a resume point: the start of the last deflate block begun (a bit
 * position in the buffered input) plus the 32 KiB of output before it, the
 * counterpart of the reference's window ring (updatewindow :617-675).  The
 * next call decodes from there over the buffered and the new input; the
 * bytes it re-decodes up to what was already delivered are skipped.  So the
 * host keeps at most one deflate block of input plus the caller's new chunk,
 * and a stream given in one piece is decoded once (its verified FLUSH-joined
 * prefix in parallel, the rest by one wave).
 */
#include <jdeflate/inflator.h>
#include <jdeflate/jdgpu.h>

#include "jd_internal.h"

#include <stdlib.h>
#include <string.h>

#define WINDOW 32768

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
	uint32 ended;        /* the final block has ended: OK once drained  */
	int32 pendingerr;    /* error to report once the output is drained  */
	uint32 needrun;      /* input (or `final`) arrived since the last decode */

	/* resume point */
	uint8* window;       /* WINDOW bytes: the output before it           */
	uintxx wlen;
	uint32 bit0;         /* bits of inbuf[0] already consumed           */
	uint8* inbuf;        /* input from the resume point on              */
	uintxx incap;
	uintxx inlen;
	uint64 skip;         /* bytes after the resume point already delivered */

	/* output of the last decode, delivered from outpos */
	uint8* outbuf;
	uintxx outcap;
	uintxx outlen;
	uintxx outpos;

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
	p->window = allctr->request(WINDOW, allctr->user);
	if (p->window == NULL) {
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
	if (PRVT->inbuf) {
		a->dispose(PRVT->inbuf, PRVT->incap, a->user);
	}
	if (PRVT->outbuf) {
		a->dispose(PRVT->outbuf, PRVT->outcap, a->user);
	}
	a->dispose(PRVT->window, WINDOW, a->user);
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
	PRVT->pendingerr = 0;
	PRVT->needrun = 0;
	PRVT->wlen = 0;
	PRVT->bit0 = 0;
	PRVT->inlen = 0;
	PRVT->skip = 0;
	PRVT->outlen = 0;
	PRVT->outpos = 0;
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
	if (size > WINDOW) {
		dict = (dict + size) - WINDOW;
		size = WINDOW;
	}
	memcpy(PRVT->window, dict, size);
	PRVT->wlen = size;
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

/* grow *buf (cap *bcap, first `keep` bytes kept) to at least `need` */
static int
reserve(struct TINFLTPrvt* state, uint8** buf, uintxx* bcap, uintxx keep, uintxx need)
{
	const struct TAllocator* a = PRVT->allctr;
	uintxx cap;
	uint8* q;

	if (need <= *bcap) {
		return 1;
	}
	cap = *bcap ? *bcap : 65536;
	while (cap < need) {
		cap *= 2;
	}
	q = a->request(cap, a->user);
	if (q == NULL) {
		return 0;
	}
	if (keep) {
		memcpy(q, *buf, keep);
	}
	if (*buf) {
		a->dispose(*buf, *bcap, a->user);
	}
	*buf = q;
	*bcap = cap;
	return 1;
}

/* move the resume point to the start of the last deflate block begun:
 * the window becomes the 32 KiB of output before it (out[0, rout) follows
 * the old window), and the input from its byte on -- src[rbit / 8, n) --
 * is what stays buffered */
static int
resume_at(struct TINFLTPrvt* state, const uint8* src, uintxx n, const uint8* out,
          uint64 rbit, uint64 rout, uint64 produced)
{
	uintxx byte = (uintxx) (rbit >> 3);
	uintxx k = (uintxx) rout;

	if (k >= WINDOW) {
		memcpy(PRVT->window, out + k - WINDOW, WINDOW);
		PRVT->wlen = WINDOW;
	}
	else if (k) {
		uintxx keep = PRVT->wlen + k > WINDOW ? WINDOW - k : PRVT->wlen;
		memmove(PRVT->window, PRVT->window + PRVT->wlen - keep, keep);
		memcpy(PRVT->window + keep, out, k);
		PRVT->wlen = keep + k;
	}
	if (src == PRVT->inbuf) {
		memmove(PRVT->inbuf, PRVT->inbuf + byte, n - byte);
	}
	else {
		if (!reserve(PRVT, &PRVT->inbuf, &PRVT->incap, 0, n - byte)) {
			return 0;
		}
		memcpy(PRVT->inbuf, src + byte, n - byte);
	}
	PRVT->inlen = n - byte;
	PRVT->bit0 = (uint32) (rbit & 7);
	PRVT->skip = produced - rout;
	return 1;
}

/* one decode of src[0, n) from the resume point into out[0, cap); the
 * checksums advance only when the result is kept (not an overflow) */
static int
run(struct TINFLTPrvt* state, const uint8* src, uintxx n, uint8* out, uint64 cap,
    JDGPUInflateResult* res)
{
	uint32 c = PRVT->crc ? *PRVT->crc : 0, a = PRVT->adler ? *PRVT->adler : 0;
	int r = jdgpu_inflate_resume(PRVT->window, (uint32) PRVT->wlen, src, n, n, PRVT->bit0, out,
	                             cap, res, PRVT->skip, PRVT->crc ? &c : NULL,
	                             PRVT->adler ? &a : NULL);
	if (r < 0) {
		PBLC->error = r == JDGPU_EOOM ? INFLT_EOOM : INFLT_EBADSTATE;
		return 0;
	}
	if (res->error != JDGPU_EBLOCKOVERFLOW) {
		if (PRVT->crc) *PRVT->crc = c;
		if (PRVT->adler) *PRVT->adler = a;
	}
	return 1;
}

/* Decode everything given since the resume point: src[0, n) is the
 * caller's buffer when nothing was buffered before (no copy), else the
 * instance's buffer.  With nothing to skip and a target at least as large
 * as the input, the bytes are decoded straight into the target; otherwise
 * (or when that target overflows) into the staging buffer.  Returns 0 on
 * an engine failure (error set). */
static int
decode(struct TINFLTPrvt* state, const uint8* src, uintxx n, uintxx callbytes)
{
	JDGPUInflateResult res;
	uint64 limit = (uint64) n * 1032 + 65536;   /* deflate's max ratio */
	uint64 cap = (uint64) n * 4 + 65536 + PRVT->skip;
	uintxx room = (uintxx) (PBLC->tend - PBLC->target);
	const uint8* out = NULL;

	if (PRVT->skip == 0 && room >= n && room >= 4096) {
		if (!run(PRVT, src, n, PBLC->target, room, &res)) {
			return 0;
		}
		if (res.error != JDGPU_EBLOCKOVERFLOW) {
			out = PBLC->target;
			PBLC->target += (uintxx) res.produced;
			PRVT->outlen = PRVT->outpos = 0;
		}
	}
	while (out == NULL) {
		if (cap > limit) {
			cap = limit;
		}
		if (!reserve(PRVT, &PRVT->outbuf, &PRVT->outcap, 0, (uintxx) cap)) {
			PBLC->error = INFLT_EOOM;
			return 0;
		}
		if (!run(PRVT, src, n, PRVT->outbuf, cap, &res)) {
			return 0;
		}
		if (res.error == JDGPU_EBLOCKOVERFLOW && cap < limit) {
			cap *= 4;
			continue;
		}
		out = PRVT->outbuf;
		PRVT->outlen = (uintxx) res.produced;
		PRVT->outpos = PRVT->skip < res.produced ? (uintxx) PRVT->skip : PRVT->outlen;
	}

	PRVT->needrun = 0;
	/* the caller's input is taken; at the end of the stream the bytes after
	 * it go back (they can only be in this call's buffer) */
	PBLC->source = PBLC->send;
	switch (res.error) {
		case 0:
			PRVT->ended = 1;
			if (res.consumed >= n - callbytes) {
				PBLC->source = PBLC->send - (n - (uintxx) res.consumed);
			}
			break;
		case INFLT_EINPUTEND:
			if (PBLC->finalinput) {
				PRVT->pendingerr = INFLT_EINPUTEND;
			}
			else if (!resume_at(PRVT, src, n, out, res.resumebit, res.resumeout, res.produced)) {
				PBLC->error = INFLT_EOOM;
				return 0;
			}
			break;
		case JDGPU_EBLOCKOVERFLOW:
			PRVT->pendingerr = INFLT_EBADSTATE;
			break;
		default:
			PRVT->pendingerr = res.error;
	}
	return 1;
}

/* copy staged output to the target; 1 when all of it went */
static int
deliver(struct TINFLTPrvt* state)
{
	uintxx n = PRVT->outlen - PRVT->outpos;
	uintxx room = (uintxx) (PBLC->tend - PBLC->target);

	if (n > room) {
		n = room;
	}
	if (n) {
		memcpy(PBLC->target, PRVT->outbuf + PRVT->outpos, n);
		PBLC->target += n;
		PRVT->outpos += n;
	}
	return PRVT->outpos == PRVT->outlen;
}

eINFLTResult
inflator_inflate(TInflator* state, uint32 final)
{
	if (PBLC->state == 0xDEADBEEF) {
		return INFLT_ERROR;
	}
	if (PBLC->finalinput == 0 && final) {
		PBLC->finalinput = 1;
		PRVT->needrun = 1;
	}
	if (validate(PRVT) == 0) {
		PBLC->state = 0xDEADBEEF;
		return INFLT_ERROR;
	}
	PRVT->used = 1;

	/* output decoded by an earlier call first */
	if (!deliver(PRVT)) {
		return (eINFLTResult) (PBLC->status = INFLT_TGTEXHSTD);
	}

	if (!PRVT->ended && !PRVT->pendingerr) {
		uintxx n = (uintxx) (PBLC->send - PBLC->source);
		const uint8* src = PBLC->source;
		uintxx srclen = n;

		if (n) {
			PRVT->needrun = 1;
		}
		if (!PRVT->needrun) {
			return (eINFLTResult) (PBLC->status = INFLT_SRCEXHSTD);
		}
		if (PRVT->inlen) {
			/* continue the buffered input */
			if (!reserve(PRVT, &PRVT->inbuf, &PRVT->incap, PRVT->inlen, PRVT->inlen + n)) {
				PBLC->error = INFLT_EOOM;
				PBLC->state = 0xDEADBEEF;
				return INFLT_ERROR;
			}
			memcpy(PRVT->inbuf + PRVT->inlen, PBLC->source, n);
			PRVT->inlen += n;
			src = PRVT->inbuf;
			srclen = PRVT->inlen;
		}
		if (!decode(PRVT, src, srclen, n)) {
			PBLC->state = 0xDEADBEEF;
			return INFLT_ERROR;
		}
		if (!deliver(PRVT)) {
			return (eINFLTResult) (PBLC->status = INFLT_TGTEXHSTD);
		}
	}

	if (PRVT->ended) {
		/* :829-833 */
		PBLC->state = 0xDEADBEEF;
		return (eINFLTResult) (PBLC->status = INFLT_OK);
	}
	if (PRVT->pendingerr) {
		PBLC->error = (uint32) PRVT->pendingerr;
		PBLC->state = 0xDEADBEEF;
		return INFLT_ERROR;
	}
	return (eINFLTResult) (PBLC->status = INFLT_SRCEXHSTD);
}
