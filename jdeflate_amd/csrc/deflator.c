/*
 * deflator.c -- drop-in deflator_* API (jdeflate/deflator.h) over the
 * MI355X engine.
 *
 * Streaming semantics follow deflator.c of the reference: the state
 * machine, flush latch (:697-699), misuse checks (validate :664-688),
 * poisoning (state 0xDEADBEEF, :780-785) and result codes are the same.
 * What differs is where blocks start: input is gathered into 64 KiB blocks
 * and every block is encoded by the GPU as a fresh reference deflator would
 * encode it (DEFLT_FLUSH, or the caller's flush for the last block of a
 * flush).  Input is batched (up to JD_BATCH bytes) so a buffer-mode call
 * compresses all its blocks in one GPU launch sequence.
 * With DEFLT_SINGLEWINDOW the input up to a flush is kept whole and encoded
 * as the reference encodes it, one window over the whole stream
 * (jdgpu_stream_deflate): the ends of the calls that delivered it are
 * recorded (they decide where the reference's window fills and slides), and
 * a DEFLT_FLUSH carries the window into the next piece (:763-768).  The
 * output is then the reference's own.
 */
#include <jdeflate/deflator.h>
#include <jdeflate/jdgpu.h>

#include "jd_internal.h"

#include <stdlib.h>
#include <string.h>

#define JD_BLOCKSIZE 65536u
/* the pending-input buffer starts at JD_BATCH0 and doubles while input keeps
 * arriving faster than it is flushed, up to JD_BATCH: a GPU launch sequence
 * needs ~16,384 blocks to fill 256 CUs (k_pspec runs a lane per segment) */
#define JD_BATCH0 (1u << 20)
#define JD_BATCH  (256u << 20)

struct TDEFLTPrvt {
	struct TDEFLTPblc {
		uint32 state;
		uint32 error;
		uint32 flags;
		uint32 flush;
		uint32 status;
		const uint8* source;
		const uint8* sbgn;
		const uint8* send;
		uint8* target;
		uint8* tbgn;
		uint8* tend;
	} public;

	int32 level;
	uint32 used;
	uint32 closing;       /* flush in progress: input closed, draining */
	uint32 swin;          /* DEFLT_SINGLEWINDOW: one window over the input */

	uint8* dict;          /* DEFLT_SINGLEWINDOW: preset dictionary     */
	uintxx dictlen;
	JDGPUStream* strm;    /* DEFLT_SINGLEWINDOW: the carried stream     */
	uint64* cends;        /* ends (in inbuf) of the calls since the flush */
	uintxx ncends;
	uintxx capcends;

	uint8* inbuf;         /* pending input (not yet compressed)        */
	uintxx incap;
	uintxx inlen;
	uint8* outbuf;        /* compressed bytes not yet delivered        */
	uintxx outcap;
	uintxx outlen;
	uintxx outpos;

	uint32* crc;          /* jd_deflator_checksums (zstrm), or NULL      */
	uint32* adler;

	const struct TAllocator* allctr;
};

/* deflator.c:201-203 */
typedef union {
	char a[-1 + (sizeof(struct TDeflator) == sizeof(struct TDEFLTPblc)) * 2];
} TDEFLTStaticAssert;

#define PRVT ((struct TDEFLTPrvt*) state)
#define PBLC ((struct TDEFLTPblc*) state)

static void* jd_request(uintxx size, void* user) { (void) user; return malloc(size); }
static void jd_dispose(void* p, uintxx size, void* user) { (void) size; (void) user; free(p); }
static const struct TAllocator jd_defaultallocator = { jd_request, jd_dispose, NULL };

static uintxx outcap_for(uintxx n)
{
	return (uintxx) jdgpu_bound(n, JD_BLOCKSIZE);
}

TDeflator*
deflator_create(uintxx flags, intxx level, const TAllocator* allctr)
{
	struct TDEFLTPrvt* p;

	if (level > 9 || level < 0) {
		return NULL;
	}
	if (allctr == NULL) {
		allctr = &jd_defaultallocator;
	}
	if (!jdgpu_available()) {
		/* the product path has no CPU fallback */
		return NULL;
	}
	p = allctr->request(sizeof(struct TDEFLTPrvt), allctr->user);
	if (p == NULL) {
		return NULL;
	}
	memset(p, 0, sizeof(*p));
	p->allctr = allctr;
	p->level = (int32) level;
	p->swin = (flags & DEFLT_SINGLEWINDOW) ? 1 : 0;
	p->outcap = outcap_for(JD_BATCH0);
	p->incap = JD_BATCH0;
	p->inbuf = allctr->request(p->incap, allctr->user);
	p->outbuf = allctr->request(p->outcap, allctr->user);
	if (p->inbuf == NULL || p->outbuf == NULL) {
		deflator_destroy((TDeflator*) p);
		return NULL;
	}
	deflator_reset((TDeflator*) p);
	p->public.flags = (uint32) flags;
	return (TDeflator*) p;
}

void
deflator_destroy(TDeflator* state)
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
	if (PRVT->dict) {
		a->dispose(PRVT->dict, 32768, a->user);
	}
	if (PRVT->cends) {
		a->dispose(PRVT->cends, PRVT->capcends * sizeof(uint64), a->user);
	}
	jdgpu_stream_destroy(PRVT->strm);
	a->dispose(PRVT, sizeof(struct TDEFLTPrvt), a->user);
}

void
deflator_reset(TDeflator* state)
{
	CTB_ASSERT(state);
	PBLC->state = 0;
	PBLC->flush = 0;
	PBLC->error = 0;
	PBLC->status = 0;
	PBLC->source = NULL;
	PBLC->target = NULL;
	PBLC->sbgn = NULL;
	PBLC->send = NULL;
	PBLC->tbgn = NULL;
	PBLC->tend = NULL;

	PRVT->used = 0;
	PRVT->closing = 0;
	PRVT->dictlen = 0;
	PRVT->ncends = 0;
	jdgpu_stream_destroy(PRVT->strm);
	PRVT->strm = NULL;
	PRVT->inlen = 0;
	PRVT->outlen = 0;
	PRVT->outpos = 0;
}

/* deflator_setdctnr :2106-2167.  With DEFLT_SINGLEWINDOW the dictionary's
 * last 32 KiB prime the window of the stream (jdgpu_deflate_stream_dict);
 * independent blocks cannot depend on bytes outside them, so in the default
 * mode the call is rejected as misuse. */
void
deflator_setdctnr(TDeflator* state, const uint8* dict, uintxx size)
{
	CTB_ASSERT(state && dict && size);
	if (PRVT->level == 0) {
		return;
	}
	if (PRVT->used || !PRVT->swin) {
		PBLC->error = DEFLT_EINCORRECTUSE;
		PBLC->state = 0xDEADBEEF;
		return;
	}
	if (PRVT->dict == NULL) {
		PRVT->dict = PRVT->allctr->request(32768, PRVT->allctr->user);
		if (PRVT->dict == NULL) {
			PBLC->error = DEFLT_EOOM;
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

void
jd_deflator_checksums(TDeflator* state, uint32* crc, uint32* adler)
{
	PRVT->crc = crc;
	PRVT->adler = adler;
}

/* validate :664-688 */
static int
validate(struct TDEFLTPrvt* state)
{
	if (PBLC->source == NULL || PBLC->target == NULL) {
		PBLC->error = DEFLT_EINCORRECTUSE;
		return 0;
	}
	switch (PBLC->status) {
		case DEFLT_SRCEXHSTD:
			if (PBLC->source == PBLC->send && PBLC->flush == 0) {
				PBLC->error = DEFLT_EINCORRECTUSE;
				return 0;
			}
			break;
		case DEFLT_TGTEXHSTD:
			if (PBLC->target == PBLC->tend) {
				PBLC->error = DEFLT_EINCORRECTUSE;
				return 0;
			}
			break;
	}
	return 1;
}

/* grow a buffer through the instance's allocator, keeping `keep` bytes */
static int
grow(struct TDEFLTPrvt* state, uint8** buf, uintxx* cap, uintxx need, uintxx keep)
{
	const struct TAllocator* a = PRVT->allctr;
	uintxx ncap = *cap;
	uint8* nb;

	if (need <= *cap) {
		return 1;
	}
	while (ncap < need) {
		ncap = ncap * 2;
	}
	nb = a->request(ncap, a->user);
	if (nb == NULL) {
		return 0;
	}
	if (keep) {
		memcpy(nb, *buf, keep);
	}
	a->dispose(*buf, *cap, a->user);
	*buf = nb;
	*cap = ncap;
	return 1;
}

/* single window: the pending input ends a reference call here */
static int
addcallend(struct TDEFLTPrvt* state)
{
	if (PRVT->ncends && PRVT->cends[PRVT->ncends - 1] == PRVT->inlen) {
		return 1;
	}
	if (PRVT->ncends == PRVT->capcends) {
		const struct TAllocator* a = PRVT->allctr;
		const uintxx ncap = PRVT->capcends ? PRVT->capcends * 2 : 64;
		uint64* nb = a->request(ncap * sizeof(uint64), a->user);
		if (nb == NULL) {
			PBLC->error = DEFLT_EOOM;
			return 0;
		}
		if (PRVT->ncends) {
			memcpy(nb, PRVT->cends, PRVT->ncends * sizeof(uint64));
		}
		if (PRVT->cends) {
			a->dispose(PRVT->cends, PRVT->capcends * sizeof(uint64), a->user);
		}
		PRVT->cends = nb;
		PRVT->capcends = ncap;
	}
	PRVT->cends[PRVT->ncends++] = PRVT->inlen;
	return 1;
}

/* compress the pending input; `last` = flush mode of its last block */
static int
compressbatch(struct TDEFLTPrvt* state, int last)
{
	int64 r;

	if (PRVT->swin) {
		/* the piece since the last flush, continuing the stream */
		if (!grow(PRVT, &PRVT->outbuf, &PRVT->outcap,
		          (uintxx) jdgpu_stream_bound(PRVT->inlen) + 16, 0)) {
			PBLC->error = DEFLT_EOOM;
			return 0;
		}
		if (PRVT->strm == NULL) {
			PRVT->strm = jdgpu_stream_create((int) PRVT->level, PBLC->flags & DEFLT_FIXEDCODES,
			                                 PRVT->dictlen ? PRVT->dict : NULL, PRVT->dictlen);
			if (PRVT->strm == NULL) {
				PBLC->error = DEFLT_EOOM;
				return 0;
			}
			PRVT->dictlen = 0;
		}
		if (!addcallend(PRVT)) {
			return 0;
		}
		r = jdgpu_stream_deflate(PRVT->strm, PRVT->inbuf, PRVT->inlen, PRVT->cends,
		                         (uint32) PRVT->ncends, last, PRVT->outbuf, PRVT->outcap);
		PRVT->ncends = 0;
	} else {
		if (!grow(PRVT, &PRVT->outbuf, &PRVT->outcap, outcap_for(PRVT->inlen), 0)) {
			PBLC->error = DEFLT_EOOM;
			return 0;
		}
		r = jdgpu_deflate_cs(PRVT->inbuf, PRVT->inlen, JD_BLOCKSIZE, PRVT->level,
		                     PBLC->flags & DEFLT_FIXEDCODES, last, PRVT->outbuf,
		                     PRVT->outcap, NULL, PRVT->crc, PRVT->adler);
	}
	if (r < 0) {
		PBLC->error = r == JDGPU_EOOM ? DEFLT_EOOM : DEFLT_EBADSTATE;
		return 0;
	}
	PRVT->inlen = 0;
	PRVT->outlen = (uintxx) r;
	PRVT->outpos = 0;
	return 1;
}

/* compress src[0, n) of the caller's buffer (no pending input); `last` =
 * flush mode of its last block */
static int
compressdirect(struct TDEFLTPrvt* state, const uint8* src, uintxx n, int last)
{
	const uintxx need = outcap_for(n);
	const uintxx room = (uintxx) (PBLC->tend - PBLC->target);
	uint8* dst = PRVT->outbuf;
	uintxx cap = PRVT->outcap;
	int64 r;

	if (room >= need) {
		dst = PBLC->target;
		cap = room;
	}
	else if (!grow(PRVT, &PRVT->outbuf, &PRVT->outcap, need, 0)) {
		PBLC->error = DEFLT_EOOM;
		return 0;
	}
	else {
		dst = PRVT->outbuf;
		cap = PRVT->outcap;
	}
	r = jdgpu_deflate_cs(src, n, JD_BLOCKSIZE, PRVT->level, PBLC->flags & DEFLT_FIXEDCODES, last,
	                     dst, cap, NULL, PRVT->crc, PRVT->adler);
	if (r < 0) {
		PBLC->error = r == JDGPU_EOOM ? DEFLT_EOOM : DEFLT_EBADSTATE;
		return 0;
	}
	if (dst == PBLC->target) {
		PBLC->target += (uintxx) r;
		PRVT->outlen = PRVT->outpos = 0;
	}
	else {
		PRVT->outlen = (uintxx) r;
		PRVT->outpos = 0;
	}
	return 1;
}

/* copy pending output to the target; 1 when everything was delivered */
static int
drain(struct TDEFLTPrvt* state)
{
	uintxx n = PRVT->outlen - PRVT->outpos;
	uintxx room = (uintxx) (PBLC->tend - PBLC->target);

	if (n > room) {
		n = room;
	}
	memcpy(PBLC->target, PRVT->outbuf + PRVT->outpos, n);
	PBLC->target += n;
	PRVT->outpos += n;
	return PRVT->outpos == PRVT->outlen;
}

eDEFLTResult
deflator_deflate(TDeflator* state, eDEFLTFlush flush)
{
	CTB_ASSERT(state);

	if (PBLC->state == 0xDEADBEEF) {
		return DEFLT_ERROR;
	}
	if (flush && (PBLC->flush == 0 || PBLC->flush == DEFLT_FLUSH)) {
		PBLC->flush = flush;
	}
	if (validate(PRVT) == 0) {
		PBLC->state = 0xDEADBEEF;
		return DEFLT_ERROR;
	}
	PRVT->used = 1;

	for (;;) {
		uintxx take;

		if (!drain(PRVT)) {
			return (eDEFLTResult) (PBLC->status = DEFLT_TGTEXHSTD);
		}
		if (PRVT->closing) {
			/* the flush has been delivered (endstream :758-773) */
			PRVT->closing = 0;
			if (PBLC->flush == DEFLT_FLUSH) {
				PBLC->state = 0;
				PBLC->flush = 0;
			} else {
				PBLC->state = 0xDEADBEEF;
			}
			return (eDEFLTResult) (PBLC->status = DEFLT_OK);
		}

		/* nothing pending: whole blocks of the caller's buffer are
		 * compressed where they lie (no copy), straight into the target
		 * when it has room for the worst case */
		if (!PRVT->swin && PRVT->inlen == 0) {
			const uintxx avail = (uintxx) (PBLC->send - PBLC->source);
			uintxx k;
			int last;

			if (PBLC->flush && avail <= JD_BATCH) {
				k = avail;                  /* the rest, ending with the flush */
			} else {
				/* more input follows these blocks (or may follow:
				 * without a flush the last block is kept back) */
				k = avail > JD_BATCH ? JD_BATCH : (avail ? (avail - 1) / JD_BLOCKSIZE * JD_BLOCKSIZE : 0);
			}
			if (k >= JD_BLOCKSIZE || (PBLC->flush && k == avail)) {
				last = (PBLC->flush && k == avail) ? (int) PBLC->flush : DEFLT_FLUSH;
				if (!compressdirect(PRVT, PBLC->source, k, last)) {
					PBLC->state = 0xDEADBEEF;
					return DEFLT_ERROR;
				}
				PBLC->source += k;
				if (PBLC->flush && PBLC->source == PBLC->send) {
					PRVT->closing = 1;
				}
				continue;
			}
		}

		/* gather input; a full batch with more input behind it is
		 * certainly not the end of the stream */
		take = (uintxx) (PBLC->send - PBLC->source);
		if (PRVT->swin) {
			/* single window: the segment is kept whole until its flush */
			if (!grow(PRVT, &PRVT->inbuf, &PRVT->incap, PRVT->inlen + take,
			          PRVT->inlen)) {
				PBLC->error = DEFLT_EOOM;
				PBLC->state = 0xDEADBEEF;
				return DEFLT_ERROR;
			}
		} else {
			if (take > PRVT->incap - PRVT->inlen && PRVT->incap < JD_BATCH) {
				uintxx want = PRVT->inlen + take < JD_BATCH ? PRVT->inlen + take : JD_BATCH;
				if (!grow(PRVT, &PRVT->inbuf, &PRVT->incap, want, PRVT->inlen)) {
					PBLC->error = DEFLT_EOOM;
					PBLC->state = 0xDEADBEEF;
					return DEFLT_ERROR;
				}
			}
			if (take > PRVT->incap - PRVT->inlen) {
				take = PRVT->incap - PRVT->inlen;
			}
		}
		memcpy(PRVT->inbuf + PRVT->inlen, PBLC->source, take);
		PRVT->inlen += take;
		PBLC->source += take;

		if (!PRVT->swin && PRVT->inlen == PRVT->incap && PBLC->source < PBLC->send) {
			if (!compressbatch(PRVT, DEFLT_FLUSH)) {
				PBLC->state = 0xDEADBEEF;
				return DEFLT_ERROR;
			}
			continue;
		}
		if (PBLC->source < PBLC->send) {
			continue;
		}
		if (PBLC->flush == 0) {
			/* the reference's call would end here, its input consumed */
			if (PRVT->swin && !addcallend(PRVT)) {
				PBLC->state = 0xDEADBEEF;
				return DEFLT_ERROR;
			}
			return (eDEFLTResult) (PBLC->status = DEFLT_SRCEXHSTD);
		}
		if (!compressbatch(PRVT, (int) PBLC->flush)) {
			PBLC->state = 0xDEADBEEF;
			return DEFLT_ERROR;
		}
		PRVT->closing = 1;
	}
}
