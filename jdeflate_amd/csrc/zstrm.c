/*
 * zstrm.c -- drop-in zstrm_* container API (jdeflate/zstrm.h) over the
 * MI355X engine: raw deflate, zlib and gzip framing; CRC-32 and Adler-32
 * computed by k_checksum on the device copy of the data.
 *
 * The state machine, error codes, flag handling and header parsing follow
 * the reference zstrm.c: zstrm_create :81-172, reset :197-241, setsource /
 * setsourcefn / settargetfn :248-308, setdctnr :327-390, the header parsers
 * :446-624, the trailer checks :626-696, zstrm_inflate :701-773, the header
 * writers :1003-1053, zstrm_deflate :1061-1110, trailers and flush
 * :1233-1318.  The engine differs underneath:
 *  - deflate gathers input into 16 MiB batches of 64 KiB independent blocks
 *    (FLUSH-terminated; the last block of a final flush ends the stream) and
 *    compresses each batch in one GPU launch sequence, scanning the batch's
 *    checksums on the device in the same call;
 *  - inflate collects the container (the source buffer, or the source
 *    callback read to its end), decodes the deflate stream on the GPU
 *    (jdgpu_inflate_stream_cs, checksums scanned where the bytes were
 *    decoded) and delivers it across zstrm_inflate calls; the trailer is
 *    checked when the caller asks past the end, as in the reference.
 * Deliberate differences are listed in include/jdeflate/zstrm.h.
 */
#include <jdeflate/zstrm.h>
#include <jdeflate/jdgpu.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define IOBFFRSIZE 32768u                   /* zstrm.c:20                    */
#define ZS_BLOCK   65536u
#define ZS_BATCH   (16u << 20)
#define ZS_MAXOUT  0xfffffff0ull            /* single-stream decoder limit   */

#define ZSTRM_MODEMASK 0x000f0000u
#define ZSTRM_TYPEMASK 0x00f00000u

typedef intxx (*TZStrmIOFn)(uint8*, uintxx, void*);

struct TZStrmPrvt {
	struct TZStrm public;

	TZStrmIOFn iofn;
	void* user;

	/* buffer source (inflate) */
	const uint8* input;
	const uint8* inputend;

	uint32 docrc;
	uint32 doadler;

	/* deflate: pending input of the current batch, compressed batch */
	int32 dflags;
	uint8* inbuf;
	uintxx inlen;
	uintxx incap;
	uint8* outbuf;
	uintxx outcap;

	/* inflate: read window (header / trailer parsing) */
	const uint8* sbgn;
	const uint8* send;
	uint32 eof;            /* the source callback returned 0            */
	uintxx pulled;         /* bytes the source callback delivered       */
	uintxx hdrlen;         /* container bytes before the deflate stream */
	/* inflate: collected container bytes after the header (callback mode) */
	uint8* cin;
	uintxx cinlen;
	uintxx cincap;
	/* inflate: decoded bytes and the delivery cursor */
	uint32 decoded;
	int32 decerr;
	uint8* dec;
	uintxx deccap;
	uintxx declen;
	uintxx decpos;
	/* preset dictionary (zstrm_setdctnr): its last 32 KiB */
	uint8 zdict[32768];
	uintxx zdictlen;
	const uint8* body;     /* deflate stream + trailer                  */
	uintxx bodylen;
	uintxx consumed;       /* bytes of the deflate stream               */

	const struct TAllocator* allctr;

	uint8 iobuffer[IOBFFRSIZE];
};

#define SETERROR(ERROR) (zstrm->public.error = (ERROR))
#define SETSTATE(STATE) (zstrm->public.state = (STATE))
#define ZPRVT(S) ((struct TZStrmPrvt*) (uintptr_t) (S))

static void* zs_request(uintxx size, void* user) { (void) user; return malloc(size); }
static void zs_dispose(void* p, uintxx size, void* user) { (void) size; (void) user; free(p); }
static const struct TAllocator zs_defaultallocator = { zs_request, zs_dispose, NULL };

/* grow *buf (capacity *cap) to hold at least need bytes, keeping len bytes */
static int zs_grow(struct TZStrmPrvt* zstrm, uint8** buf, uintxx* cap, uintxx len, uintxx need)
{
	uintxx ncap;
	uint8* nb;

	if (need <= *cap) {
		return 1;
	}
	ncap = *cap ? *cap : 65536;
	while (ncap < need) {
		ncap *= 2;
	}
	nb = zstrm->allctr->request(ncap, zstrm->allctr->user);
	if (nb == NULL) {
		return 0;
	}
	if (len) {
		memcpy(nb, *buf, len);
	}
	if (*buf) {
		zstrm->allctr->dispose(*buf, *cap, zstrm->allctr->user);
	}
	*buf = nb;
	*cap = ncap;
	return 1;
}

static void zs_free(struct TZStrmPrvt* zstrm, uint8** buf, uintxx* cap)
{
	if (*buf) {
		zstrm->allctr->dispose(*buf, *cap, zstrm->allctr->user);
	}
	*buf = NULL;
	*cap = 0;
}

const TZStrm*
zstrm_create(uintxx flags, intxx level, const TAllocator* allctr)
{
	uint32 smode;
	uint32 stype;
	struct TZStrmPrvt* zstrm;

	smode = (uint32) (flags & ZSTRM_MODEMASK);
	stype = (uint32) (flags & ZSTRM_TYPEMASK);
	if (smode != ZSTRM_INFLATE && smode != ZSTRM_DEFLATE) {
		return NULL;
	}
	if (stype == 0) {
		if (smode == ZSTRM_DEFLATE) {
			return NULL;
		}
		flags |= (stype = ZSTRM_DFLT | ZSTRM_ZLIB | ZSTRM_GZIP);
	}
	if (smode == ZSTRM_DEFLATE) {
		uintxx invalid;

		if (level > 9 || level < 0) {
			return NULL;
		}
		invalid = 0;
		invalid |= ((stype & ZSTRM_DFLT) && (stype & ~((uint32) ZSTRM_DFLT)));
		invalid |= ((stype & ZSTRM_ZLIB) && (stype & ~((uint32) ZSTRM_ZLIB)));
		invalid |= ((stype & ZSTRM_GZIP) && (stype & ~((uint32) ZSTRM_GZIP)));
		if (invalid) {
			return NULL;
		}
	}
	if (!jdgpu_available()) {
		return NULL;
	}
	if (allctr == NULL) {
		allctr = &zs_defaultallocator;
	}

	zstrm = allctr->request(sizeof(struct TZStrmPrvt), allctr->user);
	if (zstrm == NULL) {
		return NULL;
	}
	memset(zstrm, 0, sizeof(struct TZStrmPrvt));
	zstrm->allctr = allctr;

	zstrm->public.smode = smode;
	if (smode == ZSTRM_DEFLATE) {
		zstrm->public.stype = stype;
		zstrm->public.level = (int32) level;
		zstrm->dflags = (int32) (flags & 0x00ff);

		zstrm->doadler = (flags & ZSTRM_DOADLER) != 0;
		zstrm->docrc   = (flags & ZSTRM_DOCRC  ) != 0;
		if (stype == ZSTRM_ZLIB) {
			zstrm->doadler = 1;
		}
		if (stype == ZSTRM_GZIP) {
			zstrm->docrc = 1;
		}
	}
	zstrm->public.flags = (uint32) flags;
	zstrm_reset(&zstrm->public);
	return &zstrm->public;
}

void
zstrm_destroy(const TZStrm* state)
{
	struct TZStrmPrvt* zstrm;

	if (state == NULL) {
		return;
	}
	zstrm = ZPRVT(state);
	zs_free(zstrm, &zstrm->inbuf, &zstrm->incap);
	zs_free(zstrm, &zstrm->outbuf, &zstrm->outcap);
	zs_free(zstrm, &zstrm->cin, &zstrm->cincap);
	zs_free(zstrm, &zstrm->dec, &zstrm->deccap);
	zstrm->allctr->dispose(zstrm, sizeof(struct TZStrmPrvt), zstrm->allctr->user);
}

void
zstrm_reset(const TZStrm* state)
{
	struct TZStrmPrvt* zstrm;

	if (state == NULL) {
		return;
	}
	zstrm = ZPRVT(state);
	zstrm->public.state = 0;
	zstrm->public.error = 0;
	if (zstrm->public.smode == ZSTRM_INFLATE) {
		zstrm->public.stype = 0;
		zstrm->doadler = (zstrm->public.flags & ZSTRM_DOADLER) != 0;
		zstrm->docrc   = (zstrm->public.flags & ZSTRM_DOCRC  ) != 0;
	}
	zstrm->public.dictid = 0;
	zstrm->public.dict   = 0;
	zstrm->zdictlen = 0;
	zstrm->public.crc    = 0xffffffffu;
	zstrm->public.adler  = 1u;
	zstrm->public.total  = 0;
	zstrm->public.usedinput = 0;

	zstrm->iofn = NULL;
	zstrm->user = NULL;
	zstrm->input = NULL;
	zstrm->inputend = NULL;
	zstrm->sbgn = NULL;
	zstrm->send = NULL;
	zstrm->eof = 0;
	zstrm->hdrlen = 0;
	zstrm->cinlen = 0;
	zstrm->decoded = 0;
	zstrm->decerr = 0;
	zstrm->declen = 0;
	zstrm->decpos = 0;
	zstrm->body = NULL;
	zstrm->bodylen = 0;
	zstrm->consumed = 0;
	zstrm->pulled = 0;
	/* the batch buffer keeps its allocation; inlen is its fill level */
	zstrm->inlen = 0;
}

static void
badusage(struct TZStrmPrvt* zstrm)
{
	SETSTATE(ZSTRM_END);
	if (zstrm->public.error == 0) {
		SETERROR(ZSTRM_EINCORRECTUSE);
	}
}

void
zstrm_setsource(const TZStrm* state, const uint8* source, uintxx size)
{
	uint8 t[1];
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.smode != ZSTRM_INFLATE || zstrm->public.state) {
		badusage(zstrm);
		return;
	}
	SETSTATE(1);
	zstrm->input = source;
	zstrm->inputend = source + size;
	zstrm_inflate(state, t, 0);
}

void
zstrm_setsourcefn(const TZStrm* state, TZStrmIFn fn, void* user)
{
	uint8 t[1];
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.smode != ZSTRM_INFLATE || zstrm->public.state) {
		badusage(zstrm);
		return;
	}
	SETSTATE(1);
	zstrm->user = user;
	zstrm->iofn = (TZStrmIOFn) fn;
	zstrm_inflate(state, t, 0);
}

void
zstrm_settargetfn(const TZStrm* state, TZStrmOFn fn, void* user)
{
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.smode != ZSTRM_DEFLATE || zstrm->public.state) {
		badusage(zstrm);
		return;
	}
	SETSTATE(1);
	zstrm->user = user;
	zstrm->iofn = (TZStrmIOFn) (uintptr_t) fn;
}

/* ---- inflate ------------------------------------------------------------ */

/* next container byte (fetchbyte :411-444); 0 with the error set when the
 * source is exhausted */
static uint8
fetchbyte(struct TZStrmPrvt* zstrm)
{
	if (zstrm->public.error) {
		return 0;
	}
	if (zstrm->sbgn < zstrm->send) {
		return *zstrm->sbgn++;
	}
	if (zstrm->iofn && !zstrm->eof) {
		intxx n;

		n = zstrm->iofn(zstrm->iobuffer, IOBFFRSIZE, zstrm->user);
		if (n != 0) {
			if ((uintxx) n > IOBFFRSIZE) {
				SETERROR(ZSTRM_EIOERROR);
				return 0;
			}
			zstrm->pulled += (uintxx) n;
			zstrm->sbgn = zstrm->iobuffer;
			zstrm->send = zstrm->iobuffer + n;
			return *zstrm->sbgn++;
		}
		zstrm->eof = 1;
	}
	else {
		if (zstrm->iofn == NULL) {
			SETERROR(ZSTRM_ESRCEXHSTD);
		}
	}
	if (zstrm->public.error == 0) {
		SETERROR(ZSTRM_EBADDATA);
	}
	return 0;
}

/* parsegziphead :446-509 */
static int
parsegziphead(struct TZStrmPrvt* zstrm)
{
	uint32 id1, id2, flags;

	id1 = fetchbyte(zstrm);
	id2 = fetchbyte(zstrm);
	if (id1 != 0x1f || id2 != 0x8b) {
		if (zstrm->public.error == 0) {
			SETERROR(ZSTRM_EBADDATA);
		}
		return 0;
	}
	if (fetchbyte(zstrm) != 0x08) {
		if (zstrm->public.error == 0) {
			SETERROR(ZSTRM_EBADDATA);
		}
		return 0;
	}
	flags = fetchbyte(zstrm);
	/* MTIME, XFL, OS */
	fetchbyte(zstrm); fetchbyte(zstrm); fetchbyte(zstrm);
	fetchbyte(zstrm); fetchbyte(zstrm); fetchbyte(zstrm);
	if (flags & 0x04) {
		uint32 a, b, length;

		a = fetchbyte(zstrm);
		b = fetchbyte(zstrm);
		for (length = a | (b << 8); length && zstrm->public.error == 0; length--) {
			fetchbyte(zstrm);
		}
	}
	if (flags & 0x08) {
		while (fetchbyte(zstrm));
	}
	if (flags & 0x10) {
		while (fetchbyte(zstrm));
	}
	if (flags & 0x02) {
		fetchbyte(zstrm);
		fetchbyte(zstrm);
	}
	return zstrm->public.error == 0;
}

#define TOI32(A, B, C, D)  ((A) | ((B) << 0x08) | ((C) << 0x10) | ((D) << 0x18))

/* parsezlibhead :513-565 (FCHECK is not verified, as in the reference) */
static int
parsezlibhead(struct TZStrmPrvt* zstrm)
{
	uint32 a, b;

	a = fetchbyte(zstrm);
	b = fetchbyte(zstrm);
	if (zstrm->public.error) {
		return 0;
	}
	if ((a & 0x0f) == 8 && ((a >> 4) & 0x0f) <= 7) {
		if ((b >> 5) & 1) {
			uint32 c, d;

			d = fetchbyte(zstrm);
			c = fetchbyte(zstrm);
			b = fetchbyte(zstrm);
			a = fetchbyte(zstrm);
			if (zstrm->public.error) {
				return 0;
			}
			zstrm->public.dictid = TOI32(a, b, c, d);
			SETSTATE(2);
		}
		return 1;
	}
	if (zstrm->public.error == 0) {
		SETERROR(ZSTRM_EBADDATA);
	}
	return 0;
}

/* parsehead :567-624 */
static int
parsehead(struct TZStrmPrvt* zstrm)
{
	uint32 stype, head;

	head = fetchbyte(zstrm);
	if (zstrm->public.error) {
		return 0;
	}
	if (head == 0x1f) {
		stype = ZSTRM_GZIP;
	}
	else {
		if ((head & 0x0f) == 0x08) {
			stype = ZSTRM_ZLIB;
		}
		else {
			head = head & 0x07;
			if (head == 0x06 || head == 0x07) {
				/* block type 11 (reserved) */
				SETERROR(ZSTRM_EBADDATA);
				return 0;
			}
			stype = ZSTRM_DFLT;
		}
	}
	if ((zstrm->public.flags & stype) == 0) {
		SETERROR(ZSTRM_EFORMAT);
		return 0;
	}
	zstrm->public.stype = stype;

	zstrm->sbgn--;
	switch (stype) {
		case ZSTRM_GZIP: zstrm->docrc   = 1; parsegziphead(zstrm); break;
		case ZSTRM_ZLIB: zstrm->doadler = 1; parsezlibhead(zstrm); break;
		default:
			break;
	}
	if (zstrm->public.error) {
		return 0;
	}
	if (zstrm->public.flags & ZSTRM_NOADLER) {
		zstrm->doadler = 0;
	}
	if (zstrm->public.flags & ZSTRM_NOCRC) {
		zstrm->docrc = 0;
	}
	/* header bytes: fetched from the source less what is left unread */
	if (zstrm->iofn == NULL) {
		zstrm->hdrlen = (uintxx) (zstrm->sbgn - zstrm->input);
	}
	else {
		zstrm->hdrlen = zstrm->pulled - (uintxx) (zstrm->send - zstrm->sbgn);
	}
	return 1;
}

/* the container bytes after the header: the source buffer's remainder, or
 * everything the callback delivers until it returns 0 */
static int
collect(struct TZStrmPrvt* zstrm)
{
	if (zstrm->iofn == NULL) {
		zstrm->body = zstrm->sbgn;
		zstrm->bodylen = (uintxx) (zstrm->send - zstrm->sbgn);
		return 1;
	}
	zstrm->cinlen = 0;
	if (zstrm->send > zstrm->sbgn) {
		uintxx k = (uintxx) (zstrm->send - zstrm->sbgn);
		if (!zs_grow(zstrm, &zstrm->cin, &zstrm->cincap, 0, k)) {
			SETERROR(ZSTRM_EOOM);
			return 0;
		}
		memcpy(zstrm->cin, zstrm->sbgn, k);
		zstrm->cinlen = k;
	}
	while (!zstrm->eof) {
		intxx r;

		if (!zs_grow(zstrm, &zstrm->cin, &zstrm->cincap, zstrm->cinlen, zstrm->cinlen + IOBFFRSIZE)) {
			SETERROR(ZSTRM_EOOM);
			return 0;
		}
		r = zstrm->iofn(zstrm->cin + zstrm->cinlen, IOBFFRSIZE, zstrm->user);
		if (r == 0) {
			zstrm->eof = 1;
			break;
		}
		if ((uintxx) r > IOBFFRSIZE) {
			SETERROR(ZSTRM_EIOERROR);
			return 0;
		}
		zstrm->cinlen += (uintxx) r;
	}
	zstrm->body = zstrm->cin;
	zstrm->bodylen = zstrm->cinlen;
	return 1;
}

/* decode the whole deflate stream on the GPU; the checksums of the decoded
 * bytes are scanned on the device */
static int
decodeall(struct TZStrmPrvt* zstrm)
{
	uint64 cap, produced, used;
	uintxx tail;
	int32 err;
	int r;

	if (!collect(zstrm)) {
		return 0;
	}
	if (zstrm->bodylen > 0xffffffffu) {
		SETERROR(ZSTRM_ELIMIT);
		return 0;
	}
	/* the container trailer after the deflate stream */
	tail = zstrm->public.stype == ZSTRM_GZIP ? 8 : zstrm->public.stype == ZSTRM_ZLIB ? 4 : 0;
	if (tail > zstrm->bodylen) {
		tail = 0;
	}
	/* first capacity guess: gzip's ISIZE (mod 2^32), else 4x the input */
	cap = (uint64) zstrm->bodylen * 4 + 65536;
	if (zstrm->public.stype == ZSTRM_GZIP && zstrm->bodylen >= 8) {
		const uint8* t = zstrm->body + zstrm->bodylen - 4;
		uint64 isz = (uint64) TOI32((uint32) t[0], (uint32) t[1], (uint32) t[2], (uint32) t[3]);
		/* a corrupt trailer must not size the buffer: deflate expands at
		 * most ~1032:1 */
		if (isz + 64 > cap && isz <= (uint64) zstrm->bodylen * 1032) {
			cap = isz + 64;
		}
	}
	for (;;) {
		uint32 crc, adler;

		if (cap > ZS_MAXOUT) {
			cap = ZS_MAXOUT;
		}
		if (!zs_grow(zstrm, &zstrm->dec, &zstrm->deccap, 0, (uintxx) cap)) {
			SETERROR(ZSTRM_EOOM);
			return 0;
		}
		crc = zstrm->public.crc;
		adler = zstrm->public.adler;
		/* FLUSH-joined independent blocks (what this library writes) are
		 * found at their sync markers and decoded in parallel; any other
		 * stream is decoded serially */
		if (zstrm->zdictlen) {
			/* references may reach into the dictionary: one serial stream */
			r = jdgpu_inflate_stream_dict(zstrm->zdict, zstrm->zdictlen, zstrm->body,
			                              zstrm->bodylen, zstrm->dec, cap, &produced, &used,
			                              &err);
			if (!r && err != JDGPU_EBLOCKOVERFLOW && produced && (zstrm->docrc || zstrm->doadler))
				r = jdgpu_checksum(zstrm->dec, produced, zstrm->docrc ? &crc : NULL,
				                   zstrm->doadler ? &adler : NULL);
		}
		else {
			r = jdgpu_inflate_flushed(zstrm->body, zstrm->bodylen, zstrm->bodylen - tail,
			                          zstrm->dec, cap, &produced, &used, &err,
			                          zstrm->docrc ? &crc : NULL,
			                          zstrm->doadler ? &adler : NULL);
		}
		if (r) {
			SETERROR(r == JDGPU_EOOM ? ZSTRM_EOOM : ZSTRM_EDEFLATE);
			return 0;
		}
		if (err == JDGPU_EBLOCKOVERFLOW) {
			if (cap >= ZS_MAXOUT) {
				SETERROR(ZSTRM_ELIMIT);
				return 0;
			}
			cap *= 2;
			continue;
		}
		zstrm->public.crc = crc;
		zstrm->public.adler = adler;
		break;
	}
	zstrm->decoded = 1;
	zstrm->decerr = err;
	zstrm->declen = (uintxx) produced;
	zstrm->decpos = 0;
	zstrm->consumed = (uintxx) used;
	return 1;
}

/* checkgziptail :626-668 */
static void
checkgziptail(struct TZStrmPrvt* zstrm)
{
	uint32 a, b, c, d, crc, total;

	a = fetchbyte(zstrm); b = fetchbyte(zstrm);
	c = fetchbyte(zstrm); d = fetchbyte(zstrm);
	crc = TOI32(a, b, c, d);
	if (zstrm->public.error) {
		return;
	}
	if (zstrm->docrc == 1 && crc != zstrm->public.crc) {
		SETERROR(ZSTRM_ECHECKSUM);
		return;
	}
	a = fetchbyte(zstrm); b = fetchbyte(zstrm);
	c = fetchbyte(zstrm); d = fetchbyte(zstrm);
	total = TOI32(a, b, c, d);
	if (total != (uint32) zstrm->public.total) {
		if (zstrm->public.error) {
			return;
		}
		SETERROR(ZSTRM_EBADDATA);
	}
}

/* checkzlibtail :670-696 */
static void
checkzlibtail(struct TZStrmPrvt* zstrm)
{
	uint32 a, b, c, d, adler;

	d = fetchbyte(zstrm); c = fetchbyte(zstrm);
	b = fetchbyte(zstrm); a = fetchbyte(zstrm);
	adler = TOI32(a, b, c, d);
	if (zstrm->public.error == 0 && zstrm->doadler == 1 && adler != zstrm->public.adler) {
		SETERROR(ZSTRM_ECHECKSUM);
	}
}

#undef TOI32

static uintxx
inflate(struct TZStrmPrvt* zstrm, uint8* buffer, uintxx total)
{
	uintxx n, k;

	if (!zstrm->decoded && !decodeall(zstrm)) {
		SETSTATE(4);
		return 0;
	}
	n = 0;
	k = zstrm->declen - zstrm->decpos;
	if (k > total) {
		k = total;
	}
	if (k) {
		memcpy(buffer, zstrm->dec + zstrm->decpos, k);
		zstrm->decpos += k;
		n = k;
	}
	zstrm->public.total += n;
	if (n == total) {
		return n;
	}
	/* asked past the decoded bytes: the end of the stream (:903-935) */
	if (zstrm->decerr) {
		SETERROR(ZSTRM_EDEFLATE);
		SETSTATE(4);
		return n;
	}
	if (zstrm->docrc) {
		zstrm->public.crc ^= 0xffffffffu;
	}
	zstrm->sbgn = zstrm->body + zstrm->consumed;
	zstrm->send = zstrm->body + zstrm->bodylen;
	switch (zstrm->public.stype) {
		case ZSTRM_GZIP: checkgziptail(zstrm); break;
		case ZSTRM_ZLIB: checkzlibtail(zstrm); break;
		default:
			break;
	}
	zstrm->public.usedinput = zstrm->hdrlen + (uintxx) (zstrm->sbgn - zstrm->body);
	SETSTATE(4);
	return n;
}

uintxx
zstrm_inflate(const TZStrm* state, void* target, uintxx n)
{
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.smode != ZSTRM_INFLATE) {
		badusage(zstrm);
		return 0;
	}
	if (zstrm->public.state == 3) {
		if (n > (((uintxx) 1) << 31) - 1) {
			SETSTATE(4);
			SETERROR(ZSTRM_ELIMIT);
			return 0;
		}
		return inflate(zstrm, (uint8*) target, n);
	}
	if (zstrm->public.state == 1) {
		if (zstrm->input) {
			zstrm->sbgn = zstrm->input;
			zstrm->send = zstrm->inputend;
		}
		if (parsehead(zstrm) == 0) {
			SETSTATE(4);
		}
		else {
			if (zstrm->public.state == 2) {
				/* n = 0 asks whether a dictionary is needed */
				if (n == 0) {
					return 0;
				}
				SETERROR(ZSTRM_EMISSINGDICT);
			}
		}
		if (zstrm->public.error) {
			SETSTATE(4);
			return 0;
		}
		SETSTATE(3);
		if (n != 0) {
			return inflate(zstrm, (uint8*) target, n);
		}
	}
	else {
		if (zstrm->public.state == 2) {
			SETERROR(ZSTRM_EMISSINGDICT);
			SETSTATE(4);
		}
	}
	return 0;
}

static void
keepdict(struct TZStrmPrvt* zstrm, const uint8* dict, uintxx size)
{
	if (size > sizeof(zstrm->zdict)) {
		dict = (dict + size) - sizeof(zstrm->zdict);
		size = sizeof(zstrm->zdict);
	}
	memcpy(zstrm->zdict, dict, size);
	zstrm->zdictlen = size;
}

/* zstrm_setdctnr :327-390.  Inflate: the dictionary primes the stream
 * decoder's window (inflator_setdctnr).  Deflate (zlib): FDICT and DICTID go
 * into the header; the independent blocks never reach before their start,
 * so the stream decodes with the dictionary but does not use it (the
 * reference's stream would reference it). */
void
zstrm_setdctnr(const TZStrm* state, const uint8* dict, uintxx size)
{
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.state == 0 || zstrm->public.state == 4 || dict == NULL || size == 0) {
		badusage(zstrm);
		return;
	}
	if (zstrm->public.smode == ZSTRM_INFLATE) {
		if (zstrm->public.state == 1) {
			if (zstrm->input) {
				zstrm->sbgn = zstrm->input;
				zstrm->send = zstrm->inputend;
			}
			if (parsehead(zstrm) == 0) {
				badusage(zstrm);
				return;
			}
		}
		if (zstrm->public.stype == ZSTRM_GZIP) {
			badusage(zstrm);
			return;
		}
		if (zstrm->public.state == 2) {
			uint32 adler = zstrm_adler32update(1, dict, size);
			if (adler != zstrm->public.dictid) {
				SETERROR(ZSTRM_EBADDICT);
				badusage(zstrm);
				return;
			}
		}
		else if (zstrm->public.state == 3) {
			badusage(zstrm);
			return;
		}
		SETSTATE(3);
		keepdict(zstrm, dict, size);
		return;
	}
	if (zstrm->public.state != 1 || (zstrm->public.stype & ZSTRM_GZIP) || zstrm->public.dict == 1) {
		badusage(zstrm);
		return;
	}
	zstrm->public.dictid = zstrm_adler32update(1, dict, size);
	zstrm->public.dict = 1;
	keepdict(zstrm, dict, size);
}

/* ---- deflate ------------------------------------------------------------ */

static void
emit(struct TZStrmPrvt* zstrm, const uint8* p, uintxx n)
{
	while (n && zstrm->public.error == 0) {
		uintxx k = n < IOBFFRSIZE ? n : IOBFFRSIZE;
		intxx r = zstrm->iofn((uint8*) (uintptr_t) p, k, zstrm->user);
		if ((uintxx) r != k) {
			SETERROR(ZSTRM_EIOERROR);
			return;
		}
		p += k;
		n -= k;
	}
}

/* emitgziphead :1003-1022 */
static void
emitgziphead(struct TZStrmPrvt* zstrm)
{
	static const uint8 h[10] = { 0x1f, 0x8b, 0x08, 0, 0, 0, 0, 0, 0, 0 };
	emit(zstrm, h, 10);
}

/* emitzlibhead :1024-1053, with a valid FCHECK (the reference computes
 * `b + (31 - ((a << 8) | b % 31))` and writes 78 1F) */
static void
emitzlibhead(struct TZStrmPrvt* zstrm)
{
	uint8 h[6];
	uint32 a = 0x78, b = 0;
	uintxx k = 2;

	if (zstrm->public.dict) {
		b |= 1 << 5;
	}
	b += 31 - ((a << 8) | b) % 31;
	h[0] = (uint8) a;
	h[1] = (uint8) b;
	if (zstrm->public.dict) {
		uint32 id = zstrm->public.dictid;
		h[2] = (uint8) (id >> 24); h[3] = (uint8) (id >> 16);
		h[4] = (uint8) (id >> 8);  h[5] = (uint8) id;
		k = 6;
	}
	emit(zstrm, h, k);
}

/* compress the pending batch (flush: DEFLT_FLUSH or DEFLT_END), scanning
 * its checksums on the device, and hand the bytes to the target callback */
static void
dobatch(struct TZStrmPrvt* zstrm, int flush)
{
	uintxx need;
	int64 r;
	uint32 crc, adler;

	need = (uintxx) jdgpu_bound(zstrm->inlen, ZS_BLOCK);
	if (!zs_grow(zstrm, &zstrm->outbuf, &zstrm->outcap, 0, need)) {
		SETERROR(ZSTRM_EOOM);
		return;
	}
	crc = zstrm->public.crc;
	adler = zstrm->public.adler;
	r = jdgpu_deflate_cs(zstrm->inbuf, zstrm->inlen, ZS_BLOCK, zstrm->public.level,
	                     (uint32) zstrm->dflags, flush, zstrm->outbuf, zstrm->outcap, NULL,
	                     zstrm->docrc ? &crc : NULL, zstrm->doadler ? &adler : NULL);
	if (r < 0) {
		SETERROR(r == JDGPU_EOOM ? ZSTRM_EOOM : ZSTRM_EDEFLATE);
		return;
	}
	zstrm->public.crc = crc;
	zstrm->public.adler = adler;
	zstrm->inlen = 0;
	emit(zstrm, zstrm->outbuf, (uintxx) r);
}

static uintxx
deflate(struct TZStrmPrvt* zstrm, const uint8* buffer, uintxx total)
{
	uintxx done = 0;

	if (!zs_grow(zstrm, &zstrm->inbuf, &zstrm->incap, 0, ZS_BATCH)) {
		SETERROR(ZSTRM_EOOM);
		SETSTATE(4);
		return 0;
	}
	while (done < total) {
		uintxx k = ZS_BATCH - zstrm->inlen;
		if (k > total - done) {
			k = total - done;
		}
		memcpy(zstrm->inbuf + zstrm->inlen, buffer + done, k);
		zstrm->inlen += k;
		done += k;
		if (zstrm->inlen == ZS_BATCH) {
			dobatch(zstrm, DEFLT_FLUSH);
			if (zstrm->public.error) {
				SETSTATE(4);
				break;
			}
		}
	}
	return done;
}

uintxx
zstrm_deflate(const TZStrm* state, const void* source, uintxx n)
{
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.smode != ZSTRM_DEFLATE) {
		badusage(zstrm);
		return 0;
	}
	if (zstrm->public.state == 3) {
		uintxx r;

		if (n > (((uintxx) 1) << 31) - 1) {
			SETSTATE(4);
			SETERROR(ZSTRM_ELIMIT);
			return 0;
		}
		r = deflate(zstrm, (const uint8*) source, n);
		zstrm->public.total += r;
		return r;
	}
	if (zstrm->public.state == 1 || zstrm->public.state == 2) {
		switch (zstrm->public.stype) {
			case ZSTRM_GZIP: emitgziphead(zstrm); break;
			case ZSTRM_ZLIB: emitzlibhead(zstrm); break;
			default:
				break;
		}
		if (zstrm->public.error) {
			SETSTATE(4);
			return 0;
		}
		SETSTATE(3);
		return zstrm_deflate(state, source, n);
	}
	return 0;
}

/* emitgziptail :1233-1252 */
static void
emitgziptail(struct TZStrmPrvt* zstrm)
{
	uint8 t[8];
	uint32 c, n;

	zstrm->public.crc ^= 0xffffffffu;
	c = zstrm->public.crc;
	n = (uint32) zstrm->public.total;
	t[0] = (uint8) c; t[1] = (uint8) (c >> 8); t[2] = (uint8) (c >> 16); t[3] = (uint8) (c >> 24);
	t[4] = (uint8) n; t[5] = (uint8) (n >> 8); t[6] = (uint8) (n >> 16); t[7] = (uint8) (n >> 24);
	emit(zstrm, t, 8);
}

/* emitzlibtail :1254-1265 */
static void
emitzlibtail(struct TZStrmPrvt* zstrm)
{
	uint8 t[4];
	uint32 a = zstrm->public.adler;

	t[0] = (uint8) (a >> 24); t[1] = (uint8) (a >> 16); t[2] = (uint8) (a >> 8); t[3] = (uint8) a;
	emit(zstrm, t, 4);
}

void
zstrm_flush(const TZStrm* state, uint32 final)
{
	struct TZStrmPrvt* zstrm;

	zstrm = ZPRVT(state);
	if (zstrm->public.smode != ZSTRM_DEFLATE) {
		badusage(zstrm);
		return;
	}
	if (zstrm->public.state == 1 || zstrm->public.state == 2) {
		/* nothing written yet: an empty stream is still a whole container */
		if (!final) {
			return;
		}
		zstrm_deflate(state, zstrm->iobuffer, 0);
		if (zstrm->public.state != 3) {
			return;
		}
	}
	if (zstrm->public.state != 3) {
		return;
	}
	if (!zs_grow(zstrm, &zstrm->inbuf, &zstrm->incap, 0, ZS_BATCH)) {
		SETERROR(ZSTRM_EOOM);
		SETSTATE(4);
		return;
	}
	dobatch(zstrm, final ? DEFLT_END : DEFLT_FLUSH);
	if (zstrm->public.error) {
		SETSTATE(4);
		return;
	}
	if (final == 0) {
		return;
	}
	switch (zstrm->public.stype) {
		case ZSTRM_GZIP: emitgziptail(zstrm); break;
		case ZSTRM_ZLIB: emitzlibtail(zstrm); break;
		default:
			break;
	}
	SETSTATE(4);
}

/* ---- checksums (zstrm.c:1323-1527); scanned on the GPU ------------------- */

static void
noengine(const char* fn)
{
	fprintf(stderr, "jdeflate: %s needs a gfx950 device (no CPU path)\n", fn);
	abort();
}

uint32
zstrm_crc32update(uint32 chcksm, const uint8* source, uintxx size)
{
	uint32 c = chcksm;
	if (size && jdgpu_checksum(source, size, &c, NULL) != 0) {
		noengine("zstrm_crc32update");
	}
	return c;
}

uint32
zstrm_adler32update(uint32 chcksm, const uint8* source, uintxx size)
{
	uint32 a = chcksm;
	if (size && jdgpu_checksum(source, size, NULL, &a) != 0) {
		noengine("zstrm_adler32update");
	}
	return a;
}
