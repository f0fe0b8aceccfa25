/*
 * zstrm.c -- the zstrm_* container API (jdeflate/zstrm.h):
 * raw deflate, zlib (RFC 1950) and gzip (RFC 1952) framing around this
 * library's own drop-in deflator_* / inflator_*, as the reference layers its
 * zstrm over its deflator and inflator.  The CRC-32 / Adler-32 of the data
 * are scanned by k_checksum on the device copy the codec already holds
 * (jd_internal.h hooks), so the container adds no pass over the data.
 *
 * Observable behaviour follows the reference zstrm.c: the state values
 * (NOTSET, READY, NEEDDICT, NORMAL, END), the error codes, flag validation
 * (zstrm_create :81-172), the header parsers (:446-624: gzip FEXTRA /
 * FNAME / FCOMMENT / FHCRC skipped, zlib FDICT + DICTID, raw streams
 * recognised by their first block header), trailer checks (:626-696), the
 * preset-dictionary protocol (:327-390) and the trailers written
 * (:1233-1265).  The implementation is this library's:
 *
 *  - a container source is a byte cursor over the caller's buffer, or over
 *    a staging slab refilled from the read callback (32 KiB reads, up to
 *    ZS_SLAB per inflator call so the GPU decodes large pieces);
 *  - the deflate stream between header and trailer goes through
 *    inflator_inflate, whose exact `srcend` at the final block tells where
 *    the trailer starts;
 *  - deflate hands each zstrm_deflate call's bytes to deflator_deflate
 *    (64 KiB independent blocks, batched up to 256 MiB per GPU launch) and
 *    writes the compressed bytes through the target callback.
 * Deliberate differences are listed in include/jdeflate/zstrm.h.
 */
#include <jdeflate/zstrm.h>
#include <jdeflate/jdgpu.h>

#include "jd_crc.h"
#include "jd_internal.h"

#include <stdlib.h>
#include <string.h>

#define ZS_IOSIZE 32768u              /* one callback read / write (IOBFFRSIZE) */
#define ZS_SLAB   (16u << 20)          /* callback-mode input per inflator call */
#define ZS_SINK   (4u << 20)           /* deflate: output staged per callback round */
#define ZS_BATCH  (256u << 20)         /* the drop-in deflator's largest batch */

#define ZS_MODEBITS 0x000f0000u
#define ZS_TYPEBITS 0x00f00000u
#define ZS_ANYTYPE  (ZSTRM_DFLT | ZSTRM_ZLIB | ZSTRM_GZIP)

struct TZStrmPrvt {
	struct TZStrm public;
	const struct TAllocator* allctr;

	TInflator* infl;        /* inflate mode */
	TDeflator* defl;        /* deflate mode */
	uint32 docrc;
	uint32 doadler;

	/* inflate: the container bytes not read yet are [cur, lim); in callback
	 * mode they live in `slab` and `rfn` supplies more */
	const uint8* cur;
	const uint8* lim;
	TZStrmIFn rfn;
	void* ruser;
	uint32 reof;            /* the read callback returned 0              */
	uint8* slab;
	uintxx slabcap;
	uintxx used;            /* container bytes consumed                   */
	uint32 ended;           /* the deflate stream's final block ended     */

	/* deflate: target callback and the staging buffer it is fed from */
	TZStrmOFn wfn;
	void* wuser;
	uint8* sink;
	uintxx sinkcap;
};

#define ZS(S) ((struct TZStrmPrvt*) (uintptr_t) (S))

static void* zs_request(uintxx size, void* user) { (void) user; return malloc(size); }
static void zs_dispose(void* p, uintxx size, void* user) { (void) size; (void) user; free(p); }
static const struct TAllocator zs_defaultallocator = { zs_request, zs_dispose, NULL };

static void
fail(struct TZStrmPrvt* z, uint32 error)
{
	if (z->public.error == 0) {
		z->public.error = error;
	}
	z->public.state = ZSTRM_END;
}

/* a call that the current state does not allow */
static void
misuse(struct TZStrmPrvt* z)
{
	fail(z, ZSTRM_EINCORRECTUSE);
}

/* flags (:81-172): a mode; for deflate a level 0-9 and a type, where a
 * known type bit may not be combined with any other type bit; an inflate
 * stream without a type accepts all three */
static int
validflags(uintxx* flags, intxx level)
{
	const uint32 mode = (uint32) (*flags & ZS_MODEBITS);
	uint32 type = (uint32) (*flags & ZS_TYPEBITS);

	if (mode == ZSTRM_INFLATE) {
		if (type == 0) {
			*flags |= ZS_ANYTYPE;
		}
		return 1;
	}
	if (mode != ZSTRM_DEFLATE || type == 0 || level < 0 || level > 9) {
		return 0;
	}
	return !((type & ZS_ANYTYPE) && (type & (type - 1)));
}

const TZStrm*
zstrm_create(uintxx flags, intxx level, const TAllocator* allctr)
{
	struct TZStrmPrvt* z;

	if (!validflags(&flags, level) || !jdgpu_available()) {
		return NULL;
	}
	if (allctr == NULL) {
		allctr = &zs_defaultallocator;
	}
	z = allctr->request(sizeof(*z), allctr->user);
	if (z == NULL) {
		return NULL;
	}
	memset(z, 0, sizeof(*z));
	z->allctr = allctr;
	z->public.flags = (uint32) flags;
	z->public.smode = (uint32) (flags & ZS_MODEBITS);
	if (z->public.smode == ZSTRM_INFLATE) {
		z->infl = inflator_create(flags & 0xff00u, allctr);
	} else {
		z->public.stype = (uint32) (flags & ZS_TYPEBITS);
		z->public.level = (int32) level;
		z->defl = deflator_create(flags & 0x00ffu, level, allctr);
	}
	if (z->infl == NULL && z->defl == NULL) {
		allctr->dispose(z, sizeof(*z), allctr->user);
		return NULL;
	}
	zstrm_reset(&z->public);
	return &z->public;
}

void
zstrm_destroy(const TZStrm* state)
{
	struct TZStrmPrvt* z = ZS(state);

	if (z == NULL) {
		return;
	}
	inflator_destroy(z->infl);
	deflator_destroy(z->defl);
	if (z->slab) {
		z->allctr->dispose(z->slab, z->slabcap, z->allctr->user);
	}
	if (z->sink) {
		z->allctr->dispose(z->sink, z->sinkcap, z->allctr->user);
	}
	z->allctr->dispose(z, sizeof(*z), z->allctr->user);
}

void
zstrm_reset(const TZStrm* state)
{
	struct TZStrmPrvt* z = ZS(state);
	const uint32 f = z->public.flags;

	z->public.state = ZSTRM_NOTSET;
	z->public.error = 0;
	z->public.total = 0;
	z->public.usedinput = 0;
	z->public.dictid = 0;
	z->public.dict = 0;
	z->public.crc = 0xffffffffu;
	z->public.adler = 1;
	z->cur = z->lim = NULL;
	z->rfn = NULL;
	z->ruser = NULL;
	z->reof = 0;
	z->used = 0;
	z->ended = 0;
	z->wfn = NULL;
	z->wuser = NULL;
	if (z->infl) {
		z->public.stype = 0;
		z->docrc = (f & ZSTRM_DOCRC) != 0;
		z->doadler = (f & ZSTRM_DOADLER) != 0;
		inflator_reset(z->infl);
	} else {
		/* deflate: the container type fixes the checksum it carries */
		z->docrc = (f & ZSTRM_DOCRC) != 0 || z->public.stype == ZSTRM_GZIP;
		z->doadler = (f & ZSTRM_DOADLER) != 0 || z->public.stype == ZSTRM_ZLIB;
		deflator_reset(z->defl);
		jd_deflator_checksums(z->defl, z->docrc ? &z->public.crc : NULL,
		                      z->doadler ? &z->public.adler : NULL);
	}
}

/* The header inlines assert a non-empty source, and inflator_setsrc
 * refuses new input once `final` was given; zstrm hands the inflator the
 * unread rest of the same container (possibly empty) through the same
 * public fields. */
static void
insource(TInflator* i, const uint8* p, uintxx n)
{
	static const uint8 none = 0;
	i->source = i->sbgn = n ? p : &none;
	i->send = i->source + n;
}

static void
desource(TDeflator* d, const uint8* p, uintxx n)
{
	static const uint8 none = 0;
	if (n) {
		deflator_setsrc(d, p, n);
	} else if (d->flush == 0) {
		d->source = d->sbgn = d->send = &none;
	}
}

/* ---- container source (inflate) ---------------------------------------- */

/* make at least `want` unread bytes available if the callback can supply
 * them; 0 when none is left */
static uintxx
avail(struct TZStrmPrvt* z, uintxx want)
{
	uintxx have = (uintxx) (z->lim - z->cur);

	if (have >= want || z->rfn == NULL || z->reof || z->public.error) {
		return have;
	}
	if (z->slab == NULL) {
		z->slab = z->allctr->request(ZS_SLAB, z->allctr->user);
		if (z->slab == NULL) {
			fail(z, ZSTRM_EOOM);
			return have;
		}
		z->slabcap = ZS_SLAB;
	}
	if (want > z->slabcap) {
		want = z->slabcap;
	}
	memmove(z->slab, z->cur, have);
	z->cur = z->slab;
	while (have < want && !z->reof) {
		uintxx room = z->slabcap - have;
		uintxx ask = room < ZS_IOSIZE ? room : ZS_IOSIZE;
		intxx r = z->rfn(z->slab + have, ask, z->ruser);

		if (r == 0) {
			z->reof = 1;
		} else if (r < 0 || (uintxx) r > ZS_IOSIZE) {
			fail(z, ZSTRM_EIOERROR);
			break;
		} else {
			have += (uintxx) r;
			/* a short read (a pipe or socket with nothing more ready):
			 * decode what came instead of waiting for a full slab */
			if ((uintxx) r < ask && want > 1) {
				break;
			}
		}
	}
	z->lim = z->slab + have;
	return have;
}

/* next container byte; a missing byte is ESRCEXHSTD for a buffer source,
 * EBADDATA for a callback (fetchbyte :411-444) */
static uint32
nextbyte(struct TZStrmPrvt* z)
{
	if (z->public.error) {
		return 0;
	}
	if (avail(z, 1) == 0) {
		if (z->public.error == 0) {
			z->public.error = z->rfn ? ZSTRM_EBADDATA : ZSTRM_ESRCEXHSTD;
		}
		return 0;
	}
	z->used++;
	return *z->cur++;
}

static uint32
le32(struct TZStrmPrvt* z)
{
	uint32 v = 0;
	int i;
	for (i = 0; i < 4; i++) v |= nextbyte(z) << (8 * i);
	return v;
}

static uint32
be32(struct TZStrmPrvt* z)
{
	uint32 v = 0;
	int i;
	for (i = 0; i < 4; i++) v = (v << 8) | nextbyte(z);
	return v;
}

/* gzip member header (parsegziphead :446-509): ID1 ID2 CM FLG MTIME(4)
 * XFL OS, then the optional fields FLG announces */
static void
gzipheader(struct TZStrmPrvt* z)
{
	uint32 flg, k;

	if (nextbyte(z) != 0x1f || nextbyte(z) != 0x8b || nextbyte(z) != 0x08) {
		fail(z, ZSTRM_EBADDATA);
		return;
	}
	flg = nextbyte(z);
	for (k = 0; k < 6; k++) nextbyte(z);                        /* MTIME XFL OS */
	if (flg & 0x04) {                                           /* FEXTRA */
		uint32 xlen = nextbyte(z);
		xlen |= nextbyte(z) << 8;
		while (xlen-- && z->public.error == 0) nextbyte(z);
	}
	if (flg & 0x08) while (nextbyte(z) != 0);                   /* FNAME */
	if (flg & 0x10) while (nextbyte(z) != 0);                   /* FCOMMENT */
	if (flg & 0x02) { nextbyte(z); nextbyte(z); }              /* FHCRC */
}

/* zlib header (parsezlibhead :513-565): CM 8 with CINFO <= 7; FDICT brings
 * the DICTID and the NEEDDICT state.  FCHECK is not verified (as in the
 * reference). */
static void
zlibheader(struct TZStrmPrvt* z)
{
	const uint32 cmf = nextbyte(z), flg = nextbyte(z);

	if (z->public.error) {
		return;
	}
	if ((cmf & 0x0f) != 8 || (cmf >> 4) > 7) {
		fail(z, ZSTRM_EBADDATA);
		return;
	}
	if (flg & 0x20) {
		z->public.dictid = be32(z);
		if (z->public.error == 0) {
			z->public.state = ZSTRM_NEEDDICT;
		}
	}
}

/* container type from its first byte (parsehead :567-624): 1F is gzip, a
 * CM nibble of 8 is zlib, anything else is a raw deflate block header,
 * whose BTYPE may not be the reserved 11 */
static uint32
sniff(uint32 first)
{
	if (first == 0x1f) {
		return ZSTRM_GZIP;
	}
	if ((first & 0x0f) == 0x08) {
		return ZSTRM_ZLIB;
	}
	return ((first >> 1) & 3) == 3 ? 0 : ZSTRM_DFLT;
}

static void
readheader(struct TZStrmPrvt* z)
{
	uint32 type;

	if (avail(z, 1) == 0) {
		nextbyte(z);                    /* sets the exhaustion error */
		fail(z, z->public.error);
		return;
	}
	type = sniff(*z->cur);
	if (type == 0) {
		fail(z, ZSTRM_EBADDATA);
		return;
	}
	if ((z->public.flags & type) == 0) {
		fail(z, ZSTRM_EFORMAT);
		return;
	}
	z->public.stype = type;
	if (type == ZSTRM_GZIP) {
		z->docrc = 1;
		gzipheader(z);
	} else if (type == ZSTRM_ZLIB) {
		z->doadler = 1;
		zlibheader(z);
	}
	if (z->public.flags & ZSTRM_NOCRC) {
		z->docrc = 0;
	}
	if (z->public.flags & ZSTRM_NOADLER) {
		z->doadler = 0;
	}
	if (z->public.error) {
		fail(z, z->public.error);
		return;
	}
	jd_inflator_checksums(z->infl, z->docrc ? &z->public.crc : NULL,
	                      z->doadler ? &z->public.adler : NULL);
	if (z->public.state != ZSTRM_NEEDDICT) {
		z->public.state = ZSTRM_NORMAL;
	}
}

/* the trailer after the final block (checkgziptail :626-668, checkzlibtail
 * :670-696): the checksum when it is kept, and gzip's ISIZE */
static void
readtrailer(struct TZStrmPrvt* z)
{
	if (z->docrc) {
		z->public.crc ^= 0xffffffffu;
	}
	if (z->public.stype == ZSTRM_GZIP) {
		const uint32 crc = le32(z), isize = le32(z);
		if (z->public.error == 0 && z->docrc && crc != z->public.crc) {
			z->public.error = ZSTRM_ECHECKSUM;
		} else if (z->public.error == 0 && isize != (uint32) z->public.total) {
			z->public.error = ZSTRM_EBADDATA;
		}
	} else if (z->public.stype == ZSTRM_ZLIB) {
		const uint32 adler = be32(z);
		if (z->public.error == 0 && z->doadler && adler != z->public.adler) {
			z->public.error = ZSTRM_ECHECKSUM;
		}
	}
	z->public.usedinput = z->used;
	z->public.state = ZSTRM_END;
}

/* decode into target[0, n): the deflate stream through the inflator, then
 * the trailer once its final block has ended */
static uintxx
body(struct TZStrmPrvt* z, uint8* target, uintxx n)
{
	uintxx got = 0;

	while (got < n && !z->ended) {
		uintxx given, left;
		uint32 final;
		eINFLTResult r;

		/* input: everything at hand; a callback refills the slab first */
		given = avail(z, ZS_SLAB);
		if (z->public.error) {
			break;
		}
		final = z->rfn == NULL || z->reof;
		insource(z->infl, z->cur, given);
		inflator_settgt(z->infl, target + got, n - got);
		r = inflator_inflate(z->infl, final);
		got += inflator_tgtend(z->infl);
		/* the inflator keeps what it took; after the final block the
		 * bytes that follow are left to the trailer */
		left = given - inflator_srcend(z->infl);
		z->used += given - left;
		z->cur = z->lim - left;
		if (r == INFLT_OK) {
			z->ended = 1;
		} else if (r == INFLT_ERROR) {
			fail(z, ZSTRM_EDEFLATE);
		} else if (r == INFLT_SRCEXHSTD && final) {
			fail(z, ZSTRM_EDEFLATE);
		}
	}
	z->public.total += got;
	if (z->ended && z->public.state == ZSTRM_NORMAL) {
		readtrailer(z);
	}
	return got;
}

uintxx
zstrm_inflate(const TZStrm* state, void* target, uintxx n)
{
	struct TZStrmPrvt* z = ZS(state);

	if (z->infl == NULL) {
		misuse(z);
		return 0;
	}
	if (n > ((uintxx) 1 << 31) - 1) {
		fail(z, ZSTRM_ELIMIT);
		return 0;
	}
	if (z->public.state == ZSTRM_READY) {
		readheader(z);
		if (z->public.state == ZSTRM_NEEDDICT && n == 0) {
			return 0;               /* n = 0 asks whether a dictionary is needed */
		}
	}
	if (z->public.state == ZSTRM_NEEDDICT) {
		fail(z, ZSTRM_EMISSINGDICT);
	}
	if (z->public.state != ZSTRM_NORMAL || n == 0) {
		return 0;
	}
	return body(z, (uint8*) target, n);
}

void
zstrm_setsource(const TZStrm* state, const uint8* source, uintxx size)
{
	struct TZStrmPrvt* z = ZS(state);

	if (z->infl == NULL || z->public.state != ZSTRM_NOTSET) {
		misuse(z);
		return;
	}
	z->cur = source;
	z->lim = source + size;
	z->public.state = ZSTRM_READY;
	zstrm_inflate(state, NULL, 0);
}

void
zstrm_setsourcefn(const TZStrm* state, TZStrmIFn fn, void* user)
{
	struct TZStrmPrvt* z = ZS(state);

	if (z->infl == NULL || z->public.state != ZSTRM_NOTSET) {
		misuse(z);
		return;
	}
	z->rfn = fn;
	z->ruser = user;
	z->public.state = ZSTRM_READY;
	zstrm_inflate(state, NULL, 0);
}

void
zstrm_settargetfn(const TZStrm* state, TZStrmOFn fn, void* user)
{
	struct TZStrmPrvt* z = ZS(state);

	if (z->defl == NULL || z->public.state != ZSTRM_NOTSET) {
		misuse(z);
		return;
	}
	z->wfn = fn;
	z->wuser = user;
	z->public.state = ZSTRM_READY;
}

/* zstrm_setdctnr (:327-390).  Inflate: before the body, gzip excluded; a
 * zlib stream that asked for one must get the dictionary its DICTID names
 * (EBADDICT otherwise); it primes the inflator's window.  Deflate (zlib, not
 * yet written): FDICT and DICTID go into the header; the independent blocks
 * do not reference the dictionary. */
void
zstrm_setdctnr(const TZStrm* state, const uint8* dict, uintxx size)
{
	struct TZStrmPrvt* z = ZS(state);
	const uint32 st = z->public.state;

	if (st == ZSTRM_NOTSET || st == ZSTRM_END || dict == NULL || size == 0) {
		misuse(z);
		return;
	}
	if (z->infl) {
		if (st == ZSTRM_READY) {
			readheader(z);
		}
		/* only a zlib stream with FDICT takes one */
		if (z->public.state != ZSTRM_NEEDDICT || z->public.stype == ZSTRM_GZIP) {
			misuse(z);
			return;
		}
		if (zstrm_adler32update(1, dict, size) != z->public.dictid) {
			fail(z, ZSTRM_EBADDICT);
			return;
		}
		inflator_setdctnr(z->infl, dict, size);
		z->public.state = ZSTRM_NORMAL;
		return;
	}
	if (st != ZSTRM_READY || z->public.stype == ZSTRM_GZIP || z->public.dict) {
		misuse(z);
		return;
	}
	z->public.dictid = zstrm_adler32update(1, dict, size);
	z->public.dict = 1;
}

/* ---- deflate ------------------------------------------------------------ */

static void
put(struct TZStrmPrvt* z, const uint8* p, uintxx n)
{
	while (n && z->public.error == 0) {
		const uintxx k = n < ZS_IOSIZE ? n : ZS_IOSIZE;
		if (z->wfn(p, k, z->wuser) != (intxx) k) {
			fail(z, ZSTRM_EIOERROR);
			return;
		}
		p += k;
		n -= k;
	}
}

/* the container header, before the first data (emitgziphead :1003-1022,
 * emitzlibhead :1024-1053 with a valid FCHECK) */
static void
header(struct TZStrmPrvt* z)
{
	uint8 h[10];
	uintxx k = 0;

	if (z->public.stype == ZSTRM_GZIP) {
		/* ID1 ID2 CM=8, no flags, MTIME 0, XFL 0, OS 0 */
		memset(h, 0, sizeof h);
		h[0] = 0x1f;
		h[1] = 0x8b;
		h[2] = 0x08;
		k = 10;
	} else if (z->public.stype == ZSTRM_ZLIB) {
		/* CMF 78 (deflate, 32 KiB window); FLG = FDICT, FCHECK so that
		 * CMF*256 + FLG is a multiple of 31 */
		const uint32 flg = z->public.dict ? 0x20u : 0;
		h[0] = 0x78;
		h[1] = (uint8) (flg + 31 - ((0x78u << 8) | flg) % 31);
		k = 2;
		if (z->public.dict) {
			const uint32 id = z->public.dictid;
			h[2] = (uint8) (id >> 24);
			h[3] = (uint8) (id >> 16);
			h[4] = (uint8) (id >> 8);
			h[5] = (uint8) id;
			k = 6;
		}
	}
	put(z, h, k);
	z->public.state = ZSTRM_NORMAL;
}

/* run the deflator over [src, src + n) with `flush`, writing out what it
 * produces; 1 when it reached its goal (input taken, or the flush done) */
static int
pump(struct TZStrmPrvt* z, const uint8* src, uintxx n, eDEFLTFlush flush)
{
	eDEFLTResult r;
	/* a sink that holds a whole batch's worst case lets the deflator write
	 * its blocks straight into it (no staging copy); small inputs keep the
	 * 4 MiB one */
	uintxx want = ZS_SINK;

	if (n > ZS_SINK / 2) {
		const uintxx b = (uintxx) jdgpu_bound(n < ZS_BATCH ? n : ZS_BATCH, 65536) + 64;
		want = b > want ? b : want;
	}
	if (z->sink == NULL || z->sinkcap < want) {
		if (z->sink) {
			z->allctr->dispose(z->sink, z->sinkcap, z->allctr->user);
		}
		z->sinkcap = 0;
		z->sink = z->allctr->request(want, z->allctr->user);
		if (z->sink == NULL) {
			fail(z, ZSTRM_EOOM);
			return 0;
		}
		z->sinkcap = want;
	}
	desource(z->defl, src, n);
	do {
		deflator_settgt(z->defl, z->sink, z->sinkcap);
		r = deflator_deflate(z->defl, flush);
		put(z, z->sink, deflator_tgtend(z->defl));
	} while (r == DEFLT_TGTEXHSTD && z->public.error == 0);
	if (r == DEFLT_ERROR) {
		fail(z, z->defl->error == DEFLT_EOOM ? ZSTRM_EOOM : ZSTRM_EDEFLATE);
	}
	return z->public.error == 0;
}

uintxx
zstrm_deflate(const TZStrm* state, const void* source, uintxx n)
{
	struct TZStrmPrvt* z = ZS(state);

	if (z->defl == NULL) {
		misuse(z);
		return 0;
	}
	if (n > ((uintxx) 1 << 31) - 1) {
		fail(z, ZSTRM_ELIMIT);
		return 0;
	}
	if (z->public.state == ZSTRM_READY || z->public.state == ZSTRM_NEEDDICT) {
		header(z);
	}
	if (z->public.state != ZSTRM_NORMAL || z->public.error) {
		return 0;
	}
	if (n && !pump(z, (const uint8*) source, n, DEFLT_NOFLUSH)) {
		return 0;
	}
	z->public.total += n;
	return n;
}

/* zstrm_flush (:1267-1318): FLUSH ends the pending input at a byte
 * boundary; `final` ends the stream and writes the trailer
 * (emitgziptail :1233-1252, emitzlibtail :1254-1265) */
void
zstrm_flush(const TZStrm* state, uint32 final)
{
	struct TZStrmPrvt* z = ZS(state);
	uint8 t[8];

	if (z->defl == NULL) {
		misuse(z);
		return;
	}
	if (z->public.state == ZSTRM_READY || z->public.state == ZSTRM_NEEDDICT) {
		if (!final) {
			return;
		}
		header(z);                  /* an empty stream is still a container */
	}
	if (z->public.state != ZSTRM_NORMAL || z->public.error) {
		return;
	}
	if (!pump(z, NULL, 0, final ? DEFLT_END : DEFLT_FLUSH) || !final) {
		return;
	}
	if (z->public.stype == ZSTRM_GZIP) {
		const uint32 c = z->public.crc ^ 0xffffffffu, isize = (uint32) z->public.total;
		int i;
		z->public.crc = c;
		for (i = 0; i < 4; i++) {
			t[i] = (uint8) (c >> (8 * i));
			t[4 + i] = (uint8) (isize >> (8 * i));
		}
		put(z, t, 8);
	} else if (z->public.stype == ZSTRM_ZLIB) {
		const uint32 a = z->public.adler;
		int i;
		for (i = 0; i < 4; i++) t[i] = (uint8) (a >> (24 - 8 * i));
		put(z, t, 4);
	}
	z->public.state = ZSTRM_END;
}

/* ---- checksum utilities (zstrm.c:1323-1527) ------------------------------ */

/* bulk data is scanned on the GPU (k_checksum); short inputs, and any input
 * when no device is usable, on the host (a device round trip costs more
 * than scanning below 64 KiB, and these utilities have no error channel) */
#define ZS_HOSTSCAN 65536u

uint32
zstrm_crc32update(uint32 chcksm, const uint8* source, uintxx size)
{
	uint32 c = chcksm;

	if (size >= ZS_HOSTSCAN && jdgpu_checksum(source, size, &c, NULL) == 0) {
		return c;
	}
	return jdcrc_bytes(chcksm, source, size);
}

uint32
zstrm_adler32update(uint32 chcksm, const uint8* source, uintxx size)
{
	uint32 a = chcksm;

	if (size >= ZS_HOSTSCAN && jdgpu_checksum(source, size, NULL, &a) == 0) {
		return a;
	}
	return jdadler_bytes(chcksm, source, size);
}
