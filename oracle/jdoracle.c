/*
 * jdoracle.c -- CPU restatement of the jdeflate reference codec
 *               (Jpn666/jdeflate 0.4.0, src/deflator.c + src/inflator.c).
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the HIP engine and the timed CPU
 * baseline.  Never linked into the product library.  Parity: PARTIALLY
 * PINNED (see jdoracle.h and DESIGN.md "Oracle").
 *
 * Every function cites the reference lines whose behaviour it restates.  The
 * data structures deliberately mirror the reference's (int16 relative hash
 * heads, uint16 3-byte ring, uint16 token slots) so that the quirks listed in
 * SURVEY.md Appendix A come out of the same arithmetic.
 */
#include "jdoracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* constants (deflator.c:21-45, 317-324)                                     */
/* ------------------------------------------------------------------------ */
#define WSIZE      32768u          /* LZ77 window, deflator.c:30          */
#define GUARD      304u            /* WNDNGUARDSIZE on LP64, :321         */
#define MINMATCH   3u
#define MAXMATCH   258u
#define LOOKAHEAD  (MINMATCH + MAXMATCH)   /* MINLOOKAHEAD :2328           */
#define H4BITS     16
#define H3BITS     14
#define CHAINMASK  32767u
#define RING3MASK  16383u
#define EOBSYM     256

/* per-level search parameters: deflator.c:242-263 (good, nice, chain) */
static const uint32_t kgood[10]  = {0, 8, 8, 8, 8, 8, 16, 32, 64, 192};
static const uint32_t knice[10]  = {0, 4, 8, 16, 32, 64, 16, 64, 128, 256};
static const uint32_t kchain[10] = {0, 2, 8, 16, 32, 128, 48, 128, 320, 512};
/* window bits and token-list bits per level: getmeminfo deflator.c:210-230 */
static const uint8_t kwbits[10]  = {16, 16, 16, 16, 16, 16, 17, 17, 17, 17};
static const uint8_t klzbits[10] = {0, 14, 15, 15, 15, 15, 16, 16, 17, 17};

/* RFC 1951 length / distance bases (the values of deflator.c:3076-3110 and
 * inflator.c:336-373) */
static const uint16_t klbase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17,
    19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t klextra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2,
    2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kdbase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49,
    65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
    8193, 12289, 16385, 24577};
static const uint8_t kdextra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5,
    6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
/* precode transmission order, deflator.c:1357 / inflator.c:1106 */
static const uint8_t kpcorder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4,
    12, 3, 13, 2, 14, 1, 15};

static uint32_t load_le32(const uint8_t* p)
{
    return (uint32_t) p[0] | ((uint32_t) p[1] << 8) | ((uint32_t) p[2] << 16)
         | ((uint32_t) p[3] << 24);
}

/* floor(log2(x)); ctb_u32log2 assumed = floor */
static int ilog2(uint32_t x)
{
    int r = -1;
    while (x) { x >>= 1; r++; }
    return r;
}

/* length symbol index 0..28 for a match length 3..258 (getlsymbol :2281) */
static unsigned lsym_of(unsigned len)
{
    unsigned s = 0;
    if (len == 258) return 28;
    while (s < 27 && klbase[s + 1] <= len) s++;
    return s;
}

/* distance symbol 0..29 for a distance 1..32768 (getdsymbol :2237) */
static unsigned dsym_of(unsigned d)
{
    unsigned s = 0;
    while (s < 29 && kdbase[s + 1] <= d) s++;
    return s;
}

/* reverse the low `len` bits (reversecode :1084) */
static uint32_t bitrev(uint32_t code, unsigned len)
{
    uint32_t r = 0;
    unsigned i;
    for (i = 0; i < len; i++) { r = (r << 1) | (code & 1); code >>= 1; }
    return r;
}

/* ------------------------------------------------------------------------ */
/* Huffman code construction (deflator.c:934-1390)                           */
/* ------------------------------------------------------------------------ */
typedef struct { uint8_t len; uint16_t code; } hcode_t;

/* ascending sort by (frequency, symbol): the order heapsort :971 produces */
static void sort_symbols(size_t* map, const size_t* frq, size_t n)
{
    size_t i, j;
    for (i = 1; i < n; i++) {          /* insertion sort; n <= 288 */
        size_t v = map[i];
        for (j = i; j > 0; j--) {
            size_t u = map[j - 1];
            if (frq[u] < frq[v] || (frq[u] == frq[v] && u < v)) break;
            map[j] = u;
        }
        map[j] = v;
    }
}

/* Moffat-Katajainen in-place code lengths over ascending weights
 * (katajainen :1033-1081): phase 1 builds parent links, phase 2 counts the
 * nodes level by level from the root and hands depths to the leaves. */
static void mk_lengths(size_t* a, long n)
{
    long leaf = 0, root = 0, nx;
    long lvl, top, cap, avail, k;

    for (nx = 0; nx < n - 1; nx++) {
        int take_root;
        take_root = leaf >= n || (root < nx && a[root] < a[leaf]);
        if (take_root) { a[nx] = a[root]; a[root++] = (size_t) nx; }
        else a[nx] = a[leaf++];
        take_root = leaf >= n || (root < nx && a[root] < a[leaf]);
        if (take_root) { a[nx] += a[root]; a[root++] = (size_t) nx; }
        else a[nx] += a[leaf++];
    }

    /* top: lowest index of the internal level just finished; the root is
     * node n-2; `cap` = child slots opened by the previous level */
    top = root = n - 2;
    lvl = 1;
    cap = 2;
    for (k = n - 1; k > 0; lvl++) {
        avail = 0;
        while (root && (long) a[root - 1] >= top) { root--; avail++; }
        for (nx = cap - avail; nx; nx--) a[k--] = (size_t) lvl;
        cap = avail * 2;
        top = root;
    }
}

/* cbloom Kraft fix-up in sorted order (limitlengths :992-1028) */
static void clamp_lengths(size_t* l, size_t n, size_t mlen)
{
    long i;
    long k = 0;
    for (i = 0; i < (long) n; i++) {
        if (l[i] > mlen) l[i] = mlen;
        k += 0x8000L >> l[i];
    }
    for (i = 0; i < (long) n; i++)
        while (l[i] < mlen && k > 0x8000L) { l[i]++; k -= 0x8000L >> l[i]; }
    for (i = (long) n - 1; i >= 0; i--)
        while (k + (0x8000L >> l[i]) <= 0x8000L) { k += 0x8000L >> l[i]; l[i]--; }
}

/* frequencies -> code lengths written back into frq[] (setuptable :1189 +
 * computelengths :1139), canonical bit-reversed codes into out[].
 * Returns last used symbol + 1. */
static unsigned build_code(size_t* frq, unsigned nsym, unsigned mlen,
                           hcode_t* out)
{
    size_t map[288], w[288];
    unsigned used = 0, i, last = 0;
    unsigned cnt[16], nxt[16];

    for (i = 0; i < nsym; i++) used += frq[i] != 0;
    if (used == 0) { frq[0] = 1; frq[1] = 1; }
    else if (used == 1) { if (frq[0]) frq[1] = 1; else frq[0] = 1; }

    used = 0;
    for (i = 0; i < nsym; i++) if (frq[i]) map[used++] = i;
    sort_symbols(map, frq, used);
    for (i = 0; i < used; i++) w[i] = frq[map[i]];
    mk_lengths(w, (long) used);
    clamp_lengths(w, used, mlen);

    memset(cnt, 0, sizeof(cnt));
    for (i = 0; i < used; i++) { cnt[w[i]]++; frq[map[i]] = w[i]; }
    nxt[0] = 0;
    for (i = 1; i <= 15; i++) nxt[i] = (nxt[i - 1] + cnt[i - 1]) << 1;
    for (i = 0; i < nsym; i++) {
        unsigned l = (unsigned) frq[i];
        out[i].len = (uint8_t) l;
        out[i].code = 0;
        if (l == 0) continue;
        out[i].code = (uint16_t) bitrev(nxt[l]++, l);
        last = i;
    }
    return last + 1;
}

/* run-length coding of a code-length list into precode symbols, in place
 * (countprecodes :1288-1354), including the phantom zero at index `size`. */
static void rle_lengths(size_t* c, size_t size, size_t* cf)
{
    size_t i, o = 0, run = 0, prev = 0xffff, maxrun = 0, cur;
    int capped;

    c[size + 1] = 0xffff;
    for (i = 0; i <= size; i++) {
        cur = c[i];
        if (cur == prev) {
            run++;
            if (run < maxrun) continue;
            capped = 1;
        } else {
            capped = 0;
        }
        if (run > 2) {
            size_t sym = prev ? 16 : (run > 10 ? 18 : 17);
            cf[sym]++;
            c[o++] = sym;
            c[o++] = run;
            if (capped) { run = 0; continue; }
        } else if (run) {
            cf[prev] += run;
            for (; run; run--) c[o++] = prev;
        }
        cf[cur]++;
        maxrun = cur ? 6 : 136;
        c[o++] = prev = cur;
        run = 0;
    }
    c[o - 1] = 0xffff;
}

/* ------------------------------------------------------------------------ */
/* deflator state                                                            */
/* ------------------------------------------------------------------------ */
typedef struct {
    int level;
    unsigned flags;
    int flush;
    uint32_t good, nice, maxchain;

    uint8_t* win;
    size_t wend;                  /* windowend offset                      */
    size_t inputend, cursor, whence3, whence4;

    int16_t* mhlist;
    int16_t* mchain;
    uint16_t* shlist;
    uint16_t* schain;

    uint32_t currobs[32], prevobs[32], obscount, newcount, obstotal;

    uint16_t* lz;
    size_t lzcap, zend;

    size_t lfrq[290], dfrq[34], cfrq[19];
    unsigned lmax, dmax, cmax;
    hcode_t lcode[288], dcode[32], pcode[19];
    int dynamic;

    const uint8_t* src;
    size_t srcpos, srclen;

    int blockinit, hasinput;
    size_t acc0;                  /* level 0: bytes of the open stored block (aux1) */
    uint32_t h3, h4;             /* aux3 / aux4                            */
    uint32_t held;               /* aux5                                   */
    int doshort;                 /* aux6                                   */

    uint8_t* out;
    size_t opos, ocap;
    uint64_t bb;
    unsigned bc;
    int overflow;

    uint32_t* trace;
    size_t ntrace, tracecap;
} D;

static void tr(D* s, uint32_t v)
{
    if (s->trace && s->ntrace < s->tracecap) s->trace[s->ntrace] = v;
    s->ntrace++;
}

/* bit writer: LSB-first, whole bytes leave as soon as they are complete;
 * identical bytes to the reference's 64-bit buffer (putbits :603) */
static void putbits(D* s, uint32_t v, unsigned n)
{
    s->bb |= (uint64_t) v << s->bc;
    s->bc += n;
    while (s->bc >= 8) {
        if (s->opos < s->ocap) s->out[s->opos] = (uint8_t) s->bb;
        else s->overflow = 1;
        s->opos++;
        s->bb >>= 8;
        s->bc -= 8;
    }
}

static void putbyte(D* s, uint8_t v) { putbits(s, v, 8); }

static void alignbits(D* s)
{
    if (s->bc) putbits(s, 0, 8 - s->bc);
}

static int d_init(D* s, int level, unsigned flags)
{
    size_t wsz;
    memset(s, 0, sizeof(*s));
    if (level < 0 || level > 9) return 0;
    s->level = level;
    s->flags = flags;
    s->good = kgood[level];
    s->nice = knice[level];
    s->maxchain = kchain[level];
    s->wend = (size_t) 1 << kwbits[level];
    wsz = s->wend + GUARD;
    s->win = (uint8_t*) calloc(wsz, 1);
    if (level) {
        s->lzcap = (size_t) 1 << klzbits[level];
        s->lz = (uint16_t*) malloc(s->lzcap * sizeof(uint16_t));
        s->mhlist = (int16_t*) malloc(65536 * sizeof(int16_t));
        s->mchain = (int16_t*) malloc(32768 * sizeof(int16_t));
        s->shlist = (uint16_t*) calloc(16384, sizeof(uint16_t));
        s->schain = (uint16_t*) calloc(16384, sizeof(uint16_t));
        if (!s->lz || !s->mhlist || !s->mchain || !s->shlist || !s->schain)
            return 0;
        /* resetcache :418-439 */
        for (wsz = 0; wsz < 65536; wsz++) s->mhlist[wsz] = -32768;
        for (wsz = 0; wsz < 32768; wsz++) s->mchain[wsz] = -32768;
    }
    return s->win != NULL;
}

static void d_free(D* s)
{
    free(s->win); free(s->lz); free(s->mhlist); free(s->mchain);
    free(s->shlist); free(s->schain);
}

/* slidehash :1900-1911 */
static void slidehash(D* s)
{
    unsigned j;
    for (j = 0; j < 65536; j++) {
        int16_t x = s->mhlist[j];
        s->mhlist[j] = (int16_t) (x >= 0 ? x - 32768 : -32768);
    }
    for (j = 0; j < 32768; j++) {
        int16_t x = s->mchain[j];
        s->mchain[j] = (int16_t) (x >= 0 ? x - 32768 : -32768);
    }
}

/* slidewindow :1818-1862 (window buffer assumed 8-byte aligned, as any
 * malloc result is) + fillwindow :1870-1897 */
static size_t fillwindow(D* s)
{
    size_t wleft = s->wend - s->inputend;
    size_t total = s->srclen - s->srcpos;

    if (total > wleft && wleft < 0x400) {
        size_t from = s->cursor - WSIZE;
        size_t r = from & 7;
        size_t slide;
        from -= r;
        slide = from;
        memmove(s->win, s->win + from, s->inputend - from);
        s->inputend -= slide;
        s->cursor = WSIZE + r;
        s->whence3 -= slide;
        s->whence4 -= slide;
        wleft = s->wend - s->inputend;
    }
    if (total > wleft) total = wleft;
    if (total) {
        memcpy(s->win + s->inputend, s->src + s->srcpos, total);
        s->srcpos += total;
        s->inputend += total;
    }
    return total;
}

/* big-endian 4-byte head (gethead :1931) and multiplicative hash (:1944) */
static uint32_t hashat(const D* s, size_t off, unsigned bits, unsigned shift)
{
    const uint8_t* p = s->win + off;
    uint32_t head = ((uint32_t) p[0] << 24) | ((uint32_t) p[1] << 16)
                  | ((uint32_t) p[2] << 8) | (uint32_t) p[3];
    return (uint32_t) ((head >> shift) * 0x1e35a7bdu) >> (32 - bits);
}

/* common prefix length of two window positions, capped at 258
 * (getmatchlength :1978; values above 258 never change a selection because
 * nice <= 256 at every level) */
static uint32_t matchlen(const uint8_t* a, const uint8_t* b)
{
    uint32_t n = 0;
    while (n < MAXMATCH) {
        uint64_t x, y, z;
        memcpy(&x, a + n, 8);
        memcpy(&y, b + n, 8);
        z = x ^ y;
        if (z) {
            n += (uint32_t) __builtin_ctzll(z) >> 3;
            return n < MAXMATCH ? n : MAXMATCH;
        }
        n += 8;
    }
    return MAXMATCH;
}

/* insert the cursor into both chains and hash cursor+1; shared by
 * getmatch2 :2629-2648 and skipbytes2 :2743-2758 */
static void insert2(D* s, uint16_t* pos4out, uint16_t* pos3out,
                    int16_t* next4, uint16_t* next3)
{
    uint16_t pos4 = (uint16_t) (s->cursor - s->whence4);
    uint16_t pos3 = (uint16_t) (s->cursor - s->whence3);
    if (pos4 == WSIZE) {
        slidehash(s);
        s->whence4 += WSIZE;
        pos4 = 0;
    }
    if (next3) *next3 = s->shlist[s->h3];
    if (next4) *next4 = s->mhlist[s->h4];
    s->mchain[pos4 & CHAINMASK] = s->mhlist[s->h4];
    s->mhlist[s->h4] = (int16_t) pos4;
    s->schain[pos3 & RING3MASK] = s->shlist[s->h3];
    s->shlist[s->h3] = pos3;
    s->h3 = hashat(s, s->cursor + 1, H3BITS, 8);
    s->h4 = hashat(s, s->cursor + 1, H4BITS, 0);
    if (pos4out) *pos4out = pos4;
    if (pos3out) *pos3out = pos3;
}

#ifdef JDO_STATS
/* demand statistics (tools/parse_demand.c): each getmatch2 call and its chain
 * hops; the hops a threshold-2 full-budget walk takes at each position the
 * parse skips (what k_match computes there anyway) */
void jdo_stat_call(int lazy, uint32_t hops, uint32_t len);
void jdo_stat_skip(uint32_t hops);
#endif

/* getmatch2 :2606-2721 */
static void getmatch2(D* s, uint32_t length, int shrt, uint32_t* olen,
                      uint32_t* ooff)
{
#ifdef JDO_STATS
    const int lazy_ = length >= 3;
    uint32_t hops_ = 0;
#endif
    const uint8_t* w = s->win;
    size_t cur = s->cursor;
    size_t strend = cur + MAXMATCH;
    size_t best = cur;
    uint16_t pos4, pos3, next3;
    int16_t next4, limit;
    uint32_t chain;

    if (strend > s->inputend) strend = s->inputend;
    insert2(s, &pos4, &pos3, &next4, &next3);
#ifdef JDO_DEBUG
    const long dbg = getenv("JDO_DEBUG_POS") ? atol(getenv("JDO_DEBUG_POS")) : -1;
    const long spos = (long) (s->srcpos - s->inputend + cur);
    if (spos == dbg) fprintf(stderr, "getmatch2 pos %ld length %u pos4 %u next4 %d h4 %u\n", spos, length, pos4, next4, s->h4);
#endif

    chain = s->maxchain;
    if (length >= 3) chain >>= 1;
    limit = (int16_t) (pos4 - WSIZE);
    for (; chain; chain--) {
        size_t q;
        if (next4 <= limit) break;
#ifdef JDO_STATS
        hops_++;
#endif
        q = (size_t) ((ptrdiff_t) s->whence4 + next4);
#ifdef JDO_DEBUG
        if (spos == dbg) fprintf(stderr, "  cand %ld len %u\n", (long) (s->srcpos - s->inputend + q), matchlen(w + cur, w + q));
#endif
        if (w[cur + length] == w[q + length]) {
            uint32_t n = matchlen(w + cur, w + q);
            if (n > length) {
                length = n;
                best = q;
                if (length >= s->nice) goto done;
            }
        }
        next4 = s->mchain[(uint16_t) next4 & CHAINMASK];
    }

    if (shrt && length < 3) {
        uint32_t s1 = load_le32(w + cur);
        int k;
        for (k = 0; k < 2; k++) {
            uint16_t noff;
            if (next3 == 0) break;
            noff = (uint16_t) (pos3 - next3);
            if (noff > WSIZE || noff == 0) break;
            if (((load_le32(w + cur - noff) ^ s1) & 0x00ffffffu) == 0) {
                length = 3;
                best = cur - noff;
                break;
            }
            next3 = s->schain[next3 & RING3MASK];
        }
    }
done:
    if (cur + length > strend) length -= (uint32_t) (cur + length - strend);
#ifdef JDO_STATS
    jdo_stat_call(lazy_, hops_, length);
#endif
    *olen = length;
    *ooff = (uint32_t) (cur - best);
}

/* skipbytes2 :2730-2764 */
static void skipbytes2(D* s, uint32_t skip, uint32_t total)
{
    for (; skip < total; skip++) {
        s->cursor++;
#ifdef JDO_STATS
        {
            uint16_t p4, p3, n3;
            int16_t n4;
            insert2(s, &p4, &p3, &n4, &n3);
            const uint8_t* w = s->win;
            const size_t cur = s->cursor;
            uint32_t len = 2, hops = 0, chain = s->maxchain;
            const int16_t limit = (int16_t) (p4 - WSIZE);
            for (; chain; chain--) {
                if (n4 <= limit) break;
                hops++;
                const size_t q = (size_t) ((ptrdiff_t) s->whence4 + n4);
                if (w[cur + len] == w[q + len]) {
                    const uint32_t n = matchlen(w + cur, w + q);
                    if (n > len) {
                        len = n;
                        if (len >= s->nice) break;
                    }
                }
                n4 = s->mchain[(uint16_t) n4 & CHAINMASK];
            }
            jdo_stat_skip(hops);
        }
#else
        insert2(s, NULL, NULL, NULL, NULL);
#endif
    }
}

/* addmatch / addliteral :2294-2312 */
static void addmatch(D* s, uint32_t len, uint32_t off, unsigned ls,
                     unsigned ds)
{
    s->lz[s->zend++] = (uint16_t) (len | 0x8000);
    s->lz[s->zend++] = (uint16_t) off;
    s->lz[s->zend++] = (uint16_t) ((ls << 8) | ds);
    s->lfrq[257 + ls]++;
    s->dfrq[ds]++;
    tr(s, 0x80000000u | (len << 16) | off);
}

static void addliteral(D* s, unsigned c)
{
    s->lz[s->zend++] = (uint16_t) c;
    s->lfrq[c]++;
    tr(s, c);
}

/* block-split observations :2528-2596 */
static void resetobs(D* s)
{
    memset(s->currobs, 0, sizeof(s->currobs));
    memset(s->prevobs, 0, sizeof(s->prevobs));
    s->obscount = s->newcount = s->obstotal = 0;
}

static void obsmatch(D* s, uint32_t len, unsigned ls)
{
    s->currobs[16 + (ls >> 1)]++;
    s->newcount++;
    s->obstotal += len;
}

static void obsliteral(D* s, unsigned c)
{
    s->currobs[c >> 4]++;
    s->newcount++;
    s->obstotal++;
}

static int shouldsplit(D* s)
{
    unsigned j;
    if (s->obscount > 0) {
        uint32_t delta = 0;
        for (j = 0; j < 32; j++) {
            uint32_t a = s->prevobs[j], b = s->currobs[j];
            delta += a > b ? a - b : b - a;
        }
        if (delta >= 320 && s->obstotal >= 7168) {
            resetobs(s);
            return 1;
        }
    }
    for (j = 0; j < 32; j++) {
        s->prevobs[j] = (s->prevobs[j] >> 1) + (s->currobs[j] >> 1);
        s->currobs[j] = 0;
    }
    s->obscount += s->newcount;
    s->newcount = 0;
    return 0;
}

/* parser window limit :2806-2824 / :2452-2470; returns -1 for SRCEXHSTD */
static long parse_limit(D* s, size_t* limit)
{
    size_t lim = s->inputend;
    size_t srcleft = s->srclen - s->srcpos;
    if (lim - s->cursor > LOOKAHEAD + 1) {
        if (s->flush == 0 || srcleft) lim -= LOOKAHEAD;
    } else {
        if (srcleft) lim = s->cursor;
        else if (s->flush == 0) return -1;
    }
    *limit = lim;
    return 0;
}

/* lazy parser, levels 6-9 (compress2 :2767-2973).  Returns 0 when a block
 * must be flushed (state 1). */
static int compress2(D* s)
{
    uint32_t mlen, moff, plen = 0, poff = 0;
    int hasmatch;

    if (!s->blockinit) {
        memset(s->lfrq, 0, sizeof(s->lfrq));
        memset(s->dfrq, 0, sizeof(s->dfrq));
        resetobs(s);
        s->blockinit = 1;
    }
    mlen = s->held & 0xffff;
    moff = s->held >> 16;
    hasmatch = mlen != 0;

    for (;;) {
        size_t limit;
        if (parse_limit(s, &limit) < 0) return JDO_SRCEXHSTD;

        while (limit > s->cursor) {
#ifdef JDO_STATS
            jdo_stat_step(hasmatch);
#endif
            if (!hasmatch) {
                getmatch2(s, MINMATCH - 1, s->doshort, &mlen, &moff);
                if (mlen == MINMATCH && moff > 8192) mlen = MINMATCH - 1;
                if (mlen >= MINMATCH) {
                    if (mlen >= s->good) {
                        unsigned ls = lsym_of(mlen), ds = dsym_of(moff);
                        skipbytes2(s, 1, mlen);
                        addmatch(s, mlen, moff, ls, ds);
                        obsmatch(s, mlen, ls);
                    } else {
                        hasmatch = 1;
                    }
                } else {
                    unsigned c = s->win[s->cursor];
                    addliteral(s, c);
                    obsliteral(s, c);
                }
            } else {
                int accept = 0;
                plen = mlen; poff = moff;
                getmatch2(s, plen - 1, 0, &mlen, &moff);
                if (mlen >= plen) {
                    int32_t dl = (int32_t) mlen - (int32_t) plen;
                    if (dl > 4) accept = 1;
                    else accept = (dl << 2) + (ilog2(poff) - ilog2(moff)) >= 2;
                }
                if (accept) {
                    unsigned c = s->win[s->cursor - 1];
                    addliteral(s, c);
                    obsliteral(s, c);
                } else {
                    unsigned ls = lsym_of(plen), ds = dsym_of(poff);
                    skipbytes2(s, 2, plen);
                    addmatch(s, plen, poff, ls, ds);
                    obsmatch(s, plen, ls);
                    hasmatch = 0;
                }
            }

            s->cursor++;
            if (s->zend + 4 > s->lzcap) {
                resetobs(s);
                s->held = hasmatch ? (mlen | (moff << 16)) : 0;
                s->hasinput = 1;
                return 0;
            }
            if (s->newcount >= 512 && s->obstotal >= 4096) {
#ifdef JDO_STATS
                jdo_stat_obs(s->doshort, s->currobs[0] >= 16, s->cursor);
#endif
                s->doshort = s->currobs[0] >= 16;
                if (shouldsplit(s)) {
                    s->held = hasmatch ? (mlen | (moff << 16)) : 0;
                    s->hasinput = 1;
                    return 0;
                }
            }
        }
        if (fillwindow(s)) continue;
        s->held = hasmatch ? (mlen | (moff << 16)) : 0;
        if (s->flush) { s->hasinput = 0; return 0; }
        return JDO_SRCEXHSTD;
    }
}

/* greedy match finder, levels 1-5 (getmatch1 :2335-2400) */
static void getmatch1(D* s, uint32_t* olen, uint32_t* ooff)
{
    const uint8_t* w = s->win;
    size_t cur = s->cursor, best = cur;
    size_t strend = cur + MAXMATCH;
    uint16_t pos4 = (uint16_t) (cur - s->whence4);
    int16_t next4, limit;
    uint32_t chain, length = MINMATCH;

    if (strend > s->inputend) strend = s->inputend;
    if (pos4 == WSIZE) { slidehash(s); s->whence4 += WSIZE; pos4 = 0; }
    next4 = s->mhlist[s->h4];
    s->mchain[pos4 & CHAINMASK] = s->mhlist[s->h4];
    s->mhlist[s->h4] = (int16_t) pos4;
    s->h4 = hashat(s, cur + 1, H4BITS, 0);

    limit = (int16_t) (pos4 - WSIZE);
    for (chain = s->maxchain; chain; chain--) {
        size_t q;
        if (next4 <= limit) break;
        q = (size_t) ((ptrdiff_t) s->whence4 + next4);
        if (w[cur + length] == w[q + length]) {
            uint32_t n = matchlen(w + cur, w + q);
            if (n > length) {
                length = n;
                best = q;
                if (length >= s->nice) break;
            }
        }
        next4 = s->mchain[(uint16_t) next4 & CHAINMASK];
    }
    if (cur + length > strend) length -= (uint32_t) (cur + length - strend);
    *olen = length;
    *ooff = (uint32_t) (cur - best);
}

/* skipbytes1 :2402-2428 */
static void skipbytes1(D* s, uint32_t skip, uint32_t total)
{
    for (; skip < total; skip++) {
        uint16_t pos4;
        s->cursor++;
        pos4 = (uint16_t) (s->cursor - s->whence4);
        if (pos4 == WSIZE) { slidehash(s); s->whence4 += WSIZE; pos4 = 0; }
        s->mchain[pos4 & CHAINMASK] = s->mhlist[s->h4];
        s->mhlist[s->h4] = (int16_t) pos4;
        s->h4 = hashat(s, s->cursor + 1, H4BITS, 0);
    }
}

/* greedy parser, levels 1-5 (compress1 :2431-2520) */
static int compress1(D* s)
{
    if (!s->blockinit) {
        memset(s->lfrq, 0, sizeof(s->lfrq));
        memset(s->dfrq, 0, sizeof(s->dfrq));
        s->blockinit = 1;
    }
    for (;;) {
        size_t limit;
        if (parse_limit(s, &limit) < 0) return JDO_SRCEXHSTD;
        while (limit > s->cursor) {
            uint32_t mlen, moff;
            getmatch1(s, &mlen, &moff);
            if (mlen > MINMATCH) {
                addmatch(s, mlen, moff, lsym_of(mlen), dsym_of(moff));
                skipbytes1(s, 1, mlen);
            } else {
                addliteral(s, s->win[s->cursor]);
            }
            s->cursor++;
            if (s->zend + 4 > s->lzcap) { s->hasinput = 1; return 0; }
        }
        if (fillwindow(s)) continue;
        if (s->flush) { s->hasinput = 0; return 0; }
        return JDO_SRCEXHSTD;
    }
}

/* static (fixed) codes, RFC 1951 3.2.6 (slitcodes_ etc. :2987-3114) */
static void static_codes(hcode_t* lc, hcode_t* dc)
{
    size_t f[290];
    unsigned i;
    unsigned cnt[16] = {0}, nxt[16];
    for (i = 0; i < 288; i++) f[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
    for (i = 0; i < 288; i++) cnt[f[i]]++;
    nxt[0] = 0;
    for (i = 1; i <= 15; i++) nxt[i] = (nxt[i - 1] + cnt[i - 1]) << 1;
    for (i = 0; i < 288; i++) {
        lc[i].len = (uint8_t) f[i];
        lc[i].code = (uint16_t) bitrev(nxt[f[i]]++, (unsigned) f[i]);
    }
    for (i = 0; i < 32; i++) { dc[i].len = 5; dc[i].code = (uint16_t) bitrev(i, 5); }
}

/* buildtables :1362-1390 */
static void buildtables(D* s)
{
    unsigned i;
    s->lmax = build_code(s->lfrq, 288, 15, s->lcode);
    s->dmax = build_code(s->dfrq, 32, 15, s->dcode);
    memset(s->cfrq, 0, sizeof(s->cfrq));
    rle_lengths(s->lfrq, s->lmax, s->cfrq);
    rle_lengths(s->dfrq, s->dmax, s->cfrq);
    build_code(s->cfrq, 19, 7, s->pcode);
    for (i = 18; i >= 3; i--) if (s->cfrq[kpcorder[i]]) break;
    s->cmax = i + 1;
}

/* emittrees :1634-1722 */
static void emittrees(D* s)
{
    unsigned i, t;
    putbits(s, s->lmax - 257, 5);
    putbits(s, s->dmax - 1, 5);
    putbits(s, s->cmax - 4, 4);
    for (i = 0; i < s->cmax; i++) putbits(s, (uint32_t) s->cfrq[kpcorder[i]], 3);
    for (t = 0; t < 2; t++) {
        const size_t* l = t ? s->dfrq : s->lfrq;
        size_t k = 0, sym;
        while ((sym = l[k]) != 0xffff) {
            const hcode_t* c = &s->pcode[sym];
            putbits(s, c->code, c->len);
            k++;
            if (sym >= 16) {
                unsigned nb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
                uint32_t base = sym == 18 ? 11 : 3;
                putbits(s, (uint32_t) (l[k] - base), nb);
                k++;
            }
        }
    }
}

/* flushblock :1725-1805 + emitlz :1512-1631 */
static void flushblock(D* s)
{
    hcode_t slc[288], sdc[32];
    const hcode_t* lc;
    const hcode_t* dc;
    size_t total = s->zend, k;
    int dostatic;

    if (total == 0) { s->blockinit = 0; return; }
    s->lfrq[EOBSYM]++;
    s->lz[s->zend++] = EOBSYM;

    dostatic = s->level == 1 || (s->flags & JDO_FIXEDCODES) || total < 0x400;
    if (dostatic) {
        static_codes(slc, sdc);
        lc = slc; dc = sdc;
    } else {
        buildtables(s);
        lc = s->lcode; dc = s->dcode;
    }
    tr(s, 0x40000000u | (dostatic ? 1u : 2u));

    putbits(s, 0, 1);
    putbits(s, dostatic ? 1 : 2, 2);
    if (!dostatic) emittrees(s);

    for (k = 0; k < s->zend;) {
        uint16_t t = s->lz[k];
        if (t < 0x8000) {
            putbits(s, lc[t].code, lc[t].len);
            k++;
            continue;
        } else {
            unsigned len = (unsigned) t - 0x8000u;
            unsigned off = s->lz[k + 1];
            unsigned ls = s->lz[k + 2] >> 8, ds = s->lz[k + 2] & 0xff;
            putbits(s, lc[257 + ls].code, lc[257 + ls].len);
            if (klextra[ls]) putbits(s, len - klbase[ls], klextra[ls]);
            putbits(s, dc[ds].code, dc[ds].len);
            if (kdextra[ds]) putbits(s, off - kdbase[ds], kdextra[ds]);
            k += 3;
        }
    }
    s->zend = 0;
    s->blockinit = 0;
}

/* endstream :610-654 */
static void endstream(D* s)
{
    putbits(s, s->flush == JDO_END ? 1 : 0, 1);
    putbits(s, 0, 2);
    alignbits(s);
    putbyte(s, 0x00); putbyte(s, 0x00); putbyte(s, 0xff); putbyte(s, 0xff);
}

/* stored blocks, level 0 (compress0 :796-926), whole input at once */
static void compress0(D* s)
{
    for (;;) {
        size_t room = s->wend - s->inputend;
        size_t left = s->srclen - s->srcpos;
        size_t run = 0xffff;
        size_t i;
        if (run > room) run = room;
        if (run > left) run = left;
        memcpy(s->win + s->inputend, s->src + s->srcpos, run);
        s->inputend += run;
        s->srcpos += run;
        if (run == 0 && left == 0) return;
        putbits(s, 0, 3);
        alignbits(s);
        putbyte(s, (uint8_t) run); putbyte(s, (uint8_t) (run >> 8));
        putbyte(s, (uint8_t) ~run); putbyte(s, (uint8_t) (~run >> 8));
        for (i = 0; i < run; i++) putbyte(s, s->win[s->inputend - run + i]);
        s->inputend = 0;
    }
}

/* deflator_deflate :691-786 driven to completion with the whole input */
static void run_deflate(D* s)
{
    if (s->level == 0) {
        compress0(s);
        endstream(s);
        return;
    }
    for (;;) {
        if (s->level <= 5) compress1(s); else compress2(s);
        flushblock(s);
        if (s->hasinput == 0) break;
    }
    endstream(s);
}

size_t jdo_bound(size_t n)
{
    /* stored-equivalent worst cases are far below this: 9 bits per literal,
     * <= 32 bits per 3-byte match, trees <= 300 bytes per split (>= 512
     * tokens each), the terminator and byte padding */
    return n + n / 2 + (n / 1536 + 2) * 320 + 64;
}

size_t jdo_deflate(const uint8_t* src, size_t n, int level, unsigned flags,
                   int flush, uint8_t* dst, size_t cap)
{
    D s;
    size_t r;
    if (flush != JDO_END && flush != JDO_FLUSH) return (size_t) -1;
    if (!d_init(&s, level, flags)) { d_free(&s); return (size_t) -1; }
    s.src = src;
    s.srclen = n;
    s.flush = flush;
    s.out = dst;
    s.ocap = cap;
    run_deflate(&s);
    r = s.overflow ? (size_t) -1 : s.opos;
    d_free(&s);
    return r;
}

/* deflator_setdctnr :2106-2167 on a fresh deflator, then the whole input
 * (jdo_deflate).  The dictionary's last <= 32 KiB go to window [0, size);
 * positions 0 .. size-4 enter the chains with their own hashes (position 0
 * too); the last three do not; the parse starts at `size` with the hashes
 * of the cursor still 0 (the position-0 quirk moves there). */
size_t jdo_deflate_dict(const uint8_t* dict, size_t dsize, const uint8_t* src, size_t n,
                        int level, unsigned flags, int flush, uint8_t* dst, size_t cap)
{
    D s;
    size_t r, i;
    if (flush != JDO_END && flush != JDO_FLUSH) return (size_t) -1;
    if (!d_init(&s, level, flags)) { d_free(&s); return (size_t) -1; }
    if (level && dsize) {
        if (dsize > WSIZE) { dict += dsize - WSIZE; dsize = WSIZE; }
        memcpy(s.win, dict, dsize);
        if (dsize >= 4) {
            for (i = 0; i + 4 <= dsize; i++) {
                const uint32_t h4 = hashat(&s, i, H4BITS, 0);
                s.mchain[i & CHAINMASK] = s.mhlist[h4];
                s.mhlist[h4] = (int16_t) i;
                if (level > 5) {
                    const uint32_t h3 = hashat(&s, i, H3BITS, 8);
                    s.schain[i & RING3MASK] = s.shlist[h3];
                    s.shlist[h3] = (uint16_t) i;
                }
            }
        }
        s.inputend = dsize;
        s.cursor = dsize;
    }
    s.src = src;
    s.srclen = n;
    s.flush = flush;
    s.out = dst;
    s.ocap = cap;
    run_deflate(&s);
    r = s.overflow ? (size_t) -1 : s.opos;
    d_free(&s);
    return r;
}

/* compress0 :796-926 for one deflator_deflate call: stored blocks of up to
 * 65535 bytes (and the window's room), kept open across calls without a
 * flush; a flush closes the open block.  Returns JDO_SRCEXHSTD or 0. */
static int compress0_call(D* s)
{
    for (;;) {
        const size_t outleft = s->wend - s->inputend;
        const size_t srcleft = s->srclen - s->srcpos;
        size_t run = 0xffff - s->acc0, i;
        if (run > outleft) run = outleft;
        if (run > srcleft) run = srcleft;
        memcpy(s->win + s->inputend, s->src + s->srcpos, run);
        s->inputend += run;
        s->srcpos += run;
        s->acc0 += run;
        if (s->flush) {
            if (s->acc0 == 0 && srcleft == 0) return 0;
        } else if (s->acc0 < 0xffff) {
            return JDO_SRCEXHSTD;
        }
        putbits(s, 0, 3);
        alignbits(s);
        putbyte(s, (uint8_t) s->acc0); putbyte(s, (uint8_t) (s->acc0 >> 8));
        putbyte(s, (uint8_t) ~s->acc0); putbyte(s, (uint8_t) (~s->acc0 >> 8));
        for (i = 0; i < s->acc0; i++) putbyte(s, s->win[s->inputend - s->acc0 + i]);
        s->acc0 = 0;
        s->inputend = 0;
    }
}

/* deflator_deflate :691-786 once per call of a sequence: call k hands
 * src[ends[k-1], ends[k]) with flush mode flushes[k] (JDO_NOFLUSH, JDO_FLUSH
 * or JDO_END; the flush latch :697-699 applies); the window, chains and
 * parser state carry from call to call, and a JDO_FLUSH leaves the state at 0
 * with the window kept (:763-768).  The outputs are concatenated.  Returns
 * the total, or (size_t)-1 (cap too small, bad arguments, or a call after the
 * stream ended). */
size_t jdo_deflate_calls(const uint8_t* dict, size_t dsize, const uint8_t* src,
                         const size_t* ends, const int* flushes, size_t ncalls,
                         int level, unsigned flags, uint8_t* dst, size_t cap)
{
    D s;
    size_t r, i, k;
    int state = 0, dead = 0;
    if (!d_init(&s, level, flags)) { d_free(&s); return (size_t) -1; }
    if (level && dict && dsize) {
        /* deflator_setdctnr :2106-2167, as jdo_deflate_dict */
        if (dsize > WSIZE) { dict += dsize - WSIZE; dsize = WSIZE; }
        memcpy(s.win, dict, dsize);
        if (dsize >= 4) {
            for (i = 0; i + 4 <= dsize; i++) {
                const uint32_t h4 = hashat(&s, i, H4BITS, 0);
                s.mchain[i & CHAINMASK] = s.mhlist[h4];
                s.mhlist[h4] = (int16_t) i;
                if (level > 5) {
                    const uint32_t h3 = hashat(&s, i, H3BITS, 8);
                    s.schain[i & RING3MASK] = s.shlist[h3];
                    s.shlist[h3] = (uint16_t) i;
                }
            }
        }
        s.inputend = dsize;
        s.cursor = dsize;
    }
    s.src = src;
    s.out = dst;
    s.ocap = cap;
    for (k = 0; k < ncalls && !dead; k++) {
        const int f = flushes[k];
        if (f != JDO_NOFLUSH && f != JDO_FLUSH && f != JDO_END) { dead = 2; break; }
        if ((k && ends[k] < ends[k - 1]) || ends[k] < s.srcpos) { dead = 2; break; }
        s.srclen = ends[k];
        if (f && (s.flush == 0 || s.flush == JDO_FLUSH)) s.flush = f;
        for (;;) {
            if (state == 0) {
                int rc;
                if (level == 0) {
                    rc = compress0_call(&s);
                    if (rc == JDO_SRCEXHSTD) break;
                    state = 2;
                    continue;
                }
                rc = level <= 5 ? compress1(&s) : compress2(&s);
                if (rc == JDO_SRCEXHSTD) break;
                state = 1;
            }
            if (state == 1) {
                flushblock(&s);
                state = 0;
                if (s.flush && !s.hasinput) state = 2;
                continue;
            }
            /* state 2: endstream :758-773 */
            endstream(&s);
            if (s.flush == JDO_FLUSH) {
                state = 0;
                s.flush = 0;
            } else {
                dead = 1;
            }
            break;
        }
    }
    r = (s.overflow || dead == 2 || (dead && k < ncalls)) ? (size_t) -1 : s.opos;
    d_free(&s);
    return r;
}

size_t jdo_trace(const uint8_t* src, size_t n, int level, unsigned flags,
                 uint32_t* out, size_t cap)
{
    D s;
    size_t r;
    uint8_t* scratch;
    if (!d_init(&s, level, flags)) { d_free(&s); return 0; }
    scratch = (uint8_t*) malloc(jdo_bound(n) + 64);
    s.src = src; s.srclen = n; s.flush = JDO_END;
    s.out = scratch; s.ocap = jdo_bound(n) + 64;
    s.trace = out; s.tracecap = cap;
    run_deflate(&s);
    r = s.ntrace < cap ? s.ntrace : cap;
    free(scratch);
    d_free(&s);
    return r;
}

size_t jdo_deflate_blocks(const uint8_t* src, size_t n, size_t blocksize,
                          int level, unsigned flags, uint8_t* dst, size_t cap,
                          uint32_t* sizes)
{
    size_t nb = n ? (n + blocksize - 1) / blocksize : 1, i, total = 0;
    for (i = 0; i < nb; i++) {
        size_t off = i * blocksize;
        size_t len = n - off < blocksize ? n - off : blocksize;
        size_t r;
        if (n == 0) len = 0;
        r = jdo_deflate(src + off, len, level, flags,
                        i + 1 == nb ? JDO_END : JDO_FLUSH, dst + total,
                        cap - total);
        if (r == (size_t) -1) return r;
        if (sizes) sizes[i] = (uint32_t) r;
        total += r;
    }
    return total;
}

/* ------------------------------------------------------------------------ */
/* inflator (inflator.c:381-568 buildtable, :765-1518 block decoding)        */
/* ------------------------------------------------------------------------ */
/* decode table entry: bits 0-7 code length, 8-11 extra bits, 12 literal,
 * 13 end of block, 14 subtable (then bits 0-7 = total bits of the subtable,
 * 16-31 its offset), 16-31 value (literal byte / base).  0 = invalid. */
#define E_LIT 0x1000u
#define E_END 0x2000u
#define E_SUB 0x4000u

enum { T_LIT = 0, T_DIST = 1, T_PRE = 2 };

/* canonical decode table with `root` root bits; acceptance rules of
 * buildtable :424-474.  Returns 0 ok, 1 error. */
static int build_decode(const uint16_t* lens, unsigned n, unsigned mode,
                        unsigned root, uint32_t* tab, unsigned tabcap)
{
    unsigned cnt[16] = {0}, nxt[16], sublen[1024];
    unsigned i, mlen, used;
    long left;
    uint32_t code;

    memset(tab, 0, tabcap * sizeof(uint32_t));
    for (i = 0; i < n; i++) cnt[lens[i]]++;
    if (cnt[0] == n) return mode == T_DIST ? 0 : 1;
    cnt[0] = 0;
    for (mlen = 15; cnt[mlen] == 0; mlen--) {}
    left = 1;
    for (i = 1; i <= 15; i++) {
        left = (left << 1) - (long) cnt[i];
        if (left < 0) return 1;
    }
    if (left && (mlen != 1 || mode != T_DIST)) return 1;

    code = 0;
    nxt[0] = 0;
    for (i = 1; i <= 15; i++) { code = (code + cnt[i - 1]) << 1; nxt[i] = code; }

    /* pass 1: subtable widths per root prefix */
    memset(sublen, 0, sizeof(sublen));
    {
        unsigned tmp[16];
        memcpy(tmp, nxt, sizeof(tmp));
        for (i = 0; i < n; i++) {
            unsigned l = lens[i];
            if (l > root) {
                uint32_t c = bitrev(tmp[l], l);
                unsigned r = c & ((1u << root) - 1);
                if (l - root > sublen[r]) sublen[r] = l - root;
            }
            if (l) tmp[l]++;
        }
    }
    used = 1u << root;
    for (i = 0; i < (1u << root); i++) {
        if (sublen[i]) {
            if (used + (1u << sublen[i]) > tabcap) return 1;
            tab[i] = E_SUB | (used << 16) | (root + sublen[i]);
            used += 1u << sublen[i];
        }
    }
    /* pass 2: fill */
    for (i = 0; i < n; i++) {
        unsigned l = lens[i];
        uint32_t e, c;
        if (!l) continue;
        if (mode == T_PRE) e = (i << 16) | l;
        else if (mode == T_LIT && i < 256) e = E_LIT | (i << 16) | l;
        else if (mode == T_LIT && i == 256) e = E_END | l;
        else if (mode == T_LIT) {
            unsigned k = i - 257;
            /* symbols 286/287 (static only): zero-length matches,
             * inflator.c:351-352 */
            e = k < 29 ? ((uint32_t) klbase[k] << 16) | ((uint32_t) klextra[k] << 8) | l : l;
        } else {
            /* distance symbols 30/31 (static only): base 0, :372 */
            e = i < 30 ? ((uint32_t) kdbase[i] << 16) | ((uint32_t) kdextra[i] << 8) | l : l;
        }
        c = bitrev(nxt[l]++, l);
        if (l <= root) {
            uint32_t k;
            for (k = c; k < (1u << root); k += 1u << l) tab[k] = e;
        } else {
            uint32_t s = tab[c & ((1u << root) - 1)];
            unsigned sb = (s & 0xff) - root, off = s >> 16;
            uint32_t sc = c >> root, k;
            for (k = sc; k < (1u << sb); k += 1u << (l - root)) tab[off + k] = e;
        }
    }
    return 0;
}

typedef struct {
    const uint8_t* src;
    size_t n;
    size_t bitpos;
    uint8_t* dst;
    size_t cap, o;
} I;

static size_t avail_bits(const I* z) { return z->n * 8 - z->bitpos; }

/* peek up to 24 bits, zero padded past the end of the input */
static uint32_t peek(const I* z, unsigned nb)
{
    uint32_t v = 0;
    size_t byte = z->bitpos >> 3;
    unsigned sh = (unsigned) (z->bitpos & 7), k;
    for (k = 0; k < 4; k++)
        if (byte + k < z->n) v |= (uint32_t) z->src[byte + k] << (8 * k);
    v >>= sh;
    return nb >= 32 ? v : v & ((1u << nb) - 1);
}

/* decode one symbol; returns entry, or 0 with *err set */
static uint32_t decode_sym(I* z, const uint32_t* tab, unsigned root, int* err)
{
    uint32_t b = peek(z, 15);
    uint32_t e = tab[b & ((1u << root) - 1)];
    if (e & E_SUB) e = tab[(e >> 16) + ((b & ((1u << (e & 0xff)) - 1)) >> root)];
    if ((e & 0xff) == 0) { *err = 2; return 0; }            /* EBADCODE  */
    if ((e & 0xff) > avail_bits(z)) { *err = 6; return 0; } /* EINPUTEND */
    z->bitpos += e & 0xff;
    return e;
}

static int getbits(I* z, unsigned nb, uint32_t* v)
{
    if (nb > avail_bits(z)) return 0;
    *v = peek(z, nb);
    z->bitpos += nb;
    return 1;
}

/* decodednmc :1104-1190 + readlengths :1030-1101 */
static int read_dynamic(I* z, uint32_t* lt, uint32_t* dt)
{
    uint16_t lens[320 + 8];
    uint32_t pre[128];
    uint32_t hl, hd, hc, v;
    unsigned i, idx;
    int err = 0;

    if (!getbits(z, 14, &v)) return 6;
    hl = (v & 31) + 257; hd = ((v >> 5) & 31) + 1; hc = (v >> 10) + 4;
    if (hl > 286 || hd > 30) return 3;
    memset(lens, 0, sizeof(lens));
    for (i = 0; i < hc; i++) {
        if (!getbits(z, 3, &v)) return 6;
        lens[kpcorder[i]] = (uint16_t) v;
    }
    if (build_decode(lens, 19, T_PRE, 7, pre, 128)) return 3;

    memset(lens, 0, sizeof(lens));
    idx = 0;
    while (idx < hl + hd) {
        uint32_t e, sl, rep, nb, base;
        uint32_t b = peek(z, 7);
        e = pre[b];
        if ((e & 0xff) > avail_bits(z)) return 6;
        z->bitpos += e & 0xff;
        sl = e >> 16;
        if (sl < 16) { lens[idx++] = (uint16_t) sl; continue; }
        nb = sl == 16 ? 2 : sl == 17 ? 3 : 7;
        base = sl == 18 ? 11 : 3;
        if (!getbits(z, nb, &rep)) return 6;
        rep += base;
        if (sl == 16) {
            if (idx == 0) return 3;
            v = lens[idx - 1];
        } else {
            v = 0;
        }
        if (idx + rep > 320) return 3;
        while (rep--) lens[idx++] = (uint16_t) v;
    }
    if (lens[256] == 0) return 3;
    if (build_decode(lens, hl, T_LIT, 10, lt, 2048)) return 3;
    if (build_decode(lens + hl, hd, T_DIST, 8, dt, 1024)) return 3;
    (void) err;
    return 0;
}

/* Huffman block body: decodeblock :1330 / decodefast :1530 semantics for
 * valid data; a zero-length match (static symbols 286/287) emits nothing,
 * an offset-0 copy (static distance 30/31) emits zero bytes (the reference
 * copies uninitialised target bytes there). */
static int inflate_codes(I* z, const uint32_t* lt, const uint32_t* dt)
{
    for (;;) {
        /* the fast loop of decodefast :1530-1823: with >= 16 input bytes
         * and >= 266 output bytes ahead a token needs no bound checks; the
         * bit reader is one 64-bit load (>= 57 bits, a token needs <= 48).
         * A token it cannot take plainly (an invalid code, an offset of 0 or
         * past the output's start) is left unconsumed for the checked loop
         * below, which reports it exactly as before. */
        while (z->n - (z->bitpos >> 3) >= 16 && z->cap - z->o >= 266) {
            uint64_t w;
            uint32_t e, f, used, len, off;
            memcpy(&w, z->src + (z->bitpos >> 3), 8);
            w >>= z->bitpos & 7;
            e = lt[w & 1023];
            if (e & E_SUB) e = lt[(e >> 16) + ((w & ((1u << (e & 0xff)) - 1)) >> 10)];
            used = e & 0xff;
            if (!used) break;
            if (e & E_LIT) {
                z->dst[z->o++] = (uint8_t) (e >> 16);
                z->bitpos += used;
                continue;
            }
            if (e & E_END) {
                z->bitpos += used;
                return 0;
            }
            len = (e >> 16) + (uint32_t) ((w >> used) & ((1u << ((e >> 8) & 15)) - 1));
            used += (e >> 8) & 15;
            f = dt[(w >> used) & 255];
            if (f & E_SUB) f = dt[(f >> 16) + (((w >> used) & ((1u << (f & 0xff)) - 1)) >> 8)];
            if (!(f & 0xff)) break;
            off = (f >> 16) + (uint32_t) ((w >> (used + (f & 0xff))) & ((1u << ((f >> 8) & 15)) - 1));
            if (off == 0 || off > z->o) break;
            z->bitpos += used + (f & 0xff) + ((f >> 8) & 15);
            {
                uint8_t* d = z->dst + z->o;
                const uint8_t* q = d - off;
                uint32_t k;
                if (off >= 8) {
                    for (k = 0; k < len; k += 8) memcpy(d + k, q + k, 8);
                } else {
                    for (k = 0; k < len; k++) d[k] = q[k];
                }
                z->o += len;
            }
        }
        int err = 0;
        uint32_t e = decode_sym(z, lt, 10, &err), v, len, off;
        if (!e) return err;
        if (e & E_LIT) {
            if (z->o >= z->cap) return -2;
            z->dst[z->o++] = (uint8_t) (e >> 16);
            continue;
        }
        if (e & E_END) return 0;
        if (!getbits(z, (e >> 8) & 15, &v)) return 6;
        len = (e >> 16) + v;
        e = decode_sym(z, dt, 8, &err);
        if (!e) return err;
        if (!getbits(z, (e >> 8) & 15, &v)) return 6;
        off = (e >> 16) + v;
        if (off > z->o) return 4;                           /* EFAROFFSET */
        if (z->o + len > z->cap) return -2;
        while (len--) {
            z->dst[z->o] = off ? z->dst[z->o - off] : 0;
            z->o++;
        }
    }
}

static uint32_t slt[2048], sdt[1024];
static pthread_once_t sonce = PTHREAD_ONCE_INIT;

/* setstatictables :686-721 */
static void static_decode_init(void)
{
    uint16_t l[288];
    unsigned i;
    for (i = 0; i < 288; i++) l[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
    build_decode(l, 288, T_LIT, 10, slt, 2048);
    for (i = 0; i < 32; i++) l[i] = 5;
    build_decode(l, 32, T_DIST, 8, sdt, 1024);
}

static int inflate_run(I* z, int stop_at_input_end, int* finalseen)
{
    uint32_t lt[2048], dt[1024];
    uint32_t v;

    pthread_once(&sonce, static_decode_init);
    *finalseen = 0;
    for (;;) {
        int r;
        uint32_t fin, type;
        if (stop_at_input_end && ((z->bitpos + 7) >> 3) >= z->n) return 0;
        if (!getbits(z, 3, &v)) return 6;
        fin = v & 1;
        type = v >> 1;
        if (type == 0) {
            uint32_t a, b;
            size_t i;
            z->bitpos = (z->bitpos + 7) & ~(size_t) 7;
            if (!getbits(z, 16, &a) || !getbits(z, 16, &b)) return 6;
            if ((a ^ 0xffff) != b) return 5;               /* EBADBLOCK  */
            {
                size_t have = avail_bits(z) >> 3, cp = a < have ? a : have;
                if (z->o + cp > z->cap) return -2;
                for (i = 0; i < cp; i++) {
                    z->dst[z->o++] = z->src[z->bitpos >> 3];
                    z->bitpos += 8;
                }
                if (cp < a) return 6;
            }
        } else if (type == 1) {
            r = inflate_codes(z, slt, sdt);
            if (r) return r;
        } else if (type == 2) {
            r = read_dynamic(z, lt, dt);
            if (r) return r;
            r = inflate_codes(z, lt, dt);
            if (r) return r;
        } else {
            return 5;
        }
        if (fin) { *finalseen = 1; return 0; }
    }
}

int jdo_inflate(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                size_t* consumed, size_t* produced, int* error)
{
    I z;
    int r, fin;
    z.src = src; z.n = n; z.bitpos = 0; z.dst = dst; z.cap = cap; z.o = 0;
    r = inflate_run(&z, 0, &fin);
    if (consumed) *consumed = (z.bitpos + 7) >> 3;
    if (produced) *produced = z.o;
    if (error) *error = r > 0 ? r : 0;
    if (r == -2) return JDO_TGTEXHSTD;
    return r ? JDO_ERROR : JDO_OK;
}

int jdo_inflate_blocks(const uint8_t* src, const uint32_t* csizes,
                       size_t nblocks, size_t blocksize, uint8_t* dst,
                       uint32_t* usizes, int32_t* errors)
{
    size_t i, off = 0;
    int bad = 0;
    for (i = 0; i < nblocks; i++) {
        I z;
        int r, fin;
        z.src = src + off; z.n = csizes[i]; z.bitpos = 0;
        z.dst = dst + i * blocksize; z.cap = blocksize; z.o = 0;
        r = inflate_run(&z, 1, &fin);
        if (r == -2) r = 9;     /* block inflates past blocksize (jdgpu.h) */
        if (usizes) usizes[i] = (uint32_t) z.o;
        if (errors) errors[i] = r;
        bad += r != 0;
        off += csizes[i];
    }
    return bad;
}

/* ------------------------------------------------------------------------ */
/* pthread CPU baseline (one instance per thread, striped)    */
/* ------------------------------------------------------------------------ */
typedef struct {
    const uint8_t* src; size_t n, bs; int level; uint8_t* dst; size_t slot;
    uint32_t* sizes; const uint64_t* coff; const uint32_t* csz; size_t nb;
    int tid, nt, bad;
} job_t;

static void* defl_worker(void* p)
{
    job_t* j = (job_t*) p;
    size_t nb = (j->n + j->bs - 1) / j->bs, i;
    for (i = (size_t) j->tid; i < nb; i += (size_t) j->nt) {
        size_t off = i * j->bs, len = j->n - off < j->bs ? j->n - off : j->bs;
        size_t r = jdo_deflate(j->src + off, len, j->level, 0,
                               i + 1 == nb ? JDO_END : JDO_FLUSH,
                               j->dst + i * j->slot, j->slot);
        j->sizes[i] = (uint32_t) r;
        if (r == (size_t) -1) j->bad++;
    }
    return NULL;
}

static void* infl_worker(void* p)
{
    job_t* j = (job_t*) p;
    size_t i;
    for (i = (size_t) j->tid; i < j->nb; i += (size_t) j->nt) {
        I z;
        int r, fin;
        z.src = j->src + j->coff[i]; z.n = j->csz[i]; z.bitpos = 0;
        z.dst = j->dst + i * j->bs; z.cap = j->bs; z.o = 0;
        r = inflate_run(&z, 1, &fin);
        if (r) j->bad++;
    }
    return NULL;
}

static int run_threads(job_t* proto, int threads, void* (*fn)(void*))
{
    pthread_t th[256];
    job_t jobs[256];
    int t, bad = 0;
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    for (t = 0; t < threads; t++) {
        jobs[t] = *proto;
        jobs[t].tid = t;
        jobs[t].nt = threads;
        jobs[t].bad = 0;
        pthread_create(&th[t], NULL, fn, &jobs[t]);
    }
    for (t = 0; t < threads; t++) { pthread_join(th[t], NULL); bad += jobs[t].bad; }
    return bad;
}

size_t jdo_deflate_blocks_mt(const uint8_t* src, size_t n, size_t blocksize,
                             int level, uint8_t* dst, size_t slotcap,
                             uint32_t* sizes, int threads)
{
    job_t j;
    size_t nb = (n + blocksize - 1) / blocksize, i, total = 0;
    memset(&j, 0, sizeof(j));
    j.src = src; j.n = n; j.bs = blocksize; j.level = level; j.dst = dst;
    j.slot = slotcap; j.sizes = sizes;
    if (run_threads(&j, threads, defl_worker)) return (size_t) -1;
    for (i = 0; i < nb; i++) total += sizes[i];
    return total;
}

int jdo_inflate_blocks_mt(const uint8_t* src, const uint64_t* coffsets,
                          const uint32_t* csizes, size_t nblocks,
                          size_t blocksize, uint8_t* dst, int threads)
{
    job_t j;
    memset(&j, 0, sizeof(j));
    j.src = src; j.coff = coffsets; j.csz = csizes; j.nb = nblocks;
    j.bs = blocksize; j.dst = dst;
    return run_threads(&j, threads, infl_worker);
}
