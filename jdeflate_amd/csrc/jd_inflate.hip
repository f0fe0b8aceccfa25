/*
 * jd_inflate.hip -- gfx950 inflate of independent blocks.
 *
 * One wave per compressed block.  The Huffman decode (inflator.c
 * decodeblock :1330 / decodefast :1530) is inherently serial inside a block,
 * so the 64 lanes run it in lockstep on identical (uniform) state and split
 * the work that is parallel: table construction (buildtable :381-568),
 * stored-block copies and back-reference copies.  A back-reference of any
 * length and distance is copied in one pass: lane i writes
 * out[pos + i] = out[pos - off + (i mod off)], which only reads bytes that
 * existed before the match (RFC 1951 overlap semantics).
 *
 * Decode tables live in LDS as 16-bit entries: bit 15 = subtable link
 * (bits 0-3 subtable bits, 4-14 offset), otherwise bits 0-3 = code length
 * (0 = no such code) and bits 4-12 = symbol.
 *
 * Error codes are inflator.h:57-66; acceptance rules follow buildtable
 * :424-474, decodednmc :1122-1186, readlengths :1042-1098, decodestrd
 * :945-1019.  Block-level semantics: decode until the block's compressed
 * bytes are exhausted at a deflate-block boundary, or until BFINAL.
 */
#include "jd_device.h"
#include "jd_kernels.h"
#include "jd_prof.h"

#define LROOT 10
#define DROOT 8
#define PROOT 7
#define LT_CAP 1344
#define DT_CAP 416
#define E_SUB 0x8000u

enum { E_OK = 0, E_BADSTATE = 1, E_BADCODE = 2, E_BADTREE = 3, E_FAROFFSET = 4,
       E_BADBLOCK = 5, E_INPUTEND = 6, E_OVERFLOW = 9 };

__constant__ uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct InfShared {
    uint32_t cnt[16], nxt[16];
    uint16_t lt[LT_CAP];
    uint16_t dt[DT_CAP];
    uint16_t pt[128];
    uint16_t codes[320];
    uint8_t lens[336];
    uint32_t flag;
};

struct Reader {
    const uint8_t* in;
    uint64_t inlen;
    uint64_t start;   /* absolute offset of the block               */
    uint32_t clen;    /* compressed bytes of the block              */
    uint64_t bb;      /* bits [ip*8 - bc, ip*8)                     */
    uint32_t bc;
    uint32_t ip;
    uint32_t nw;      /* the 4 bytes at ip (prefetched)             */
};

__device__ static inline uint32_t rd_load4(const Reader& r, uint32_t ip)
{
    if (ip >= r.clen) return 0;
    const uint64_t A = r.start + ip;
    uint32_t v;
    if ((A & ~3ull) + 8 <= r.inlen) {
        const uint32_t* p = (const uint32_t*) (r.in + (A & ~3ull));
        v = __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t) (A & 3));
    } else {
        v = 0;
        for (uint32_t k = 0; k < 4; k++)
            if (A + k < r.inlen) v |= (uint32_t) r.in[A + k] << (8 * k);
    }
    const uint32_t left = r.clen - ip;
    if (left < 4) v &= (1u << (8 * left)) - 1;
    return v;
}

__device__ static inline void rd_init(Reader& r, uint32_t byte)
{
    r.bb = 0;
    r.bc = 0;
    r.ip = byte;
    r.nw = rd_load4(r, byte);
}

__device__ static inline void rd_fill(Reader& r)
{
    if (r.bc <= 32) {
        r.bb |= (uint64_t) r.nw << r.bc;
        r.bc += 32;
        r.ip += 4;
        r.nw = rd_load4(r, r.ip);
    }
}

/* consumed bit position */
__device__ static inline uint64_t rd_pos(const Reader& r) { return (uint64_t) r.ip * 8 - r.bc; }
__device__ static inline uint64_t rd_avail(const Reader& r) { return (uint64_t) r.clen * 8 - rd_pos(r); }

/* read nb (<= 24) bits; false if the input is exhausted */
__device__ static inline bool rd_bits(Reader& r, uint32_t nb, uint32_t* v)
{
    rd_fill(r);
    if (nb > rd_avail(r)) return false;
    *v = (uint32_t) r.bb & ((1u << nb) - 1);
    r.bb >>= nb;
    r.bc -= nb;
    return true;
}

/* decode one symbol; returns symbol or -code */
__device__ static inline int rd_sym(Reader& r, const uint16_t* tab, uint32_t root)
{
    rd_fill(r);
    uint32_t e = tab[(uint32_t) r.bb & ((1u << root) - 1)];
    if (e & E_SUB)
        e = tab[((e >> 4) & 0x7ff) + (((uint32_t) r.bb >> root) & ((1u << (e & 15)) - 1))];
    const uint32_t L = e & 15;
    if (L == 0) return -E_BADCODE;
    if (L > rd_avail(r)) return -E_INPUTEND;
    r.bb >>= L;
    r.bc -= L;
    return (int) ((e >> 4) & 0x1ff);
}

/* decode table from code lengths (buildtable :381-568 acceptance rules).
 * mode 0 lit/len, 1 distance, 2 precode.  Returns 0 or E_BADTREE.  Called
 * by the whole wave. */
__device__ static uint32_t build_table(InfShared& s, const uint8_t* lens,
                                       uint32_t n, uint32_t root, uint16_t* tab,
                                       uint32_t cap, int mode)
{
    const uint32_t lane = threadIdx.x;
    for (uint32_t i = lane; i < cap; i += 64) tab[i] = 0;
    __syncthreads();
    if (lane == 0) {
        uint32_t* cnt = s.cnt;
        uint32_t* nxt = s.nxt;
        for (int i = 0; i < 16; i++) cnt[i] = 0;
        for (uint32_t i = 0; i < n; i++) cnt[lens[i]]++;
        uint32_t bad = 0;
        if (cnt[0] == n) {
            bad = mode == 1 ? 0 : 1;
            n = 0;   /* empty distance table */
        } else {
            cnt[0] = 0;
            uint32_t mlen = 15;
            while (cnt[mlen] == 0) mlen--;
            int left = 1;
            for (int i = 1; i <= 15; i++) {
                left = (left << 1) - (int) cnt[i];
                if (left < 0) { bad = 1; break; }
            }
            if (!bad && left && (mlen != 1 || mode != 1)) bad = 1;
            if (!bad) {
                uint32_t code = 0;
                nxt[0] = 0;
                for (int i = 1; i <= 15; i++) { code = (code + cnt[i - 1]) << 1; nxt[i] = code; }
                const uint32_t rmask = (1u << root) - 1;
                for (uint32_t i = 0; i < n; i++) {
                    const uint32_t l = lens[i];
                    if (!l) continue;
                    const uint32_t c = jd_rev(nxt[l]++, l);
                    s.codes[i] = (uint16_t) c;
                    if (l > root) {
                        const uint32_t p = c & rmask;
                        const uint32_t sb = l - root;
                        const uint32_t cur = tab[p] & 15;
                        tab[p] = (uint16_t) (E_SUB | (sb > cur ? sb : cur));
                    }
                }
                uint32_t off = 1u << root;
                for (uint32_t p = 0; p <= rmask; p++) {
                    const uint32_t e = tab[p];
                    if (e & E_SUB) {
                        const uint32_t sb = e & 15;
                        if (off + (1u << sb) > cap) { bad = 1; break; }
                        tab[p] = (uint16_t) (E_SUB | (off << 4) | sb);
                        off += 1u << sb;
                    }
                }
            }
        }
        s.flag = bad ? 0xffffffffu : n;
    }
    __syncthreads();
    const uint32_t st = s.flag;
    __syncthreads();
    if (st == 0xffffffffu) return E_BADTREE;
    n = st;
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t l = lens[i];
        if (!l) continue;
        const uint32_t c = s.codes[i];
        const uint16_t e = (uint16_t) ((i << 4) | l);
        if (l <= root) {
            for (uint32_t k = c; k < (1u << root); k += 1u << l) tab[k] = e;
        } else {
            const uint32_t P = tab[c & ((1u << root) - 1)];
            const uint32_t off = (P >> 4) & 0x7ff, sb = P & 15;
            for (uint32_t k = c >> root; k < (1u << sb); k += 1u << (l - root)) tab[off + k] = e;
        }
    }
    __syncthreads();
    return 0;
}

__device__ static uint32_t build_static(InfShared& s)
{
    for (uint32_t i = threadIdx.x; i < 288; i += 64)
        s.lens[i] = i < 144 ? 8 : i < 256 ? 9 : i < 280 ? 7 : 8;
    __syncthreads();
    uint32_t r = build_table(s, s.lens, 288, LROOT, s.lt, LT_CAP, 0);
    if (threadIdx.x < 32) s.lens[threadIdx.x] = 5;
    __syncthreads();
    r |= build_table(s, s.lens, 32, DROOT, s.dt, DT_CAP, 1);
    return r;
}

/* dynamic block header (decodednmc :1104-1190, readlengths :1030-1101) */
__device__ static uint32_t read_dynamic(InfShared& s, Reader& r)
{
    uint32_t v;
    if (!rd_bits(r, 14, &v)) return E_INPUTEND;
    const uint32_t hl = (v & 31) + 257, hd = ((v >> 5) & 31) + 1, hc = (v >> 10) + 4;
    if (hl > 286 || hd > 30) return E_BADTREE;
    for (uint32_t i = threadIdx.x; i < 336; i += 64) s.lens[i] = 0;
    __syncthreads();
    for (uint32_t i = 0; i < hc; i++) {
        if (!rd_bits(r, 3, &v)) return E_INPUTEND;
        if (threadIdx.x == 0) s.lens[kOrder[i]] = (uint8_t) v;
    }
    __syncthreads();
    if (build_table(s, s.lens, 19, PROOT, s.pt, 128, 2)) return E_BADTREE;
    for (uint32_t i = threadIdx.x; i < 336; i += 64) s.lens[i] = 0;
    __syncthreads();
    uint32_t idx = 0, prevlen = 0;
    while (idx < hl + hd) {
        const int sym = rd_sym(r, s.pt, PROOT);
        if (sym < 0) return (uint32_t) -sym;
        if (sym < 16) {
            if (threadIdx.x == 0) s.lens[idx] = (uint8_t) sym;
            prevlen = (uint32_t) sym;
            idx++;
            continue;
        }
        const uint32_t nb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
        const uint32_t base = sym == 18 ? 11 : 3;
        if (!rd_bits(r, nb, &v)) return E_INPUTEND;
        const uint32_t rep = base + v;
        uint32_t val = 0;
        if (sym == 16) {
            if (idx == 0) return E_BADTREE;
            val = prevlen;
        }
        if (idx + rep > 320) return E_BADTREE;
        for (uint32_t k = threadIdx.x; k < rep; k += 64) s.lens[idx + k] = (uint8_t) val;
        prevlen = val;
        idx += rep;
    }
    __syncthreads();
    if (s.lens[256] == 0) return E_BADTREE;
    if (build_table(s, s.lens, hl, LROOT, s.lt, LT_CAP, 0)) return E_BADTREE;
    /* the distance lengths follow the literal/length ones */
    for (uint32_t i = threadIdx.x; i < hd; i += 64) s.lens[i] = s.lens[hl + i];
    __syncthreads();
    if (build_table(s, s.lens, hd, DROOT, s.dt, DT_CAP, 1)) return E_BADTREE;
    return E_OK;
}

__device__ static inline uint8_t out_byte_l2(const uint8_t* p)
{
    /* L1-bypassing (sc1) read of bytes this wave stored earlier */
    const uint32_t* w = (const uint32_t*) ((uintptr_t) p & ~(uintptr_t) 3);
    const uint32_t x = __hip_atomic_load((uint32_t*) w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (uint8_t) (x >> (8 * ((uintptr_t) p & 3)));
}

__global__ __launch_bounds__(64) void k_inflate(JdInflateLaunch a)
{
    __shared__ InfShared s;
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    Reader r;
    r.in = a.in;
    r.inlen = a.inlen;
    r.start = a.coff[b];
    r.clen = a.csize[b];
    rd_init(r, 0);
    uint8_t* out = a.out + (uint64_t) b * a.bs;
    const uint32_t cap = a.bs;
    uint32_t pos = 0, vis = 0, err = E_OK;

    for (;;) {
        /* stop cleanly at the end of the block's bytes (FLUSH-joined
         * streams end every block with a byte-aligned empty stored block) */
        if (rd_pos(r) + 7 >= (uint64_t) r.clen * 8) {
            if (a.require_final) err = E_INPUTEND;
            break;
        }
        uint32_t hdr;
        if (!rd_bits(r, 3, &hdr)) { err = E_INPUTEND; break; }
        const uint32_t fin = hdr & 1, type = hdr >> 1;
        if (type == 0) {
            /* stored (decodestrd :931-1019) */
            const uint64_t bp = (rd_pos(r) + 7) & ~7ull;
            const uint32_t byte = (uint32_t) (bp >> 3);
            rd_init(r, byte);
            uint32_t ln, nln;
            if (!rd_bits(r, 16, &ln) || !rd_bits(r, 16, &nln)) { err = E_INPUTEND; break; }
            if ((ln ^ 0xffff) != nln) { err = E_BADBLOCK; break; }
            const uint32_t at = byte + 4;
            const uint32_t have = at < r.clen ? r.clen - at : 0;
            const uint32_t cp = min(ln, have);
            if (pos + cp > cap) { err = E_OVERFLOW; break; }
            for (uint32_t i = lane; i < cp; i += 64) out[pos + i] = r.in[r.start + at + i];
            pos += cp;
            if (cp < ln) { err = E_INPUTEND; break; }
            rd_init(r, at + ln);
        } else if (type == 1 || type == 2) {
            if (type == 1) err = build_static(s);
            else err = read_dynamic(s, r);
            if (err) break;
            for (;;) {
                const int sym = rd_sym(r, s.lt, LROOT);
                if (sym < 0) { err = (uint32_t) -sym; break; }
                if (sym < 256) {
                    if (pos >= cap) { err = E_OVERFLOW; break; }
                    if (lane == 0) out[pos] = (uint8_t) sym;
                    pos++;
                    continue;
                }
                if (sym == 256) break;
                const uint32_t ls = (uint32_t) sym - 257;
                uint32_t len = 0, v;
                if (ls < 29) {
                    if (!rd_bits(r, jd_lextra(ls), &v)) { err = E_INPUTEND; break; }
                    len = jd_lbase(ls) + v;
                } /* 286/287 (static only): zero-length match, inflator.c:351 */
                const int dsy = rd_sym(r, s.dt, DROOT);
                if (dsy < 0) { err = (uint32_t) -dsy; break; }
                uint32_t off = 0;
                if (dsy < 30) {
                    if (!rd_bits(r, jd_dextra((uint32_t) dsy), &v)) { err = E_INPUTEND; break; }
                    off = jd_dbase((uint32_t) dsy) + v;
                } /* 30/31 (static only): distance 0, inflator.c:372 */
                if (off > pos) { err = E_FAROFFSET; break; }
                if (pos + len > cap) { err = E_OVERFLOW; break; }
                if (!len) continue;
                const uint32_t span = min(len, off ? off : len);
                if (off && pos - off + span > vis) {
                    /* make every earlier store of this wave visible */
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    vis = pos;
                }
                for (uint32_t i = lane; i < len; i += 64) {
                    uint8_t c = 0;
                    if (off) c = out_byte_l2(out + pos - off + (i % off));
                    out[pos + i] = c;
                }
                pos += len;
            }
            if (err) break;
        } else {
            err = E_BADBLOCK;
            break;
        }
        if (fin) break;
    }
    if (lane == 0) {
        a.usize[b] = pos;
        a.err[b] = (int32_t) err;
        if (a.used) a.used[b] = (uint32_t) ((rd_pos(r) + 7) >> 3);
    }
}

extern "C" int jdk_inflate_launch(const JdInflateLaunch* L)
{
    if (!L->nblocks) return 0;
    hipStream_t st = (hipStream_t) L->stream;
    JDPROF_RUN(JDK_INFLATE, st, (k_inflate<<<L->nblocks, 64, 0, st>>>(*L)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
