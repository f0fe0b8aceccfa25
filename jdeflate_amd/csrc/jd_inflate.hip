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
    /* the decode tables first: k_inflate_par overlays the header scratch
     * behind them with its sync bitmaps (ParShared) */
    uint16_t lt[LT_CAP];
    uint16_t dt[DT_CAP];
    uint32_t cnt[16], nxt[16];
    uint16_t pt[128];
    uint16_t codes[320];
    uint8_t lens[336];
    uint32_t flag;
};

#define RD_LW 1024u    /* LDS input window of the wave-uniform decoders, dwords */

struct Reader {
    const uint8_t* in;
    uint64_t inlen;
    uint64_t start;   /* absolute offset of the block               */
    uint32_t clen;    /* compressed bytes of the block              */
    uint64_t bb;      /* bits [ip*8 - bc, ip*8)                     */
    uint32_t bc;
    uint32_t ip;
    uint32_t nw;      /* the 4 bytes at ip (prefetched)             */
    /* optional LDS window over the input (NULL: read global memory):
     * lw[i] = the 4 bytes at absolute offset wa + 4 i.  A serial decoder
     * would otherwise wait a full global-load latency every few tokens. */
    uint32_t* lw;
    uint64_t wa;
    uint32_t lwn;     /* the window's size in dwords (a multiple of 4)  */
};

/* refill the LDS window to start at A (wave-uniform; every lane loads 16-byte
 * pieces, bytes past the input read as zero) */
__device__ __attribute__((always_inline)) static void rd_window(Reader& r, uint64_t A)
{
    const uint64_t wa = A & ~15ull;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < r.lwn / 4; k += 64) {
        const uint64_t g = wa + (uint64_t) k * 16;
        uint4 q = make_uint4(0, 0, 0, 0);
        if (g + 16 <= r.inlen) {
            JD_CHECK(r.in + g, 16, r.in + r.inlen);
            q = *(const uint4*) (r.in + g);
        } else {
            uint8_t t[16];
            for (uint32_t j = 0; j < 16; j++) t[j] = g + j < r.inlen ? r.in[g + j] : 0;
            __builtin_memcpy(&q, t, 16);
        }
        *(uint4*) (r.lw + 4 * k) = q;
    }
    __syncthreads();
    r.wa = wa;
}

__device__ static inline uint32_t rd_load4(Reader& r, uint32_t ip)
{
    if (ip >= r.clen) return 0;
    const uint64_t A = r.start + ip;
    uint32_t v;
    if (r.lw) {
        if (A < r.wa || A + 8 > r.wa + 4 * r.lwn) rd_window(r, A);
        const uint32_t o = (uint32_t) (A - r.wa);
        v = __builtin_amdgcn_alignbyte(r.lw[(o >> 2) + 1], r.lw[o >> 2], o & 3);
    } else if ((A & ~3ull) + 8 <= r.inlen) {
        JD_CHECK(r.in + (A & ~3ull), 8, r.in + r.inlen);
        const uint32_t* p = (const uint32_t*) (r.in + (A & ~3ull));
        v = __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t) (A & 3));
    } else {
        v = 0;
        for (uint32_t k = 0; k < 4; k++)
            if (A + k < r.inlen) v |= (uint32_t) r.in[A + k] << (8 * k);
    }
    /* returned as loaded: rd_fill masks the bytes past clen and makes it
     * wave-uniform when it uses the word, one refill later, so a global load
     * is in flight while the 32 bits before it are decoded (taking it into
     * a scalar register here waited for it at once) */
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
        /* the reader's state is wave-uniform: keep it in scalar registers,
         * so the decode loops branch on SCC instead of exec masks */
        uint32_t w = __builtin_amdgcn_readfirstlane(r.nw);
        const uint32_t left = r.clen - r.ip;          /* r.nw holds the bytes at r.ip */
        if (left < 4) w &= (1u << (8 * left)) - 1;
        r.bb |= (uint64_t) w << r.bc;
        r.bc += 32;
        r.ip += 4;
        r.nw = rd_load4(r, r.ip);
    }
}

/* the reader's state is the same on every lane: say so, so that the
 * compiler keeps it (and what is computed from it) in scalar registers and
 * the decode loops branch on SCC rather than exec masks */
__device__ static inline uint32_t jd_uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ static inline uint64_t jd_uni64(uint64_t x)
{
    return ((uint64_t) jd_uni((uint32_t) (x >> 32)) << 32) | jd_uni((uint32_t) x);
}
__device__ static inline void rd_uniform(Reader& r)
{
    r.bb = jd_uni64(r.bb);
    r.bc = jd_uni(r.bc);
    r.ip = jd_uni(r.ip);
    r.nw = jd_uni(r.nw);
    r.wa = jd_uni64(r.wa);
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
    uint32_t e = __builtin_amdgcn_readfirstlane(tab[(uint32_t) r.bb & ((1u << root) - 1)]);
    if (e & E_SUB)
        e = __builtin_amdgcn_readfirstlane(
            tab[((e >> 4) & 0x7ff) + (((uint32_t) r.bb >> root) & ((1u << (e & 15)) - 1))]);
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
    /* wave 0 builds (with more waves present, they take the barriers only);
     * the serial steps of buildtable (:381-568) become a histogram, a rank
     * per code length by ballots, and a scan over the root entries */
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const bool w0 = tid < 64;
    for (uint32_t i = tid; i < cap; i += blockDim.x) tab[i] = 0;
    if (tid < 16) s.cnt[tid] = 0;
    __syncthreads();
    if (w0)
        for (uint32_t i = lane; i < n; i += 64) atomicAdd(&s.cnt[lens[i]], 1u);
    __syncthreads();
    if (tid == 0) {
        uint32_t* cnt = s.cnt;
        uint32_t* nxt = s.nxt;
        uint32_t bad = 0;
        if (cnt[0] == n) {
            bad = mode == 1 ? 0 : 1;
            n = 0;   /* empty distance table */
        } else {
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
                for (int i = 1; i <= 15; i++) { code = (code + (i > 1 ? cnt[i - 1] : 0)) << 1; nxt[i] = code; }
            }
        }
        s.flag = bad ? 0xffffffffu : n;
    }
    __syncthreads();
    const uint32_t st = s.flag;
    if (st == 0xffffffffu) {
        __syncthreads();
        return E_BADTREE;
    }
    n = st;
    const uint32_t rsize = 1u << root, rmask = rsize - 1;
    if (w0) {
        /* code of symbol i = first code of its length + its rank among the
         * symbols of that length (lanes 1-15 keep the running counts) */
        uint32_t base = 0;
        for (uint32_t c0 = 0; c0 < n; c0 += 64) {
            const uint32_t i = c0 + lane;
            const uint32_t l = i < n ? lens[i] : 0u;
            uint64_t mym = 0;
            uint32_t cl = 0;
#pragma unroll
            for (uint32_t L = 1; L <= 15; L++) {
                const uint64_t m = __ballot(l == L);
                if (l == L) mym = m;
                if (lane == L) cl = (uint32_t) __popcll(m);
            }
            const uint32_t before = (uint32_t) __popcll(mym & ((1ull << lane) - 1));
            const uint32_t bl = (uint32_t) __shfl((int) base, (int) l);
            if (l) s.codes[i] = (uint16_t) jd_rev(s.nxt[l] + bl + before, l);
            base += cl;
        }
    }
    __syncthreads();
    /* root entries with a subtable: the widest code under each (lane 0, over
     * the few codes longer than the root), then the subtables laid out in
     * root order by a scan over the root entries */
    uint32_t bad = 0;
    if (w0) {
        for (uint32_t c0 = 0; c0 < n; c0 += 64) {
            const uint32_t i = c0 + lane;
            uint64_t m = __ballot(i < n && lens[i] > root);
            if (lane == 0) {
                while (m) {
                    const uint32_t k = (uint32_t) __builtin_ctzll(m);
                    m &= m - 1;
                    const uint32_t j = c0 + k, l = lens[j];
                    const uint32_t pfx = s.codes[j] & rmask, sb = l - root, cur = tab[pfx] & 15;
                    tab[pfx] = (uint16_t) (E_SUB | (sb > cur ? sb : cur));
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xc07f);      /* lgkmcnt(0): lane 0's marks */
        const uint32_t per = rsize >= 64 ? rsize / 64 : 1u;
        const uint32_t p0 = lane * per;
        uint32_t mine = 0;
        for (uint32_t k = 0; k < per && p0 + k < rsize; k++) {
            const uint32_t e = tab[p0 + k];
            if (e & E_SUB) mine += 1u << (e & 15);
        }
        uint32_t inc = mine;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t x = (uint32_t) __shfl_up((int) inc, d);
            if (lane >= d) inc += x;
        }
        const uint32_t total = (uint32_t) __shfl((int) inc, 63);
        uint32_t off = rsize + inc - mine;
        for (uint32_t k = 0; k < per && p0 + k < rsize; k++) {
            const uint32_t e = tab[p0 + k];
            if (e & E_SUB) {
                const uint32_t sb = e & 15;
                tab[p0 + k] = (uint16_t) (E_SUB | (off << 4) | sb);
                off += 1u << sb;
            }
        }
        bad = rsize + total > cap;
        if (tid == 0) s.flag = bad ? 0xffffffffu : 0u;
    }
    __syncthreads();
    if (s.flag == 0xffffffffu) {
        __syncthreads();
        return E_BADTREE;
    }
    if (w0)
        for (uint32_t i = lane; i < n; i += 64) {
            const uint32_t l = lens[i];
            if (!l) continue;
            const uint32_t c = s.codes[i];
            const uint16_t e = (uint16_t) ((i << 4) | l);
            if (l <= root) {
                for (uint32_t k = c; k < rsize; k += 1u << l) tab[k] = e;
            } else {
                const uint32_t P = tab[c & rmask];
                const uint32_t o = (P >> 4) & 0x7ff, sb = P & 15;
                for (uint32_t k = c >> root; k < (1u << sb); k += 1u << (l - root)) tab[o + k] = e;
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
__device__ __attribute__((always_inline)) static uint32_t read_dynamic(InfShared& s, Reader& r)
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

/* 32-bit decode entries for the fast loops, made from a block's 16-bit
 * tables: F_SUB | subtable link (as the 16-bit one); F_LIT | literal << 16;
 * F_EOB; or base << 16 | extra bits << 8 (length or distance).  Bits 0-3 =
 * code length, 0 = no such code. */
#define F_SUB 0x80000000u
#define F_LIT 0x40000000u
#define F_EOB 0x20000000u

__device__ static void fast_tables(const InfShared& s, uint32_t* lt32, uint32_t* dt32)
{
    for (uint32_t i = threadIdx.x; i < LT_CAP; i += 64) {
        const uint32_t e = s.lt[i];
        const uint32_t L = e & 15, sym = (e >> 4) & 0x1ff;
        uint32_t f = 0;
        if (e & E_SUB) f = F_SUB | (e & 0x7fff);
        else if (!L) f = 0;
        else if (sym < 256) f = F_LIT | (sym << 16) | L;
        else if (sym == 256) f = F_EOB | L;
        else if (sym - 257 < 29) f = (jd_lbase(sym - 257) << 16) | (jd_lextra(sym - 257) << 8) | L;
        else f = L;             /* 286/287 (static only): zero-length match */
        lt32[i] = f;
    }
    for (uint32_t i = threadIdx.x; i < DT_CAP; i += 64) {
        const uint32_t e = s.dt[i];
        const uint32_t L = e & 15, sym = (e >> 4) & 0x1ff;
        uint32_t f = 0;
        if (e & E_SUB) f = F_SUB | (e & 0x7fff);
        else if (!L) f = 0;
        else if (sym < 30) f = (jd_dbase(sym) << 16) | (jd_dextra(sym) << 8) | L;
        else f = L;             /* 30/31 (static only): distance 0 */
        dt32[i] = f;
    }
    __syncthreads();
}

/* scope of the loads that read bytes this wave stored: the wave runs on one
 * CU, whose write-through L1 and XCD L2 see its own stores, so workgroup
 * scope (a plain load) suffices; agent scope would bypass the per-XCD L2 and
 * read HBM (measured 7.9 GiB of fetches per GiB resolved) */
#ifndef JD_RSCOPE
#define JD_RSCOPE __HIP_MEMORY_SCOPE_WORKGROUP
#endif
#define JD_GLOBAL __attribute__((address_space(1)))

__device__ static inline uint8_t out_byte_l2(const uint8_t* p)
{
    /* read of a byte this wave stored earlier (JD_RSCOPE) */
    const uint32_t* w = (const uint32_t*) ((uintptr_t) p & ~(uintptr_t) 3);
    const uint32_t x = __hip_atomic_load((JD_GLOBAL uint32_t*) w, __ATOMIC_RELAXED, JD_RSCOPE);
    return (uint8_t) (x >> (8 * ((uintptr_t) p & 3)));
}

__global__ __launch_bounds__(64) void k_inflate(JdInflateLaunch a)
{
    __shared__ InfShared s;
    __shared__ __attribute__((aligned(16))) uint32_t lwin[RD_LW];
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (a.fb && !a.fb[b]) return;         /* fallback pass: flagged blocks only */
    Reader r;
    r.in = a.in;
    r.inlen = a.inlen;
    r.start = a.coff[b];
    r.clen = a.csize[b];
    r.lw = lwin;
    r.lwn = RD_LW;
    r.wa = ~0ull;
    rd_init(r, 0);
    uint8_t* out = a.out + (uint64_t) b * a.bs;
    const uint32_t cap = a.bs;
    uint32_t pos = a.pos0, vis = a.pos0, err = E_OK, sawfin = 0;
    if (a.bit0) {
        /* resumed stream: the first bit0 bits belong to the previous call */
        uint32_t v;
        if (!rd_bits(r, a.bit0, &v)) err = E_INPUTEND;
    }
    /* start of the last deflate block begun (resume point, inflator.c:800) */
    uint64_t hbit = a.bit0;
    uint32_t hout = pos;

    while (!err) {
        hbit = rd_pos(r);
        hout = pos;
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
            for (uint32_t i = lane; i < cp; i += 64) {
                JD_CHECK(r.in + r.start + at + i, 1, r.in + r.inlen);
                out[pos + i] = r.in[r.start + at + i];
            }
            pos += cp;
            if (cp < ln) { err = E_INPUTEND; break; }
            rd_init(r, at + ln);
        } else if (type == 1 || type == 2) {
            if (type == 1) err = build_static(s);
            else err = read_dynamic(s, r);
            if (err) break;
            for (;;) {
                rd_uniform(r);
                pos = jd_uni(pos);
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
                if (off >= len) {
                    for (uint32_t i = lane; i < len; i += 64) out[pos + i] = out_byte_l2(out + pos - off + i);
                } else {
                    for (uint32_t i = lane; i < len; i += 64) {
                        uint8_t c = 0;
                        if (off) c = out_byte_l2(out + pos - off + (i % off));
                        out[pos + i] = c;
                    }
                }
                pos += len;
            }
            if (err) break;
        } else {
            err = E_BADBLOCK;
            break;
        }
        if (fin) { sawfin = 1; break; }
    }
    if (lane == 0) {
        a.usize[b] = pos;
        a.err[b] = (int32_t) err;
        if (a.used) a.used[b] = (uint32_t) ((rd_pos(r) + 7) >> 3);
        if (a.fin) a.fin[b] = sawfin | ((rd_pos(r) & 7) ? 2u : 0u);
        if (a.hdr) {
            a.hdr[2 * b] = hbit;
            a.hdr[2 * b + 1] = hout;
        }
    }
}

/* ======================================================================== */
/* Resumable single-stream decoder (the drop-in inflator_inflate,
 * inflator.c:765-903).  One wave decodes wave-uniformly as k_inflate does,
 * but from a state that an earlier launch left in device memory (JdInfState:
 * block mode, final flag, the current block's decode tables, a pending
 * back-reference copy, the stored-block remainder), and every stop leaves
 * such a state with the exact bit to continue from:
 *   - the input ends inside a token            -> NEEDINPUT at that token's
 *     first bit (the reference keeps the bits in its bit buffer, decodeblock
 *     :1381-1400; nothing decoded twice beyond that partial token);
 *   - the input ends inside a block header     -> NEEDINPUT at the header's
 *     first bit (headers are read whole);
 *   - the input ends inside stored data        -> NEEDINPUT after the bytes
 *     copied (decodestrd :988-1010);
 *   - the output reaches `cap`                 -> FULL, with a literal left
 *     undecoded or a back-reference split into a pending copy (copybytes
 *     :1214-1290);
 *   - the final block's end-of-block           -> ENDED;
 *   - optionally, a header that follows an empty stored block (a sync
 *     marker) with >= markmin input bytes left -> MARKER (the host decodes
 *     the FLUSH-joined rest in parallel from there);
 *   - corrupt data                             -> ERROR (inflator.h codes).
 * The window (<= 32 KiB of earlier output, or the dictionary) is out[-pos0,
 * 0): back-references reach it as they reach this launch's own bytes.
 * ======================================================================== */
static_assert(LT_CAP == JD_RS_LT && DT_CAP == JD_RS_DT, "JdInfState table sizes");

/* the last 64 KiB of output, in LDS: back-references read here instead of
 * re-reading the wave's own global stores (which needs a vmcnt drain and an
 * L2 round trip per copy) */
#define RS_RING 65536u

/* the state's head (the fields the host decides on) also into host-pinned
 * memory, by the thread that just wrote it: the host then waits for the
 * launch alone instead of a launch and a copy back */
__device__ static inline void head_to_host(const JdInfState* S, JdInfState* H)
{
    if (!H) return;
    H->mode = S->mode;
    H->fin = S->fin;
    H->plen = S->plen;
    H->poff = S->poff;
    H->srem = S->srem;
    H->status = S->status;
    H->err = S->err;
    H->pad = S->pad;
    H->bit = S->bit;
    H->produced = S->produced;
}

__global__ __launch_bounds__(64) void k_inflate_resume(JdResumeLaunch a)
{
    __shared__ InfShared s;
    __shared__ __attribute__((aligned(16))) uint8_t ring[RS_RING];
    __shared__ __attribute__((aligned(16))) uint32_t lwin[RD_LW];
    __shared__ uint32_t lt32[LT_CAP], dt32[DT_CAP];
    const uint32_t lane = threadIdx.x;
    JdInfState* S = a.st;
    Reader r;
    r.in = a.in;
    r.inlen = a.inlen;
    r.start = 0;
    r.clen = a.inlen;
    r.lw = lwin;
    r.lwn = RD_LW;
    r.wa = ~0ull;
    rd_init(r, (uint32_t) (a.bitpos >> 3));
    uint8_t* out = a.out - a.pos0;
    const uint32_t lim = a.pos0 + a.cap;
    uint32_t pos = a.pos0, vis = a.pos0;
    uint32_t mode = S->mode, fin = S->fin, plen = S->plen, poff = S->poff, srem = S->srem;
    uint32_t status = JD_RST_NEEDINPUT, err = 0, v = 0;
    uint64_t sbit = a.bitpos;
    bool marker = false, newtab = false;

    if (mode == JD_RS_HUFF) {
        for (uint32_t i = lane; i < LT_CAP; i += 64) s.lt[i] = S->lt[i];
        for (uint32_t i = lane; i < DT_CAP; i += 64) s.dt[i] = S->dt[i];
        __syncthreads();
        fast_tables(s, lt32, dt32);
    }
    /* the window (<= 32 KiB before pos0) into the ring */
    for (uint32_t i = lane; i < a.pos0; i += 64) ring[i & (RS_RING - 1)] = out[i];
    __syncthreads();
    (void) vis;
    /* bytes [pos, pos + len) <- distance off (RFC 1951 overlap semantics):
     * lane i copies pos - off + (i mod off), a byte that existed before the
     * match; the ring holds 64 KiB, so no destination of this copy aliases a
     * source (off <= 32768, len <= 258) */
    auto copy = [&](uint32_t len, uint32_t off) {
        if (off >= len) {
            for (uint32_t i = lane; i < len; i += 64) {
                const uint8_t c = ring[(pos - off + i) & (RS_RING - 1)];
                out[pos + i] = c;
                ring[(pos + i) & (RS_RING - 1)] = c;
            }
        } else {
            for (uint32_t i = lane; i < len; i += 64) {
                uint8_t c = 0;
                if (off) c = ring[(pos - off + (i % off)) & (RS_RING - 1)];
                out[pos + i] = c;
                ring[(pos + i) & (RS_RING - 1)] = c;
            }
        }
        __builtin_amdgcn_wave_barrier();
        pos += len;
    };

    if ((a.bitpos & 7) && !rd_bits(r, (uint32_t) (a.bitpos & 7), &v)) goto done;
    for (;;) {
        if (mode == JD_RS_ENDED) {
            status = JD_RST_ENDED;
            sbit = rd_pos(r);
            break;
        }
        if (mode == JD_RS_HEADER) {
            const uint64_t hb = rd_pos(r);
            sbit = hb;
            if ((marker && a.markmin && (uint64_t) r.clen * 8 - hb >= (uint64_t) a.markmin * 8) ||
                (hb >= a.stopat && hb > a.bitpos)) {
                status = JD_RST_MARKER;
                break;
            }
            marker = false;
            if (!rd_bits(r, 3, &v)) break;                       /* NEEDINPUT */
            fin = v & 1;
            const uint32_t type = v >> 1;
            if (type == 0) {
                /* decodestrd :931-1019 */
                const uint32_t byte = (uint32_t) ((rd_pos(r) + 7) >> 3);
                rd_init(r, byte);
                uint32_t ln, nln;
                if (!rd_bits(r, 16, &ln) || !rd_bits(r, 16, &nln)) break;   /* NEEDINPUT */
                if ((ln ^ 0xffff) != nln) { status = JD_RST_ERROR; err = E_BADBLOCK; break; }
                rd_init(r, byte + 4);
                srem = ln;
                marker = ln == 0;
                mode = JD_RS_STORED;
                continue;
            }
            if (type == 3) { status = JD_RST_ERROR; err = E_BADBLOCK; break; }
            const uint32_t e2 = type == 1 ? build_static(s) : read_dynamic(s, r);
            if (e2 == E_INPUTEND) break;                          /* NEEDINPUT */
            if (e2) { status = JD_RST_ERROR; err = e2; break; }
            fast_tables(s, lt32, dt32);
            mode = JD_RS_HUFF;
            plen = 0;
            newtab = true;
            continue;
        }
        if (mode == JD_RS_STORED) {
            const uint32_t at = (uint32_t) (rd_pos(r) >> 3);
            const uint32_t have = at < r.clen ? r.clen - at : 0;
            const uint32_t n = min(srem, min(have, lim - pos));
            for (uint32_t i = lane; i < n; i += 64) {
                JD_CHECK(r.in + at + i, 1, r.in + r.inlen);
                const uint8_t c = r.in[at + i];
                out[pos + i] = c;
                ring[(pos + i) & (RS_RING - 1)] = c;
            }
            __builtin_amdgcn_wave_barrier();
            pos += n;
            srem -= n;
            rd_init(r, at + n);
            if (srem == 0) {
                mode = fin ? JD_RS_ENDED : JD_RS_HEADER;
                continue;
            }
            sbit = (uint64_t) (at + n) * 8;
            status = pos == lim ? JD_RST_FULL : JD_RST_NEEDINPUT;
            break;
        }
        /* Huffman block body: a pending copy first */
        if (plen) {
            const uint32_t n = min(plen, lim - pos);
            copy(n, poff);
            plen -= n;
            if (plen || a.stopcopy) {
                status = JD_RST_FULL;
                sbit = rd_pos(r);
                break;
            }
        }
        bool stop = false;
        for (;;) {
            /* fast tokens (as k_fsp_decode): >= 16 input bytes and >= 258
             * output bytes of room; a token the fast loop cannot finish
             * (bad code, distance too far) is rolled back and redone below,
             * where the error is reported at its first bit */
            bool eob = false;
            if (r.ip + 16 <= r.clen && pos + 258 <= lim) {
                {
                    const uint64_t A = r.start + r.ip;
                    if (A < r.wa || A + 16 > r.wa + 4 * RD_LW) rd_window(r, A);
                }
                uint64_t bb = jd_uni64(r.bb);
                uint32_t bc = jd_uni(r.bc), ip = jd_uni(r.ip), nw = jd_uni(r.nw);
                uint32_t p = jd_uni(pos);
                const uint32_t iplim = r.clen - 16, plim = lim - 258;
                const uint32_t wend = jd_uni((uint32_t) (r.wa + 4 * RD_LW - r.start)) - 16;
                const uint32_t wb = jd_uni((uint32_t) (r.wa - r.start));
                const uint32_t ilim = min(iplim, wend);
                uint32_t n = 0;                          /* tokens that need no check */
                for (;;) {
                    if (!n) {
                        if (p > plim || ip > ilim) break;
                        n = min((ilim - ip) >> 3, (plim - p) / 258u) + 1;
                    }
                    n--;
                    const uint64_t sbb = bb;
                    const uint32_t sbc = bc, sip = ip, snw = nw;
                    if (bc <= 32) {
                        bb |= (uint64_t) nw << bc;
                        bc += 32;
                        ip += 4;
                        const uint32_t o = ip - wb;
                        nw = jd_uni(__builtin_amdgcn_alignbyte(lwin[(o >> 2) + 1], lwin[o >> 2], o & 3));
                    }
                    uint32_t e = jd_uni(lt32[(uint32_t) bb & ((1u << LROOT) - 1)]);
                    if (e & F_SUB)
                        e = jd_uni(lt32[((e >> 4) & 0x7ff) + (((uint32_t) bb >> LROOT) & ((1u << (e & 15)) - 1))]);
                    const uint32_t L = e & 15;
                    if (!L) { bb = sbb; bc = sbc; ip = sip; nw = snw; break; }
                    bb >>= L;
                    bc -= L;
                    if (e & F_LIT) {
                        /* every lane stores the same byte to the same address */
                        out[p] = (uint8_t) (e >> 16);
                        ring[p & (RS_RING - 1)] = (uint8_t) (e >> 16);
                        p++;
                        continue;
                    }
                    if (e & F_EOB) { eob = true; break; }
                    const uint32_t xl = (e >> 8) & 15;
                    const uint32_t len = (e >> 16) + ((uint32_t) bb & ((1u << xl) - 1));
                    bb >>= xl;
                    bc -= xl;
                    if (bc <= 32) {
                        bb |= (uint64_t) nw << bc;
                        bc += 32;
                        ip += 4;
                        const uint32_t o = ip - wb;
                        nw = jd_uni(__builtin_amdgcn_alignbyte(lwin[(o >> 2) + 1], lwin[o >> 2], o & 3));
                    }
                    uint32_t d = jd_uni(dt32[(uint32_t) bb & ((1u << DROOT) - 1)]);
                    if (d & F_SUB)
                        d = jd_uni(dt32[((d >> 4) & 0x7ff) + (((uint32_t) bb >> DROOT) & ((1u << (d & 15)) - 1))]);
                    const uint32_t Ld = d & 15;
                    const uint32_t xd = (d >> 8) & 15;
                    const uint32_t off = (d >> 16) + ((uint32_t) (bb >> Ld) & ((1u << xd) - 1));
                    if (!Ld || off > p) { bb = sbb; bc = sbc; ip = sip; nw = snw; break; }
                    bb >>= Ld + xd;
                    bc -= Ld + xd;
                    if (!len) continue;
                    if (off >= len) {
                        for (uint32_t i0 = 0; i0 < len; i0 += 64) {
                            const uint32_t i = i0 + lane;
                            if (i < len) {
                                const uint8_t c = ring[(p - off + i) & (RS_RING - 1)];
                                out[p + i] = c;
                                ring[(p + i) & (RS_RING - 1)] = c;
                            }
                        }
                    } else {
                        for (uint32_t i0 = 0; i0 < len; i0 += 64) {
                            const uint32_t i = i0 + lane;
                            if (i < len) {
                                const uint8_t c = off ? ring[(p - off + (i % off)) & (RS_RING - 1)] : 0;
                                out[p + i] = c;
                                ring[(p + i) & (RS_RING - 1)] = c;
                            }
                        }
                    }
                    __builtin_amdgcn_wave_barrier();
                    p += len;
                }
                r.bb = bb;
                r.bc = bc;
                r.ip = ip;
                r.nw = nw;
                pos = p;
            }
            if (eob) {
                mode = fin ? JD_RS_ENDED : JD_RS_HEADER;
                break;
            }
            rd_uniform(r);
            pos = jd_uni(pos);
            const uint64_t tb = rd_pos(r);
            const int sym = rd_sym(r, s.lt, LROOT);
            if (sym < 0) {
                sbit = tb;
                if (sym != -E_INPUTEND) { status = JD_RST_ERROR; err = (uint32_t) -sym; }
                stop = true;
                break;
            }
            if (sym < 256) {
                if (pos >= lim) { status = JD_RST_FULL; sbit = tb; stop = true; break; }
                if (lane == 0) {
                    out[pos] = (uint8_t) sym;
                    ring[pos & (RS_RING - 1)] = (uint8_t) sym;
                }
                __builtin_amdgcn_wave_barrier();
                pos++;
                continue;
            }
            if (sym == 256) {
                mode = fin ? JD_RS_ENDED : JD_RS_HEADER;
                break;
            }
            const uint32_t ls = (uint32_t) sym - 257;
            uint32_t len = 0;
            if (ls < 29) {
                if (!rd_bits(r, jd_lextra(ls), &v)) { sbit = tb; stop = true; break; }
                len = jd_lbase(ls) + v;
            } /* 286/287 (static only): zero-length match, inflator.c:351 */
            const int dsy = rd_sym(r, s.dt, DROOT);
            if (dsy < 0) {
                sbit = tb;
                if (dsy != -E_INPUTEND) { status = JD_RST_ERROR; err = (uint32_t) -dsy; }
                stop = true;
                break;
            }
            uint32_t off = 0;
            if (dsy < 30) {
                if (!rd_bits(r, jd_dextra((uint32_t) dsy), &v)) { sbit = tb; stop = true; break; }
                off = jd_dbase((uint32_t) dsy) + v;
            } /* 30/31 (static only): distance 0, inflator.c:372 */
            if (off > pos) { status = JD_RST_ERROR; err = E_FAROFFSET; sbit = tb; stop = true; break; }
            if (!len) continue;
            const uint32_t n = min(len, lim - pos);
            copy(n, off);
            if (n < len) {
                plen = len - n;
                poff = off;
                status = JD_RST_FULL;
                sbit = rd_pos(r);
                stop = true;
                break;
            }
        }
        if (stop) break;
    }
done:
    if (lane == 0) {
        S->mode = mode;
        S->fin = fin;
        S->plen = plen;
        S->poff = poff;
        S->srem = srem;
        S->status = status;
        S->err = (int32_t) err;
        S->bit = sbit;
        S->produced = pos - a.pos0;
        head_to_host(S, a.hhead);
    }
    if (newtab && mode == JD_RS_HUFF) {
        for (uint32_t i = lane; i < LT_CAP; i += 64) S->lt[i] = s.lt[i];
        for (uint32_t i = lane; i < DT_CAP; i += 64) S->dt[i] = s.dt[i];
    }
}

extern "C" int jdk_inflate_resume_launch(const JdResumeLaunch* L)
{
    hipStream_t st = (hipStream_t) L->stream;
    JdResumeLaunch a = *L;
    JDPROF_RUN(JDK_INFLATE, st, (k_inflate_resume<<<1, 64, 0, st>>>(a)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* ======================================================================== */
/* Parallel decode of a stream without sync markers (JdFspLaunch).
 *
 * k_fsp_find: one workgroup per search region, one candidate bit per lane
 * per round; the first candidate of the region that passes wins.  The checks
 * are the decoder's own acceptance rules for a dynamic block header, so a
 * true header always passes; a false one (random bits that pass every rule)
 * is caught later because no exact chunk ends a block on it.
 * ======================================================================== */
#define FSP_FIND_T 256u



/* The search reads the input through an LDS tile: FSP_TILE bytes of
 * candidate positions plus FSP_MARGIN bytes, more than the longest header
 * (17 + 57 + 316 x 14 bits < 4,500 bits) */
#define FSP_TILE 8192u
#define FSP_MARGIN 640u

struct FspBits {
    const uint32_t* tile;       /* dword i = input bytes tb/8 + 4i (tb 32-bit aligned) */
    uint64_t at, buf;           /* at: bit offset from the tile start */
    uint32_t nb;
    __device__ uint32_t peek(uint32_t n)
    {
        if (nb < n) {
            const uint32_t w = (uint32_t) (at >> 5), sh = (uint32_t) (at & 31);
            buf = (((uint64_t) tile[w + 1] << 32) | tile[w]) >> sh;
            if (sh) buf |= (uint64_t) tile[w + 2] << (64 - sh);
            nb = 64;
        }
        return (uint32_t) buf & ((1u << n) - 1);
    }
    __device__ void skip(uint32_t n) { buf >>= n; nb -= n; at += n; }
    __device__ uint32_t get(uint32_t n) { const uint32_t v = peek(n); skip(n); return v; }
};

/* the cheap part of fsp_header: block type, HLIT/HDIST ranges and a
 * complete precode (about 1 position in 100 of compressed data passes) */
__device__ static bool fsp_quick(const uint32_t* tile, uint32_t b)
{
    FspBits R{tile, b, 0, 0};
    if ((R.get(3) >> 1) != 2) return false;
    const uint32_t v = R.get(14);
    if ((v & 31) > 29 || ((v >> 5) & 31) > 29) return false;
    const uint32_t hc = (v >> 10) + 4;
    uint32_t ks = 0;
    for (uint32_t i = 0; i < hc; i++) {
        const uint32_t l = R.get(3);
        if (l) ks += 128u >> l;
    }
    return ks == 128;
}

/* does a dynamic block header that read_dynamic + build_table accept start
 * at bit b?  tab: this lane's 128-byte precode table */
__device__ static bool fsp_header(const uint32_t* tile, uint32_t b, uint8_t* tab)
{
    FspBits R{tile, b, 0, 0};
    if ((R.get(3) >> 1) != 2) return false;
    const uint32_t v = R.get(14);
    const uint32_t hl = (v & 31) + 257, hd = ((v >> 5) & 31) + 1, hc = (v >> 10) + 4;
    if (hl > 286 || hd > 30) return false;
    /* precode lengths, 3 bits per symbol; complete (buildtable mode 2) */
    uint64_t pl = 0;
    for (uint32_t i = 0; i < hc; i++) pl |= (uint64_t) R.get(3) << (3 * kOrder[i]);
    uint32_t ks = 0;
    for (uint32_t sy = 0; sy < 19; sy++) {
        const uint32_t l = (uint32_t) (pl >> (3 * sy)) & 7;
        if (l) ks += 128u >> l;
    }
    if (ks != 128) return false;
    uint32_t code = 0;
    for (uint32_t l = 1; l <= 7; l++) {
        for (uint32_t sy = 0; sy < 19; sy++) {
            if (((uint32_t) (pl >> (3 * sy)) & 7) != l) continue;
            for (uint32_t k = jd_rev(code, l); k < 128; k += 1u << l) tab[k] = (uint8_t) ((l << 5) | sy);
            code++;
        }
        code <<= 1;
    }
    /* literal/length and distance lengths (readlengths; repeats bounded by
     * 320), Kraft sums in units of 2^-15: lit/len complete with a code for
     * 256; distance empty, complete, or one code of length 1 */
    uint32_t idx = 0, prev = 0, lsum = 0, dsum = 0, dmax = 0;
    bool l256 = false;
    while (idx < hl + hd) {
        const uint32_t e = tab[R.peek(7)];
        R.skip(e >> 5);
        const uint32_t sy = e & 31;
        uint32_t val = 0, rep = 1;
        if (sy < 16) val = sy;
        else if (sy == 16) {
            if (idx == 0) return false;
            val = prev;
            rep = 3 + R.get(2);
        } else rep = sy == 17 ? 3 + R.get(3) : 11 + R.get(7);
        if (idx + rep > 320) return false;
        if (val) {
            const uint32_t e1 = min(idx + rep, hl);
            const uint32_t nl = e1 > idx ? e1 - idx : 0;
            const uint32_t s2 = max(idx, hl), e2 = min(idx + rep, hl + hd);
            const uint32_t nd = e2 > s2 ? e2 - s2 : 0;
            lsum += nl << (15 - val);
            dsum += nd << (15 - val);
            if (nd && val > dmax) dmax = val;
            if (idx <= 256 && 256 < idx + rep) l256 = true;
            if (lsum > 32768 || dsum > 32768) return false;
        }
        prev = val;
        idx += rep;
    }
    return l256 && lsum == 32768 && (dsum == 0 || dsum == 32768 || (dsum == 16384 && dmax == 1));
}

#define FSP_LIST 4096u

__global__ __launch_bounds__(FSP_FIND_T) void k_fsp_find(JdFspLaunch a)
{
    __shared__ uint8_t ptab[FSP_FIND_T][128];
    __shared__ uint32_t tile[(FSP_TILE + FSP_MARGIN) / 4 + 4];
    __shared__ uint32_t cand[FSP_TILE * 8 / 32];       /* stage A bitmap of the tile */
    __shared__ uint32_t list[FSP_LIST];                 /* stage A survivors, in order */
    __shared__ uint32_t cnt[FSP_FIND_T];
    __shared__ uint32_t first;
    const uint32_t c = blockIdx.x + 1, t = threadIdx.x;
    const uint64_t lo = a.bit0 + (uint64_t) c * a.span * 8;
    const uint64_t hi = min(lo + (uint64_t) a.span * 8, a.endbit);
    constexpr uint32_t PER = FSP_TILE * 8 / FSP_FIND_T;   /* positions per thread in stage A */
    uint64_t found = ~0ull;
    for (uint64_t tb = lo & ~31ull; tb < hi && found == ~0ull; tb += FSP_TILE * 8) {
        /* stage bytes [tb/8, tb/8 + TILE + MARGIN), zero past the input */
        const uint64_t A = tb >> 3;
        __syncthreads();
        for (uint32_t k = t; k < (FSP_TILE + FSP_MARGIN) / 4 + 4; k += FSP_FIND_T) {
            const uint64_t g = A + 4ull * k;
            uint32_t x = 0;
            if (g + 4 <= a.inlen) {
                JD_CHECK(a.in + g, 4, a.in + a.inlen);
                x = *(const uint32_t*) (a.in + g);
            } else {
                for (uint32_t j = 0; j < 4; j++) if (g + j < a.inlen) x |= (uint32_t) a.in[g + j] << (8 * j);
            }
            tile[k] = x;
        }
        __syncthreads();
        /* positions [p0, p1) of this tile, relative to tb */
        const uint32_t p0 = (uint32_t) (max(tb, lo) - tb);
        const uint32_t p1 = (uint32_t) (min(tb + FSP_TILE * 8, hi) - tb);
        /* stage A: thread t tests positions [t PER, (t+1) PER) */
        uint32_t n = 0;
        for (uint32_t w = 0; w < PER / 32; w++) {
            uint32_t m = 0;
            for (uint32_t j = 0; j < 32; j++) {
                const uint32_t q = t * PER + w * 32 + j;
                if (q >= p0 && q < p1 && fsp_quick(tile, q)) m |= 1u << j;
            }
            cand[t * (PER / 32) + w] = m;
            n += __builtin_popcount(m);
        }
        cnt[t] = n;
        __syncthreads();
        /* list the survivors in position order, up to FSP_LIST per pass */
        uint32_t from = 0;                 /* survivors already listed */
        uint32_t tot = 0, before = 0;
        for (uint32_t k = 0; k < FSP_FIND_T; k++) {
            const uint32_t x = cnt[k];
            if (k < t) before += x;
            tot += x;
        }
        while (from < tot && found == ~0ull) {
            __syncthreads();
            /* thread t writes its survivors with list index in [from, from + LIST) */
            uint32_t idx = before;
            for (uint32_t w = 0; w < PER / 32 && idx < from + FSP_LIST; w++) {
                uint32_t m = cand[t * (PER / 32) + w];
                while (m) {
                    const uint32_t j = __builtin_ctz(m);
                    m &= m - 1;
                    if (idx >= from && idx < from + FSP_LIST) list[idx - from] = t * PER + w * 32 + j;
                    idx++;
                }
            }
            __syncthreads();
            const uint32_t nl = min(tot - from, FSP_LIST);
            /* stage B: the full check, FSP_FIND_T survivors at a time */
            for (uint32_t k0 = 0; k0 < nl; k0 += FSP_FIND_T) {
                if (t == 0) first = FSP_LIST;
                __syncthreads();
                if (k0 + t < nl && fsp_header(tile, list[k0 + t], ptab[t])) atomicMin(&first, k0 + t);
                __syncthreads();
                const uint32_t f = first;
                __syncthreads();
                if (f < FSP_LIST) { found = tb + list[f]; break; }
            }
            from += nl;
        }
    }
    if (t == 0) a.starts[c] = found;
}

/* k_fsp_decode: chunk c on one wave, from its start until a block ends at or
 * past the next chunk's start, the BFINAL block ends, or it cannot go on.
 * The last 32768 entries live in an LDS ring whose slot p & 32767 holds
 * position p; before the chunk, slot j stands for position j - 32768 and
 * holds its marker 0x100 + j, so back-references need no special case.
 * Entries go to global memory from the ring in 4096-entry pieces. */
#define FSP_RING 32768u
#define FSP_FLUSH 4096u

__global__ __launch_bounds__(64) void k_fsp_decode(JdFspLaunch a)
{
    __shared__ InfShared s;
    __shared__ __attribute__((aligned(16))) uint16_t ring[FSP_RING];
    __shared__ __attribute__((aligned(16))) uint32_t lwin[RD_LW];
    __shared__ uint32_t lt32[LT_CAP], dt32[DT_CAP];
    const uint32_t c = blockIdx.x, lane = threadIdx.x;
    const uint32_t M = FSP_RING - 1;
    uint64_t* res = a.res + 4 * (uint64_t) c;
    const uint64_t b0 = c == 0 ? a.bit0 : a.starts[c];
    if (b0 == ~0ull) {
        if (lane == 0) { res[0] = JD_FSP_NONE; res[1] = 0; res[2] = 0; res[3] = 0; }
        return;
    }
    uint64_t stop = ~0ull;
    for (uint32_t k = c + 1; k < a.nchunk; k++)
        if (a.starts[k] != ~0ull) { stop = a.starts[k]; break; }
    uint16_t* o = a.o16 + (uint64_t) c * a.ocap;
    const uint32_t vw = c == 0 ? a.wlen : FSP_RING;
    Reader r;
    r.in = a.in;
    r.inlen = a.inlen;
    r.start = 0;
    r.clen = (uint32_t) min(a.inlen, (a.endbit + 7) >> 3);
    r.lw = lwin;
    r.lwn = RD_LW;
    r.wa = ~0ull;
    for (uint32_t i = lane; i < FSP_RING; i += 64) ring[i] = (uint16_t) (0x100u + i);
    __syncthreads();
    rd_init(r, (uint32_t) (b0 >> 3));
    uint32_t pos = 0, flushed = 0, v = 0, status = JD_FSP_STOPPED, lo = 0;
    uint64_t lb = b0;
    auto flush = [&]() {
        __builtin_amdgcn_wave_barrier();
        while (pos - flushed >= 2 * FSP_FLUSH) {
            for (uint32_t k = lane; k < FSP_FLUSH / 8; k += 64)
                *(uint4*) (o + flushed + 8 * k) = *(const uint4*) (ring + ((flushed + 8 * k) & M));
            flushed += FSP_FLUSH;
        }
    };
    if ((b0 & 7) && !rd_bits(r, (uint32_t) (b0 & 7), &v)) goto done;
    for (;;) {
        const uint64_t hb = rd_pos(r);
        lb = hb;
        lo = pos;
        if (hb >= stop) { status = hb == stop ? JD_FSP_REACHED : JD_FSP_PASSED; break; }
        if (!rd_bits(r, 3, &v)) break;
        const uint32_t fin = v & 1, type = v >> 1;
        if (type == 0) {
            const uint32_t byte = (uint32_t) ((rd_pos(r) + 7) >> 3);
            rd_init(r, byte);
            uint32_t ln, nln;
            if (!rd_bits(r, 16, &ln) || !rd_bits(r, 16, &nln) || (ln ^ 0xffff) != nln) break;
            const uint32_t at = byte + 4;
            if (at + ln > r.clen || pos + ln > a.ocap) break;
            for (uint32_t q = 0; q < ln; q += FSP_FLUSH) {
                const uint32_t n = min(FSP_FLUSH, ln - q);
                for (uint32_t i = lane; i < n; i += 64) {
                    JD_CHECK(r.in + at + q + i, 1, r.in + r.inlen);
                    ring[(pos + i) & M] = r.in[at + q + i];
                }
                pos += n;
                flush();
            }
            rd_init(r, at + ln);
        } else {
            if (type == 3) break;
            if ((type == 1 ? build_static(s) : read_dynamic(s, r)) != E_OK) break;
            fast_tables(s, lt32, dt32);
            bool ok = false;
            for (;;) {
                /* fast tokens: local scalar state, no input/output checks
                 * while >= 16 input bytes and >= 258 output entries remain */
                uint32_t fr = 0;                     /* 1 end of block, 2 error */
                if (r.ip + 16 <= r.clen && pos + 258 <= a.ocap) {
                    {
                        const uint64_t A = r.start + r.ip;
                        if (A < r.wa || A + 16 > r.wa + 4 * RD_LW) rd_window(r, A);
                    }
                    uint64_t bb = jd_uni64(r.bb);
                    uint32_t bc = jd_uni(r.bc), ip = jd_uni(r.ip), nw = jd_uni(r.nw);
                    uint32_t p = jd_uni(pos);
                    const uint32_t iplim = r.clen - 16, plim = a.ocap - 258;
                    const uint32_t wend = jd_uni((uint32_t) (r.wa + 4 * RD_LW - r.start)) - 16;
                    const uint32_t wb = jd_uni((uint32_t) (r.wa - r.start));
                    const uint32_t ilim = min(iplim, wend);
                    uint32_t n = 0;                      /* tokens that need no check */
                    for (;;) {
                        if (!n) {
                            if (p > plim || ip > ilim) break;   /* slow token (window moves) */
                            n = min((ilim - ip) >> 3, (plim - p) / 258u) + 1;
                        }
                        n--;
                        if (bc <= 32) {
                            bb |= (uint64_t) nw << bc;
                            bc += 32;
                            ip += 4;
                            const uint32_t o = ip - wb;
                            nw = jd_uni(__builtin_amdgcn_alignbyte(lwin[(o >> 2) + 1], lwin[o >> 2], o & 3));
                        }
                        uint32_t e = jd_uni(lt32[(uint32_t) bb & ((1u << LROOT) - 1)]);
                        if (e & F_SUB)
                            e = jd_uni(lt32[((e >> 4) & 0x7ff) + (((uint32_t) bb >> LROOT) & ((1u << (e & 15)) - 1))]);
                        const uint32_t L = e & 15;
                        if (!L) { fr = 2; break; }
                        bb >>= L;
                        bc -= L;
                        if (e & F_LIT) {
                            ring[p & M] = (uint16_t) ((e >> 16) & 0xff);   /* every lane, same word */
                            p++;
                            if (!(p & (FSP_FLUSH - 1))) { pos = p; flush(); }
                            continue;
                        }
                        if (e & F_EOB) { fr = 1; break; }
                        const uint32_t xl = (e >> 8) & 15;
                        const uint32_t len = (e >> 16) + ((uint32_t) bb & ((1u << xl) - 1));
                        bb >>= xl;
                        bc -= xl;
                        if (bc <= 32) {
                            bb |= (uint64_t) nw << bc;
                            bc += 32;
                            ip += 4;
                            const uint32_t o = ip - wb;
                            nw = jd_uni(__builtin_amdgcn_alignbyte(lwin[(o >> 2) + 1], lwin[o >> 2], o & 3));
                        }
                        uint32_t d = jd_uni(dt32[(uint32_t) bb & ((1u << DROOT) - 1)]);
                        if (d & F_SUB)
                            d = jd_uni(dt32[((d >> 4) & 0x7ff) + (((uint32_t) bb >> DROOT) & ((1u << (d & 15)) - 1))]);
                        const uint32_t Ld = d & 15;
                        if (!Ld) { fr = 2; break; }
                        bb >>= Ld;
                        bc -= Ld;
                        const uint32_t xd = (d >> 8) & 15;
                        const uint32_t off = (d >> 16) + ((uint32_t) bb & ((1u << xd) - 1));
                        bb >>= xd;
                        bc -= xd;
                        if (off > p + vw) { fr = 2; break; }          /* E_FAROFFSET */
                        if (!len) continue;
                        if (off >= len) {
                            for (uint32_t i0 = 0; i0 < len; i0 += 64) {
                                const uint32_t i = i0 + lane;
                                if (i < len) ring[(p + i) & M] = ring[(p - off + i) & M];
                            }
                        } else {
                            for (uint32_t i0 = 0; i0 < len; i0 += 64) {
                                const uint32_t i = i0 + lane;
                                if (i < len) ring[(p + i) & M] = off ? ring[(p - off + (i % off)) & M] : 0;
                            }
                        }
                        const uint32_t p0 = p;
                        p += len;
                        if ((p0 ^ p) & ~(FSP_FLUSH - 1)) { pos = p; flush(); }
                    }
                    r.bb = bb;
                    r.bc = bc;
                    r.ip = ip;
                    r.nw = nw;
                    pos = p;
                }
                if (fr == 1) { ok = true; break; }
                if (fr == 2) break;
                rd_uniform(r);
                pos = jd_uni(pos);
                const int sym = rd_sym(r, s.lt, LROOT);
                if (sym < 0) break;
                if (sym < 256) {
                    if (pos >= a.ocap) break;
                    if (lane == 0) ring[pos & M] = (uint16_t) sym;
                    pos++;
                    if (!(pos & (FSP_FLUSH - 1))) flush();
                    continue;
                }
                if (sym == 256) { ok = true; break; }
                const uint32_t ls = (uint32_t) sym - 257;
                uint32_t len = 0;
                if (ls < 29) {
                    if (!rd_bits(r, jd_lextra(ls), &v)) break;
                    len = jd_lbase(ls) + v;
                } /* 286/287 (static only): zero-length match, inflator.c:351 */
                const int dsy = rd_sym(r, s.dt, DROOT);
                if (dsy < 0) break;
                uint32_t off = 0;
                if (dsy < 30) {
                    if (!rd_bits(r, jd_dextra((uint32_t) dsy), &v)) break;
                    off = jd_dbase((uint32_t) dsy) + v;
                } /* 30/31 (static only): distance 0, inflator.c:372 */
                if (off > pos + vw) break;                       /* E_FAROFFSET */
                if (!len) continue;
                if (pos + len > a.ocap) break;
                /* overlap semantics as in k_inflate_resume; a source slot is
                 * never one this copy writes (len <= 258, off <= 32768) */
                if (off >= len) {
                    for (uint32_t i = lane; i < len; i += 64) ring[(pos + i) & M] = ring[(pos - off + i) & M];
                } else {
                    for (uint32_t i = lane; i < len; i += 64) {
                        const uint16_t x = off ? ring[(pos - off + (i % off)) & M] : 0;
                        ring[(pos + i) & M] = x;
                    }
                }
                const uint32_t p0 = pos;
                pos += len;
                if ((p0 ^ pos) & ~(FSP_FLUSH - 1)) flush();
            }
            if (!ok) break;
        }
        __builtin_amdgcn_wave_barrier();
        if (fin) {
            status = JD_FSP_ENDED;
            lb = rd_pos(r);
            lo = pos;
            break;
        }
    }
done:
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = flushed + lane; i < pos; i += 64) o[i] = ring[i & M];
    if (lane == 0) { res[0] = status; res[1] = lb; res[2] = lo; res[3] = pos; }
}

/* k_fsp_wtail: per piece, in parallel: a piece of >= 32768 entries whose
 * last 32768 hold no marker fixes the window after it by itself (stored
 * here); flag[1 + p] = 1 marks the pieces whose window needs the one before */
#define FSP_WT 1024u

__global__ __launch_bounds__(256) void k_fsp_wtail(JdFspResolve a)
{
    __shared__ uint32_t any;
    const uint32_t p = blockIdx.x, t = threadIdx.x;
    const uint64_t* pc = a.piece + 4 * (uint64_t) p;
    const uint32_t len = (uint32_t) pc[1];
    if (len < FSP_RING) {
        if (t == 0) a.flag[1 + p] = 1;
        return;
    }
    const uint16_t* o = a.o16 + pc[0] * a.ocap + (len - FSP_RING);
    if (t == 0) any = 0;
    __syncthreads();
    /* o is 2-byte aligned only (any piece length) */
    uint32_t m = 0;
    for (uint32_t j = 4 * t; j < FSP_RING; j += 4 * 256) m |= o[j] | o[j + 1] | o[j + 2] | o[j + 3];
    m &= 0xff00u;
    if (m) any = 1;
    __syncthreads();
    if (any) {
        if (t == 0) a.flag[1 + p] = 1;
        return;
    }
    uint8_t* G = a.win + (uint64_t) (p + 1) * FSP_RING;
    for (uint32_t j = 4 * t; j < FSP_RING; j += 4 * 256)
        *(uint32_t*) (G + j) = o[j] | ((uint32_t) o[j + 1] << 8) | ((uint32_t) o[j + 2] << 16) | ((uint32_t) o[j + 3] << 24);
    if (t == 0) a.flag[1 + p] = 0;
}

/* k_fsp_window: one workgroup walks the flagged pieces in order; the window
 * after piece p (its last 32768 bytes, markers resolved against the window
 * before it) is kept in LDS for the next step and stored for k_fsp_resolve;
 * unflagged pieces' windows came from k_fsp_wtail */
__global__ __launch_bounds__(FSP_WT) void k_fsp_window(JdFspResolve a)
{
    __shared__ __attribute__((aligned(16))) uint8_t w[2][FSP_RING];
    const uint32_t t = threadIdx.x;
    bool have = false;                   /* w[p & 1] holds the window before p */
    for (uint32_t p = 0; p < a.npiece; p++) {
        if (!a.flag[1 + p]) { have = false; continue; }
        uint8_t* W = w[p & 1];
        uint8_t* N = w[(p + 1) & 1];
        if (!have) {
            const uint8_t* src = a.win + (uint64_t) p * FSP_RING;
            for (uint32_t j = 4 * t; j < FSP_RING; j += 4 * FSP_WT) *(uint32_t*) (W + j) = *(const uint32_t*) (src + j);
            __syncthreads();
        }
        const uint64_t* pc = a.piece + 4 * (uint64_t) p;
        const uint16_t* o = a.o16 + pc[0] * a.ocap;
        const int64_t len = (int64_t) pc[1];
        uint8_t* G = a.win + (uint64_t) (p + 1) * FSP_RING;
        /* all 32 loads of a thread in flight at once */
        uint32_t e[FSP_RING / FSP_WT];
#pragma unroll
        for (uint32_t k = 0; k < FSP_RING / FSP_WT; k++) {
            const int64_t q = len - (int64_t) FSP_RING + t + k * FSP_WT;
            e[k] = q >= 0 ? o[q] : 0x100u + (uint32_t) (FSP_RING + q);
        }
#pragma unroll
        for (uint32_t k = 0; k < FSP_RING / FSP_WT; k++) {
            const uint32_t j = t + k * FSP_WT;
            const uint8_t x = e[k] < 0x100u ? (uint8_t) e[k] : W[e[k] - 0x100u];
            N[j] = x;
            G[j] = x;
        }
        __syncthreads();
        have = true;
    }
}

/* k_fsp_resolve: grid (piece, 16384-entry tile); bytes to the output */
#define FSP_RT 256u
#define FSP_RTILE 16384u

__global__ __launch_bounds__(FSP_RT) void k_fsp_resolve(JdFspResolve a)
{
    const uint32_t p = blockIdx.x, t = threadIdx.x;
    const uint64_t* pc = a.piece + 4 * (uint64_t) p;
    const uint32_t len = (uint32_t) pc[1];
    const uint32_t j0 = blockIdx.y * FSP_RTILE;
    if (j0 >= len) return;
    const uint16_t* o = a.o16 + pc[0] * a.ocap;
    uint8_t* out = a.out + pc[2];
    const uint8_t* W = a.win + (uint64_t) p * FSP_RING;
    const uint32_t wmin = FSP_RING - (uint32_t) pc[3];
    const uint32_t j1 = min(len, j0 + FSP_RTILE);
    bool far = false;
    for (uint32_t j = j0 + 4 * t; j < j1; j += 4 * FSP_RT) {
        uint16_t e[4];
        if (j + 4 <= j1) {
            const uint2 q = *(const uint2*) (o + j);
            e[0] = (uint16_t) q.x; e[1] = (uint16_t) (q.x >> 16);
            e[2] = (uint16_t) q.y; e[3] = (uint16_t) (q.y >> 16);
        } else {
            for (uint32_t k = 0; k < 4; k++) e[k] = j + k < j1 ? o[j + k] : 0;
        }
        for (uint32_t k = 0; k < 4 && j + k < j1; k++) {
            uint32_t x = e[k];
            if (x >= 0x100u) {
                x -= 0x100u;
                far |= x < wmin;
                x = W[x];
            }
            out[j + k] = (uint8_t) x;
        }
    }
    if (far) a.flag[0] = 1;
}

extern "C" int jdk_fsp_decode_launch(const JdFspLaunch* L)
{
    hipStream_t st = (hipStream_t) L->stream;
    JdFspLaunch a = *L;
    if (a.nchunk == 0 || (a.ocap & (FSP_FLUSH - 1))) return -1;
    if (a.nchunk > 1)
        JDPROF_RUN(JDK_FSP_FIND, st, (k_fsp_find<<<a.nchunk - 1, FSP_FIND_T, 0, st>>>(a)));
    JDPROF_RUN(JDK_FSP_DECODE, st, (k_fsp_decode<<<a.nchunk, 64, 0, st>>>(a)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int jdk_fsp_resolve_launch(const JdFspResolve* R)
{
    hipStream_t st = (hipStream_t) R->stream;
    JdFspResolve a = *R;
    if (a.npiece == 0) return 0;
    JDPROF_RUN(JDK_FSP_WINDOW, st, (k_fsp_wtail<<<a.npiece, 256, 0, st>>>(a)));
    JDPROF_RUN(JDK_FSP_WINDOW, st, (k_fsp_window<<<1, FSP_WT, 0, st>>>(a)));
    if (a.maxlen) {
        dim3 g(a.npiece, (a.maxlen + FSP_RTILE - 1) / FSP_RTILE);
        JDPROF_RUN(JDK_FSP_RESOLVE, st, (k_fsp_resolve<<<g, FSP_RT, 0, st>>>(a)));
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* ======================================================================== */
/* Block-mode inflate, two phases (bs <= 64 KiB, 16-byte aligned slots).
 *
 * The wave-per-block decoder above runs the serial Huffman decode on all 64
 * lanes at once, so 63/64 of every issued instruction is redundant and the
 * kernel is instruction-issue bound.  Here the 64 lanes share the work:
 *
 *   P1 k_inflate_par  one wave per block: headers wave-uniform, the body by
 *      64 self-synchronising segment walks (below).  Literals are stored
 *      straight to the output; every back-reference and stored run becomes
 *      a record (pos, len, off / src).  k_inflate_mp takes the blocks whose
 *      walks cannot sync (a flat literal code).
 *   P2 k_inflate_resolve  one wave per block, in place in the output slot:
 *      stored runs are copied first (they depend on nothing), then the
 *      back-references in groups of 64, each round copying every record
 *      whose source bytes no unresolved earlier record of the group writes.
 *
 * Decode semantics, error codes and their order are exactly k_inflate's
 * (and the reference's, inflator.c).  A block whose record list exceeds the
 * budget, or that is in any way unusual, is flagged and decoded by k_inflate.
 * ======================================================================== */
#ifndef P1_RING
#define P1_RING 8u                   /* dwords of input staged per lane     */
#endif
#ifndef P1_PRE
#define P1_PRE 4u                     /* dwords in flight per lane           */
#endif
#ifndef P1_K
#define P1_K 4u                     /* tokens between input batches        */
#endif

struct LReader {
    uint64_t bb;
    uint32_t bc, ip, clen, sk, fetched;
    uint64_t base;          /* absolute, 4-aligned start of the stream     */
};

__device__ static inline uint32_t p1_gload(const uint8_t* in, uint64_t inlen, uint64_t A)
{
    if (A + 4 <= inlen) {
        JD_CHECK(in + A, 4, in + inlen);
        return *(const uint32_t*) (in + A);
    }
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; k++)
        if (A + k < inlen) v |= (uint32_t) in[A + k] << (8 * k);
    return v;
}

/* (re)start the lane's reader at byte `byte` of its block: synchronous ring
 * fill of P1_RING - P1_PRE dwords, then P1_PRE dwords in flight */
template <uint32_t RS = 64>
__device__ static inline void p1_rinit(uint32_t* ring, LReader& r, const uint8_t* in, uint64_t inlen,
                                       uint32_t byte, uint32_t (&pre)[P1_PRE], uint32_t lane)
{
    r.bb = 0;
    r.bc = 0;
    r.ip = byte;
    const uint32_t t0 = (byte + r.sk) >> 2;
    uint32_t v[P1_RING - P1_PRE];
#pragma unroll
    for (uint32_t k = 0; k < P1_RING - P1_PRE; k++) v[k] = p1_gload(in, inlen, r.base + 4ull * (t0 + k));
#pragma unroll
    for (uint32_t k = 0; k < P1_RING - P1_PRE; k++) ring[((t0 + k) & (P1_RING - 1)) * RS + lane] = v[k];
    r.fetched = t0 + P1_RING - P1_PRE;
#pragma unroll
    for (uint32_t k = 0; k < P1_PRE; k++) pre[k] = p1_gload(in, inlen, r.base + 4ull * (r.fetched + k));
}

template <uint32_t RS = 64>
__device__ static inline void p1_fill(const uint32_t* ring, LReader& r, const uint8_t* in,
                                      uint64_t inlen, uint32_t lane)
{
    /* a whole token needs up to 48 bits; a refill leaves >= 56 */
    if (r.bc >= 48) return;
    const uint32_t a = r.ip + r.sk, t = a >> 2;
    uint32_t w0, w1, w2;
    if (t + 3 <= r.fetched) {
        w0 = ring[(t & (P1_RING - 1)) * RS + lane];
        w1 = ring[((t + 1) & (P1_RING - 1)) * RS + lane];
        w2 = ring[((t + 2) & (P1_RING - 1)) * RS + lane];
    } else {        /* the ring ran dry: read directly (rare) */
        w0 = p1_gload(in, inlen, r.base + 4ull * t);
        w1 = p1_gload(in, inlen, r.base + 4ull * (t + 1));
        w2 = p1_gload(in, inlen, r.base + 4ull * (t + 2));
    }
    const uint32_t sh = (a & 3) * 8;
    uint64_t x = ((uint64_t) w1 << 32 | w0) >> sh;
    if (sh) x |= (uint64_t) w2 << (64 - sh);
    const uint32_t left = r.ip < r.clen ? r.clen - r.ip : 0;
    if (left < 8) x &= left ? (~0ull >> (64 - 8 * left)) : 0ull;
    r.bb |= x << r.bc;
    const uint32_t nb = (63 - r.bc) >> 3;
    r.ip += nb;
    r.bc += nb * 8;
}

/* move the P1_PRE dwords in flight into the ring (after the caller's
 * vmcnt wait) and issue the next P1_PRE, when the ring has room */
template <uint32_t RS = 64>
__device__ static inline void p1_batch(uint32_t* ring, LReader& r, const uint8_t* in, uint64_t inlen,
                                       uint32_t (&pre)[P1_PRE], uint32_t lane)
{
    const uint32_t t = (r.ip + r.sk) >> 2;
    if (r.fetched - t <= P1_RING - P1_PRE) {
#pragma unroll
        for (uint32_t k = 0; k < P1_PRE; k++) ring[((r.fetched + k) & (P1_RING - 1)) * RS + lane] = pre[k];
        r.fetched += P1_PRE;
#pragma unroll
        for (uint32_t k = 0; k < P1_PRE; k++) pre[k] = p1_gload(in, inlen, r.base + 4ull * (r.fetched + k));
    }
}

__device__ static inline uint64_t p1_pos(const LReader& r) { return (uint64_t) r.ip * 8 - r.bc; }
__device__ static inline uint32_t p1_take(LReader& r, uint32_t nb)
{
    const uint32_t v = (uint32_t) r.bb & ((1u << nb) - 1);
    r.bb >>= nb;
    r.bc -= nb;
    return v;
}
/* root-only lookup: the entry for a code no longer than the root, or a
 * subtable link (E_SUB set) */
__device__ static inline uint32_t p1_root(const uint16_t* tab, uint32_t root, uint64_t bb)
{
    return tab[(uint32_t) bb & ((1u << root) - 1)];
}

/* table entry for the bits at the reader (no consumption); the subtable
 * read is issued for every lane (its index clamped to the root entry when
 * there is no subtable), which costs less than a divergent branch */
#ifndef P1_USKIP
#define P1_USKIP 1              /* measured: k_inflate_par 6.59-6.65 vs 6.72-6.77 ms */
#endif
__device__ static inline uint32_t p1_entry(const uint16_t* tab, uint32_t root, uint64_t bb)
{
    const uint32_t i0 = (uint32_t) bb & ((1u << root) - 1);
    const uint32_t e = tab[i0];
    const uint32_t i1 = ((e >> 4) & 0x7ff) + (((uint32_t) bb >> root) & ((1u << (e & 15)) - 1));
#if P1_USKIP
    /* the second read only when some lane of the wave needs a subtable (a
     * wave-uniform branch; most codes fit the root) */
    if (!__ballot((e & E_SUB) != 0)) return e;
#endif
    return tab[(e & E_SUB) ? i1 : i0];
}

/* record: match   bit63=0  pos[0,16) len[16,25) off[32,48)
 *         stored  bit63=1  pos[0,16) len[16,32) src-offset-in-block[32,63) */
#define REC_STORED (1ull << 63)
/* JdInflateLaunch.nrec: the record count, and this bit when one of them is a
 * stored run (k_inflate_resolve's stored pre-pass is skipped without it) */
#define NREC_STORED 0x80000000u

/* ======================================================================== */
/* P1 (default): one wave per block, the Huffman body decoded by all 64 lanes
 * at once using the self-synchronisation of prefix codes.
 *
 * The header of each deflate block is read by the whole wave (the
 * wave-uniform reader and table builder of k_inflate).  The body is cut
 * into nseg segments of W >= PAR_WIN bits:
 *   A1  lane k decodes from its segment start s_k (an arbitrary bit, not a
 *       token boundary), marking every token start it visits in the first
 *       PAR_WIN bits in a bitmap, with (ordinal, output, record) counts
 *       every PAR_CK boundaries and every end-of-block it meets;
 *   A2  it keeps decoding past s_{k+1} until one of its token starts is
 *       marked in a later lane's bitmap: from that sync point on the two
 *       decodes are the same, so lane k owns the span up to it;
 *   B   the spans are chained from the body start (lane 0 starts on a true
 *       boundary) until the span holding the true end-of-block; each span's
 *       output/record counts come from the checkpoints;
 *   C   an exclusive scan gives every span its output and record offsets;
 *   D   every span is decoded again from its true start, writing literals
 *       to the output and back-references / stored runs as records (P2
 *       k_inflate_resolve fills them in).
 * Anything unusual -- an invalid code or a read past the block on the true
 * path, no sync point, an offset or length out of range, too many records
 * -- flags the block, and k_inflate decodes it with exact reference error
 * semantics.  Decode semantics of clean blocks are those of k_inflate.
 * ======================================================================== */
#ifndef PAR_WIN
#define PAR_WIN 512u           /* bits of each segment's boundary bitmap   */
#endif
#ifndef PAR_CK
#define PAR_CK 16u             /* boundaries between count checkpoints     */
#endif
#ifndef PAR_NCK
#define PAR_NCK 4u               /* checkpoints kept per lane                */
#endif
#ifndef P1_A2MAX
#define P1_A2MAX 2048u         /* A2 bits past a segment before giving up  */
#endif
#ifndef PAR_NEOB
#define PAR_NEOB 4u            /* end-of-block events kept per lane        */
#endif

/* k_inflate_par's own bitmap window (the parallel resume keeps PAR_WIN).
 * 480 bits (measured when it set the occupancy: 14 waves per CU instead of
 * 13) moves the segment boundaries, and on mixed data at level 9 more lanes
 * then start their span on a distance-1 match whose byte they do not know:
 * k_inflate_resolve 4.9 -> 6.4 ms per 256 MiB (gpurun_out/r6n, r6o) */
#ifndef P1_WIN
#define P1_WIN 512u
#endif
/* 9.4 KiB per wave (was 14.8 KiB: 10 waves per CU, now 16).  The sync
 * bitmaps are live only from A1 to A2, the header scratch only while a
 * header is read, so the bitmaps overlay the scratch behind the decode
 * tables; the count checkpoints and end-of-block events live in registers
 * (the chain walk reads other lanes' events by shuffle). */
struct ParShared {
    union {
        InfShared t;                    /* decode tables, header scratch    */
        struct {
            uint16_t tabs[LT_CAP + DT_CAP];     /* t.lt, t.dt (live in the walks) */
            uint32_t bm[(P1_WIN / 32) * 64];    /* [word][lane], over the scratch */
        } w;
    };
    __attribute__((aligned(16))) uint32_t ring[P1_RING * 64];   /* per-lane compressed-input ring (and the header reader's window) */
};
static_assert(offsetof(InfShared, dt) == 2 * LT_CAP && offsetof(InfShared, cnt) == 2 * (LT_CAP + DT_CAP),
              "ParShared's bitmaps overlay InfShared's scratch, behind lt and dt");
#define PACKC(o, r) ((o) | ((r) << 17))

/* one token at the lane's reader: kind 0 literal (v), 1 match (len, off),
 * 2 end of block, 3 zero-length match (static 286/287); false on an invalid
 * code.  *nbits = bits the token takes. */
template <uint32_t RS = 64>
__device__ static inline bool par_tok(const uint32_t* ring, LReader& r, const uint8_t* in,
                                      uint64_t inlen, uint32_t lane, const uint16_t* lt,
                                      const uint16_t* dt, uint32_t* kind, uint32_t* v,
                                      uint32_t* len, uint32_t* off, uint32_t* nbits)
{
    p1_fill<RS>(ring, r, in, inlen, lane);
    const uint64_t bb = r.bb;
    const uint32_t e = p1_entry(lt, LROOT, bb);
    const uint32_t L = e & 15, sym = (e >> 4) & 0x1ff;
    if (!L) return false;
    if (sym <= 256) {
        *kind = sym < 256 ? 0 : 2;
        *v = sym;
        *nbits = L;
        p1_take(r, L);
        return true;
    }
    const uint32_t ls = sym - 257;
    const bool lsv = ls < 29;
    const uint32_t nbL = lsv ? jd_lextra(ls) : 0;
    const uint64_t bb1 = bb >> L;
    const uint32_t ln = lsv ? jd_lbase(ls) + ((uint32_t) bb1 & ((1u << nbL) - 1)) : 0;
    const uint64_t bb2 = bb1 >> nbL;
    const uint32_t e2 = p1_entry(dt, DROOT, bb2);
    const uint32_t L2 = e2 & 15, dsy = (e2 >> 4) & 0x1ff;
    if (!L2) return false;
    const bool dsv = dsy < 30;
    const uint32_t nbD = dsv ? jd_dextra(dsy) : 0;
    *off = dsv ? jd_dbase(dsy) + ((uint32_t) (bb2 >> L2) & ((1u << nbD) - 1)) : 0;
    *len = ln;
    *kind = ln ? 1 : 3;
    const uint32_t nb = L + nbL + L2 + nbD;
    *nbits = nb;
    p1_take(r, nb);
    return true;
}

/* after a literal: up to two more literals from the same refill (root-table
 * hits; a subtable link reads as a symbol >= 256); returns how many */
__device__ static inline uint32_t par_lits(const uint16_t* lt, LReader& r)
{
    uint32_t n = 0;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const uint32_t e = p1_root(lt, LROOT, r.bb);
        const uint32_t L = e & 15, sym = (e >> 4) & 0xfff;
        if (!(L != 0 && sym < 256)) break;
        p1_take(r, L);
        n++;
    }
    return n;
}

/* position the lane's reader at bit `bit` of its block */
template <uint32_t RS = 64>
__device__ static inline void par_seek(uint32_t* ring, LReader& r, const uint8_t* in, uint64_t inlen,
                                       uint32_t bit, uint32_t (&pre)[P1_PRE], uint32_t lane)
{
    p1_rinit<RS>(ring, r, in, inlen, bit >> 3, pre, lane);
    if (bit & 7) {
        p1_fill<RS>(ring, r, in, inlen, lane);
        p1_take(r, bit & 7);
    }
}

/* P1_FUSE: P1 resolves its own block's records right after writing them
 * (the bytes are still in L2) when the block has many records or long ones
 * (>= P1_FN records, or >= P1_FL output bytes per record: the long chains of
 * dependent copies of ramp, run and zero data), k_inflate_resolve the rest
 * (text's short independent copies run faster there, at its own occupancy) */
#ifndef P1_FUSE
#define P1_FUSE 1
#endif
#ifndef P1_FN
#define P1_FN 8192u
#endif
#ifndef P1_FL
#define P1_FL 48u
#endif
#ifndef P1_RSB
#define P1_RSB 4u               /* RS_B of the fused resolve */
#endif
template <uint32_t RB>
__device__ __attribute__((always_inline)) static void resolve_block(const JdInflateLaunch& a, uint32_t b,
                                                                    uint32_t nr, uint32_t usize, bool hasst);

#define PAR_BATCH(running)                                                     \
    if ((it & (P1_K - 1)) == 0) {                                              \
        if (!__ballot(running)) break;                                         \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                       \
        if (running) p1_batch(s.ring, r, a.in, a.inlen, pre, lane);            \
    }                                                                          \
    if (!(running)) continue;

__global__ __launch_bounds__(64) void k_inflate_par(JdInflateLaunch a)
{
    __shared__ ParShared s;
    uint32_t* const bm = s.w.bm;
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (b >= a.nblocks) return;
    const uint32_t cap = a.bs;
    uint8_t* out = a.out + (uint64_t) b * a.bs;
    uint64_t* recs = a.recs + (uint64_t) b * a.reccap;
    const uint64_t A0 = a.coff[b];
    const uint32_t clen = a.csize[b];
    const uint32_t cbits = clen * 8;

    Reader R;                      /* wave-uniform: headers */
    R.in = a.in;
    R.inlen = a.inlen;
    R.start = A0;
    R.clen = clen;
    /* the headers read through an LDS window held in the body walks' input
     * ring, idle while a header is read (one load round per 2 KiB of
     * headers instead of a dependent global load per dword); the walks
     * overwrite it, so it is marked empty after every body */
    R.lw = s.ring;
    R.lwn = P1_RING * 64;
    R.wa = ~0ull;
    rd_init(R, 0);
    LReader r;                     /* per lane: bodies, through s.ring */
    r.clen = clen;
    r.base = A0 & ~3ull;
    r.sk = (uint32_t) (A0 & 3);
    uint32_t pre[P1_PRE];

    uint32_t pos = 0, nrec = 0, sawfin = 0;
    bool fb = false, hasst = false;       /* hasst: a stored-run record */
    uint32_t v;

    for (;;) {
        /* the block's bytes end at a deflate-block boundary */
        if (rd_pos(R) + 7 >= (uint64_t) cbits) break;
        uint32_t hdr;
        if (!rd_bits(R, 3, &hdr)) { fb = true; break; }
        const uint32_t fin = hdr & 1, type = hdr >> 1;
        if (type == 0) {
            /* stored (decodestrd :931-1019): one record */
            const uint32_t byte = (uint32_t) ((rd_pos(R) + 7) >> 3);
            rd_init(R, byte);
            uint32_t ln, nln;
            if (!rd_bits(R, 16, &ln) || !rd_bits(R, 16, &nln) || (ln ^ 0xffff) != nln) { fb = true; break; }
            const uint32_t at = byte + 4;
            if (at + ln > clen || pos + ln > cap) { fb = true; break; }
            if (ln) {
                if (nrec >= a.reccap) { fb = true; break; }
                if (lane == 0)
                    recs[nrec] = REC_STORED | (uint64_t) pos | ((uint64_t) ln << 16) | ((uint64_t) at << 32);
                hasst = true;
                nrec++;
                pos += ln;
            }
            rd_init(R, at + ln);
            if (fin) { sawfin = 1; break; }
            continue;
        }
        if (type == 3) { fb = true; break; }
        if ((type == 1 ? build_static(s.t) : read_dynamic(s.t, R)) != E_OK) { fb = true; break; }
        const uint16_t* lt = s.t.lt;
        const uint16_t* dt = s.t.dt;
        /* flat literal code (every literal 7 bits or longer: incompressible
         * data, or fixed codes): walks may never fall into step, so A2 gives
         * up after P1_A2MAX bits and k_inflate_mp takes the block */
        bool flat;
        {
            uint32_t lmin = 15;
            for (uint32_t i = lane; i < (1u << LROOT); i += 64) {
                const uint32_t e = lt[i];
                if (!(e & E_SUB) && (e & 15) && ((e >> 4) & 0x1ff) < 256) lmin = min(lmin, e & 15);
            }
#pragma unroll
            for (uint32_t d = 32; d; d >>= 1) lmin = min(lmin, (uint32_t) __shfl_xor((int) lmin, (int) d));
            flat = lmin >= 7;
        }
        const uint32_t a2max = flat ? P1_A2MAX : 0xffffffffu;

        /* ---- body: segments ---- */
        const uint32_t B0 = (uint32_t) rd_pos(R);
        const uint32_t span = cbits > B0 ? cbits - B0 : 0;
        uint32_t nseg = span / P1_WIN;
        nseg = nseg < 1 ? 1 : nseg > 64 ? 64 : nseg;
        const uint32_t W = (span + nseg - 1) / nseg;   /* >= P1_WIN unless nseg == 1 */
        const bool act = lane < nseg;
        const uint32_t sk = B0 + lane * W;
        const uint32_t sk1 = B0 + (lane + 1) * W;

        /* A1: mark the token starts of the first P1_WIN bits */
        for (uint32_t w = 0; w < P1_WIN / 32; w++) bm[w * 64 + lane] = 0;
        uint32_t cout = 0, crec = 0, nbd = 0, nck = 0, neob = 0;
        uint32_t ckp[PAR_NCK], ckc[PAR_NCK];    /* bit offset of boundary i*PAR_CK; counts before it */
#pragma unroll
        for (uint32_t i = 0; i < PAR_NCK; i++) { ckp[i] = 0; ckc[i] = 0; }
        uint32_t eps[PAR_NEOB], eo[PAR_NEOB];   /* end-of-block start << 4 | code length; counts before it */
#pragma unroll
        for (uint32_t i = 0; i < PAR_NEOB; i++) { eps[i] = 0; eo[i] = 0; }
        bool dead = !act;
        if (act) par_seek(s.ring, r, a.in, a.inlen, sk, pre, lane);
        const uint32_t winend = min(sk + P1_WIN, min(cbits, sk1));
        for (uint32_t it = 0;; it++) {
            const bool running = !dead && (uint32_t) p1_pos(r) < winend;
            PAR_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            const uint32_t o = p - sk;
            atomicOr(&bm[(o >> 5) * 64 + lane], 1u << (o & 31));
            /* a checkpoint at the first boundary at or past every PAR_CK-th */
            if (nbd >= nck * PAR_CK && nck < PAR_NCK) {
#pragma unroll
                for (uint32_t i = 0; i < PAR_NCK; i++)
                    if (i == nck) { ckp[i] = o; ckc[i] = PACKC(cout, crec); }
                nck++;
            }
            nbd++;
            uint32_t kind, ln, off, nbits;
            if (!par_tok(s.ring, r, a.in, a.inlen, lane, lt, dt, &kind, &v, &ln, &off, &nbits)) {
                dead = true;
                continue;
            }
            if (kind == 2 && neob < PAR_NEOB) {
#pragma unroll
                for (uint32_t i = 0; i < PAR_NEOB; i++)
                    if (i == neob) { eps[i] = (p << 4) | nbits; eo[i] = PACKC(cout, crec); }
                neob++;
            }
            cout += kind == 0 ? 1 : kind == 1 ? ln : 0;
            crec += kind == 1;
            /* following literals from the same refill, each marked, inside
             * the window */
            if (kind == 0) {
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++) {
                    const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                    const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                    const uint32_t p3 = (uint32_t) p1_pos(r);
                    if (!(L3 != 0 && s3 < 256 && p3 < winend)) break;
                    const uint32_t o3 = p3 - sk;
                    atomicOr(&bm[(o3 >> 5) * 64 + lane], 1u << (o3 & 31));
                    p1_take(r, L3);
                    nbd++;
                    cout++;
                }
            }
        }
        __syncthreads();

        /* A2: continue to the first token start marked by a later lane */
        uint32_t nxt = 64, y = 0xffffffffu, yout = 0, yrec = 0;
        bool synced = false;
        for (uint32_t it = 0;; it++) {
            /* with a flat literal code, a walk that has not met a later
             * lane's token starts within P1_A2MAX bits past its segment keeps
             * a wrong bit phase: it stops, the chain fails, and
             * k_inflate_mp's multi-phase walks take the block */
            const bool running = !dead && !synced && (uint32_t) p1_pos(r) < cbits &&
                                 p1_pos(r) < (uint64_t) sk1 + a2max;
            PAR_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            if (p >= sk1) {
                uint32_t j = (p - B0) / W;
                j = j > nseg - 1 ? nseg - 1 : j;
                const uint32_t sj = B0 + j * W;
                if (j > lane && p - sj < P1_WIN) {
                    const uint32_t o = p - sj;
                    if ((bm[(o >> 5) * 64 + j] >> (o & 31)) & 1) {
                        nxt = j; y = p; yout = cout; yrec = crec;
                        synced = true;
                        continue;
                    }
                }
            }
            uint32_t kind, ln, off, nbits;
            if (!par_tok(s.ring, r, a.in, a.inlen, lane, lt, dt, &kind, &v, &ln, &off, &nbits)) {
                dead = true;
                continue;
            }
            if (kind == 2 && neob < PAR_NEOB) {
#pragma unroll
                for (uint32_t i = 0; i < PAR_NEOB; i++)
                    if (i == neob) { eps[i] = (p << 4) | nbits; eo[i] = PACKC(cout, crec); }
                neob++;
            }
            cout += kind == 0 ? 1 : kind == 1 ? ln : 0;
            crec += kind == 1;
            /* well before the next segment (whose token starts must each be
             * checked for sync), following literals decode from the same
             * refill: root-table hits only (>= 33 bits left after a literal) */
            if (kind == 0 && p + 64 < sk1) cout += par_lits(lt, r);
        }
        const uint32_t deadpos = dead ? (uint32_t) p1_pos(r) : 0xffffffffu;
        __syncthreads();

        /* B: chain the spans from the body start (wave-uniform walk) */
        uint32_t tstart = 0xffffffffu;             /* my span's true start   */
        uint32_t endlane = 64, eobk = 0;
        bool bad = false;
        {
            uint32_t cur = 0, t = B0;
            for (uint32_t guard = 0; guard < 65; guard++) {
                const uint32_t tc = t;
                if (lane == cur) tstart = tc;
                /* the first end-of-block on lane cur at or after t */
                uint32_t found = PAR_NEOB;
                const uint32_t yc = (uint32_t) __shfl((int) y, (int) cur);
                const uint32_t ne = (uint32_t) __shfl((int) neob, (int) cur);
#pragma unroll
                for (uint32_t i = 0; i < PAR_NEOB; i++) {
                    const uint32_t ep = (uint32_t) __shfl((int) eps[i], (int) cur) >> 4;
                    if (i < ne && found == PAR_NEOB && ep >= tc && ep < yc) found = i;
                }
                if (found < PAR_NEOB) { endlane = cur; eobk = found; break; }
                const uint32_t dp = (uint32_t) __shfl((int) deadpos, (int) cur);
                const uint32_t nx = (uint32_t) __shfl((int) nxt, (int) cur);
                /* invalid code on the true path, no sync, or end-of-block
                 * events beyond the ones kept: let the exact decoder do it */
                if (dp != 0xffffffffu || nx >= 64 || ne >= PAR_NEOB) { bad = true; break; }
                t = yc;
                cur = nx;
            }
            if (endlane >= 64) bad = true;
        }
        if (bad) { fb = true; break; }
        const bool inchain = tstart != 0xffffffffu;

        /* counts at my true start: the last checkpoint at or before it, then
         * decode forward to it (at most PAR_CK - 1 tokens) */
        uint32_t o0 = 0, r0 = 0;
        if (inchain) {
            uint32_t cp = ckp[0], cc = ckc[0];
#pragma unroll
            for (uint32_t i = 1; i < PAR_NCK; i++)
                if (i < nck && sk + ckp[i] <= tstart) { cp = ckp[i]; cc = ckc[i]; }
            o0 = cc & 0x1ffff;
            r0 = cc >> 17;
            par_seek(s.ring, r, a.in, a.inlen, sk + cp, pre, lane);
            while ((uint32_t) p1_pos(r) < tstart) {
                uint32_t kind, ln, off, nbits;
                if (!par_tok(s.ring, r, a.in, a.inlen, lane, lt, dt, &kind, &v, &ln, &off, &nbits)) {
                    o0 = 0xffffffffu;
                    break;
                }
                o0 += kind == 0 ? 1 : kind == 1 ? ln : 0;
                r0 += kind == 1;
                if (kind == 0) {
#pragma unroll
                    for (int k2 = 0; k2 < 2; k2++) {
                        const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                        const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                        if (!(L3 != 0 && s3 < 256 && (uint32_t) p1_pos(r) < tstart)) break;
                        p1_take(r, L3);
                        o0++;
                    }
                }
            }
        }
        if (__ballot(o0 == 0xffffffffu)) { fb = true; break; }   /* cannot happen: same path */
        /* my span ends at the sync point, or at the true end-of-block */
        uint32_t endpos = y, o1 = yout, r1 = yrec;
        uint32_t ekp = 0, eko = 0;                /* my end-of-block event eobk */
#pragma unroll
        for (uint32_t i = 0; i < PAR_NEOB; i++)
            if (i == eobk) { ekp = eps[i]; eko = eo[i]; }
        if (lane == endlane) {
            endpos = ekp >> 4;
            o1 = eko & 0x1ffff;
            r1 = eko >> 17;
        }
        const bool live = inchain && lane <= endlane;
        const uint32_t myo = live ? o1 - o0 : 0, myr = live ? r1 - r0 : 0;

        /* C: exclusive scan of the span counts (lane order = chain order) */
        uint32_t so = myo, sr = myr;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t xo = (uint32_t) __shfl_up((int) so, d), xr = (uint32_t) __shfl_up((int) sr, d);
            if (lane >= d) { so += xo; sr += xr; }
        }
        const uint32_t tot_o = (uint32_t) __shfl((int) so, 63), tot_r = (uint32_t) __shfl((int) sr, 63);
        so -= myo;
        sr -= myr;
        if (pos + tot_o > cap || nrec + tot_r > a.reccap) { fb = true; break; }

        /* D: decode my span again, writing.  A distance-1 match whose byte
         * before it this lane wrote itself (a literal, or a run filled here)
         * is a fill with a known byte: written now, its record left empty,
         * so the resolve has no chain of dependent rounds for it (all-zero
         * and run blocks are such chains) */
        bool err = false;
        if (live) par_seek(s.ring, r, a.in, a.inlen, tstart, pre, lane);
        uint32_t op = pos + so, rp = nrec + sr;
        int32_t lastv = -1;                       /* the byte before op, if known */
        for (uint32_t it = 0;; it++) {
            const bool running = live && !err && (uint32_t) p1_pos(r) < endpos;
            PAR_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            uint32_t kind, ln, off, nbits;
            if (!par_tok(s.ring, r, a.in, a.inlen, lane, lt, dt, &kind, &v, &ln, &off, &nbits) ||
                p + nbits > cbits) {
                err = true;
                continue;
            }
            if (kind == 0) {
                out[op] = (uint8_t) v;
                op++;
                lastv = (int32_t) (v & 0xff);
                /* up to two more literals from the same refill, not past the
                 * span end */
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++) {
                    const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                    const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                    if (!(L3 != 0 && s3 < 256 && (uint32_t) p1_pos(r) < endpos)) break;
                    p1_take(r, L3);
                    out[op] = (uint8_t) s3;
                    op++;
                    lastv = (int32_t) s3;
                }
            } else if (kind == 1) {
                if (off > op) { err = true; continue; }
                if (off == 1 && lastv >= 0) {
                    uint8_t* dp = out + op;
                    const uint32_t vv = (uint32_t) lastv * 0x01010101u;
                    uint32_t k = 0;
                    for (; k < ln && ((op + k) & 3); k++) dp[k] = (uint8_t) lastv;
                    for (; k + 4 <= ln; k += 4) *(uint32_t*) (dp + k) = vv;
                    for (; k < ln; k++) dp[k] = (uint8_t) lastv;
                    recs[rp++] = (uint64_t) op;            /* empty: nothing to resolve */
                } else {
                    recs[rp++] = (uint64_t) op | ((uint64_t) ln << 16) | ((uint64_t) off << 32);
                    lastv = -1;
                }
                op += ln;
            }
        }
        if (__ballot(err)) { fb = true; break; }
        pos += tot_o;
        nrec += tot_r;
        /* the header reader continues after the end-of-block symbol (its
         * window was the walks' ring) */
        const uint32_t ce = (uint32_t) __shfl((int) ekp, (int) endlane);
        const uint32_t after = (ce >> 4) + (ce & 15);
        R.wa = ~0ull;
        rd_init(R, after >> 3);
        if (after & 7) rd_bits(R, after & 7, &v);
        __syncthreads();
        if (fin) { sawfin = 1; break; }
    }
    const bool fuse = P1_FUSE && !fb && nrec && (nrec >= P1_FN || pos >= P1_FL * nrec);
    if (lane == 0) {
        a.fb[b] = fb ? 1 : 0;
        if (!fb) {
            a.usize[b] = pos;
            a.err[b] = E_OK;
            a.nrec[b] = fuse ? 0u : nrec | (hasst ? NREC_STORED : 0u);
            if (a.used) a.used[b] = (uint32_t) ((rd_pos(R) + 7) >> 3);
            if (a.fin) a.fin[b] = sawfin | ((rd_pos(R) & 7) ? 2u : 0u);
        }
    }
    if (fuse) {
        /* the literals and fills this wave stored are read back below */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        resolve_block<P1_RSB>(a, b, nrec, pos, hasst);
    }
}

/* P2: resolve one block's records in place in its output slot (HBM/L2).
 * One wave per block and no LDS, so many blocks' waves share a CU and hide
 * each other's latency.  Between rounds every store of the wave is waited
 * for, so a round's loads see the bytes written by the rounds before it. */
__device__ static inline uint32_t gl_word(const uint8_t* p, uint32_t n, const uint8_t* end)
{
    (void) end;
    /* the n (1..4) bytes at any address, from one or two dword loads
     * (JD_RSCOPE); the dword after the first is loaded only when one of the
     * n bytes is in it: a source ending at the last byte of the output
     * buffer must not read past it (that page may be unmapped) */
    const uintptr_t a = (uintptr_t) p;
    const uint32_t* w = (const uint32_t*) (a & ~(uintptr_t) 3);
    JD_CHECK(p, n, end);     /* the bytes needed lie in the block's output */
    const uint32_t x0 = __hip_atomic_load((JD_GLOBAL uint32_t*) w, __ATOMIC_RELAXED, JD_RSCOPE);
    const uint32_t x1 = (a & 3) + n > 4
        ? __hip_atomic_load((JD_GLOBAL uint32_t*) (w + 1), __ATOMIC_RELAXED, JD_RSCOPE) : 0u;
    return __builtin_amdgcn_alignbyte(x1, x0, (uint32_t) (a & 3));
}

/* gl_word in two halves, so that a batch of loads can be issued before
 * any of them is used: gl_raw loads the dword(s), gl_join aligns them */
__device__ static inline void gl_raw(const uint8_t* p, uint32_t n, const uint8_t* end,
                                     uint32_t& x0, uint32_t& x1)
{
    (void) end;
    const uintptr_t a = (uintptr_t) p;
    const uint32_t* w = (const uint32_t*) (a & ~(uintptr_t) 3);
    JD_CHECK(p, n, end);
    x0 = __hip_atomic_load((JD_GLOBAL uint32_t*) w, __ATOMIC_RELAXED, JD_RSCOPE);
    x1 = 0;
    if ((a & 3) + n > 4) x1 = __hip_atomic_load((JD_GLOBAL uint32_t*) (w + 1), __ATOMIC_RELAXED, JD_RSCOPE);
}

__device__ static inline uint32_t gl_join(const uint8_t* p, uint32_t x0, uint32_t x1)
{
    return __builtin_amdgcn_alignbyte(x1, x0, (uint32_t) ((uintptr_t) p & 3));
}

/* write n (<= 4) bytes of v at dst: a whole dword when aligned and full,
 * else byte stores (a dword may hold bytes of a neighbouring record) */
__device__ static inline void gl_put(uint8_t* dst, uint32_t v, uint32_t n)
{
    if (n == 4 && ((uintptr_t) dst & 3) == 0) {
        *(uint32_t*) dst = v;
    } else {
        for (uint32_t k = 0; k < n; k++) dst[k] = (uint8_t) (v >> (8 * k));
    }
}

#ifndef RS_B
#define RS_B 8u                 /* copy steps whose loads go out together  */
#endif
/* the records of block b (nr of them; usize output bytes) copied in place,
 * RB copy steps' loads issued together */
template <uint32_t RB>
__device__ __attribute__((always_inline)) static void resolve_block(const JdInflateLaunch& a, uint32_t b,
                                                                    uint32_t nr, uint32_t usize, bool hasst)
{
    const uint32_t lane = threadIdx.x;
    uint8_t* out = a.out + (uint64_t) b * a.bs;
    const uint64_t* recs = a.recs + (uint64_t) b * a.reccap;
    const uint8_t* oend = out + usize;
    (void) oend;

    /* stored runs: copied by the whole wave, they depend on nothing */
    const uint8_t* cin = a.in + a.coff[b];
    bool anystored = false;
    for (uint32_t g = 0; hasst && g < nr; g += 64) {
        const uint32_t i = g + lane;
        const uint64_t rc = i < nr ? recs[i] : 0;
        uint64_t st = __ballot(i < nr && (rc & REC_STORED));
        anystored |= st != 0;
        while (st) {
            const uint32_t j = __builtin_ctzll(st);
            st &= st - 1;
            const uint32_t lo = (uint32_t) __shfl((int) (uint32_t) rc, j);
            const uint32_t hi = (uint32_t) __shfl((int) (uint32_t) (rc >> 32), j);
            const uint32_t p = lo & 0xffff, ln = lo >> 16, at = hi & 0x7fffffff;
            for (uint32_t k = lane; k < ln; k += 64) out[p + k] = cin[at + k];
        }
    }
    if (anystored) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    /* back-references, 64 at a time; the next group's records load while
     * this group's rounds run */
    uint64_t rnext = lane < nr ? recs[lane] : 0;
    for (uint32_t g = 0; g < nr; g += 64) {
        const uint32_t i = g + lane;
        const bool have = i < nr;
        const uint64_t rc = rnext;
        rnext = g + 64 + lane < nr ? recs[g + 64 + lane] : 0;
        const bool stored = (rc & REC_STORED) != 0;
        const bool m = have && !stored;
        /* every record keeps its real destination range so the ends stay
         * sorted across the group; stored runs are already in place and
         * are never waited on (they are not in U below) */
        const uint32_t d = have ? (uint32_t) rc & 0xffff : 0xffffffffu;
        const uint32_t len = !have ? 0 : stored ? ((uint32_t) rc >> 16) & 0xffff
                                                : ((uint32_t) rc >> 16) & 0x1ff;
        const uint32_t off = m ? (uint32_t) (rc >> 32) & 0xffff : 0;
        const uint32_t e = have ? d + len : 0xffffffffu;
        /* sources [s0, s1) precede d; the records whose destinations
         * intersect them are the contiguous lane range [j0, j1) */
        const uint32_t s0 = d - off, s1 = min(d, s0 + len);
        uint32_t j0 = 0, j1 = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) {
            const uint32_t ej = (uint32_t) __shfl((int) e, (int) (j0 + step - 1));
            if (ej <= s0) j0 += step;
            const uint32_t dj = (uint32_t) __shfl((int) d, (int) (j1 + step - 1));
            if (dj < s1) j1 += step;
        }
        const uint32_t jend = min(j1, lane);
        const uint64_t dep = (m && off && j0 < jend)
            ? (((jend >= 64) ? ~0ull : ((1ull << jend) - 1)) & ~((1ull << j0) - 1)) : 0ull;
        uint64_t U = __ballot(m);
        while (U) {
            const bool ready = ((U >> lane) & 1) && !(U & dep);
            if (ready) {
                uint8_t* dst = out + d;
                if (!off) {
                    for (uint32_t k = 0; k < len; k++) dst[k] = 0;
                } else if (off >= len) {
                    /* no overlap: 4 bytes per step, RB steps' loads issued
                     * before their stores (one memory latency per 4*RB
                     * bytes instead of one per 4) */
                    const uint8_t* src = out + d - off;
                    for (uint32_t k0 = 0; k0 < len; k0 += 4 * RB) {
                        uint32_t x0[RB], x1[RB];
#pragma unroll
                        for (uint32_t j = 0; j < RB; j++) {
                            const uint32_t k = k0 + 4 * j;
                            x0[j] = x1[j] = 0;
                            if (k < len) gl_raw(src + k, min(4u, len - k), oend, x0[j], x1[j]);
                        }
#pragma unroll
                        for (uint32_t j = 0; j < RB; j++) {
                            const uint32_t k = k0 + 4 * j;
                            if (k < len) gl_put(dst + k, gl_join(src + k, x0[j], x1[j]), min(4u, len - k));
                        }
                    }
                } else if (off < 4) {
                    /* period 1..3: the pattern bytes are read once */
                    const uint32_t pb = gl_word(out + d - off, off, oend);
                    uint32_t ph = 0;
                    for (uint32_t k = 0; k < len; k += 4) {
                        uint32_t v = 0;
#pragma unroll
                        for (uint32_t j = 0; j < 4; j++) {
                            v |= ((pb >> (8 * ph)) & 0xff) << (8 * j);
                            ph = ph + 1 == off ? 0 : ph + 1;
                        }
                        gl_put(dst + k, v, min(4u, len - k));
                    }
                } else {
                    /* period `off` >= 4: byte k is source byte k mod off,
                     * copied in chunks that never wrap (RFC 1951 overlap
                     * semantics without reading bytes of this match) */
                    const uint8_t* src = out + d - off;
                    for (uint32_t k = 0, km = 0; k < len;) {
                        /* RB steps: their sources are the pattern bytes
                         * before d (final already), so the loads go first */
                        uint32_t x0[RB], x1[RB], nn[RB], kk[RB], mm[RB];
#pragma unroll
                        for (uint32_t j = 0; j < RB; j++) {
                            const uint32_t n = k < len ? min(min(4u, len - k), off - km) : 0u;
                            nn[j] = n;
                            kk[j] = k;
                            mm[j] = km;
                            x0[j] = x1[j] = 0;
                            if (n) gl_raw(src + km, n, oend, x0[j], x1[j]);
                            k += n;
                            km += n;
                            if (km == off) km = 0;
                        }
#pragma unroll
                        for (uint32_t j = 0; j < RB; j++)
                            if (nn[j]) gl_put(dst + kk[j], gl_join(src + mm[j], x0[j], x1[j]), nn[j]);
                    }
                }
            }
            /* this round's stores land before the next round reads */
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            U &= ~__ballot(ready);
        }
    }
}

/* minimum waves per SIMD the resolve is compiled for (1: its 76 VGPRs, 6
 * waves).  7 or 8 (RS_B 4-8) cut it on mixed data at level 9, 4.9 -> 3.9-4.8
 * ms per 256 MiB, where blocks are long chains of dependent records, but
 * slow it on text, 2.69 -> 2.77-2.81 ms per GiB, where more waves only
 * thrash the L2 (gpurun_out/r6w, r6x) */
#ifndef RS_WPE
#define RS_WPE 1
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RS_WPE))) void k_inflate_resolve(JdInflateLaunch a)
{
    const uint32_t b = blockIdx.x;
    if (a.fb[b]) return;
    const uint32_t nv = a.nrec[b], nr = nv & ~NREC_STORED;
    if (!nr) return;                      /* literals only: in place */
    resolve_block<RS_B>(a, b, nr, a.usize[b], (nv & NREC_STORED) != 0);
}

/* bytes of the parallel resume's LDS window || output buffer */
__device__ static inline uint32_t ob_word(const uint8_t* ob, uint32_t i)
{
    const uint32_t* w = (const uint32_t*) ob;
    return __builtin_amdgcn_alignbyte(w[(i >> 2) + 1], w[i >> 2], i);
}

__device__ static inline void ob_put(uint8_t* ob, uint32_t i, uint32_t v, uint32_t n)
{
    if (n == 4 && (i & 3) == 0) {
        *(uint32_t*) (ob + i) = v;
    } else {
        for (uint32_t k = 0; k < n; k++) ob[i + k] = (uint8_t) (v >> (8 * k));
    }
}


/* ======================================================================== */
/* P1b, for the blocks P1 flagged: a multi-phase parallel decode.  P1 relies
 * on lanes that start at arbitrary bits falling into step with the true
 * token boundaries; with near-uniform 8/9-bit literal codes (incompressible
 * data) a walk keeps its wrong bit phase, no lane syncs, and lane 0 would
 * decode the whole block.  Here every lane walks its segment from MP_P
 * consecutive start bits (its segment start + 0 .. MP_P-1), each walk to its
 * first token start at or past the next segment.  The true token start of
 * segment i lies exactly where the true walk of segment i-1 ended, so the
 * spans chain from the body start without any sync: the walk of lane i with
 * phase (t - s_i) is the true one, and a true start more than MP_P-1 bits
 * into a segment (a long match token across the boundary) is walked on the
 * spot by that lane alone.  Each walk is deterministic from its start, so
 * the chained spans decode exactly as the serial decoder does; then, as in
 * P1, the spans are decoded again writing literals and records for P2.
 * A block it cannot take (an invalid code on the true path, too many
 * records, ...) stays flagged for k_inflate's exact error semantics.
 * Semantics: inflator.c decodefast :1530-1823 on the body, decodednmc
 * :1104-1190 / buildtable :381-568 for the headers (shared with k_inflate).
 * ======================================================================== */
#define MP_P 8u

struct MpShared {
    InfShared t;
    uint32_t ring[P1_RING * 64];
    uint32_t we[(MP_P + 1) * 64];     /* [phase][lane] bit after the walk      */
    uint32_t wc[(MP_P + 1) * 64];     /*   output | records << 17 on the walk  */
    uint32_t wf[(MP_P + 1) * 64];     /*   1 = invalid code / past the block, 2 = ended at EOB */
};

__global__ __launch_bounds__(64) void k_inflate_mp(JdInflateLaunch a)
{
    __shared__ MpShared s;
    const uint32_t b = blockIdx.x, lane = threadIdx.x;
    if (b >= a.nblocks || !a.fb[b]) return;
    const uint32_t cap = a.bs;
    uint8_t* out = a.out + (uint64_t) b * a.bs;
    uint64_t* recs = a.recs + (uint64_t) b * a.reccap;
    const uint64_t A0 = a.coff[b];
    const uint32_t clen = a.csize[b];
    const uint32_t cbits = clen * 8;

    Reader R;
    R.in = a.in;
    R.inlen = a.inlen;
    R.start = A0;
    R.clen = clen;
    R.lw = nullptr;
    R.wa = 0;
    R.lwn = 0;
    rd_init(R, 0);
    LReader r;
    r.clen = clen;
    r.base = A0 & ~3ull;
    r.sk = (uint32_t) (A0 & 3);
    uint32_t pre[P1_PRE];
    uint32_t pos = 0, nrec = 0, sawfin = 0, v;
    bool fb = false, hasst = false;       /* hasst: a stored-run record */

    for (;;) {
        if (rd_pos(R) + 7 >= (uint64_t) cbits) break;
        uint32_t hdr;
        if (!rd_bits(R, 3, &hdr)) { fb = true; break; }
        const uint32_t fin = hdr & 1, type = hdr >> 1;
        if (type == 0) {
            const uint32_t byte = (uint32_t) ((rd_pos(R) + 7) >> 3);
            rd_init(R, byte);
            uint32_t ln, nln;
            if (!rd_bits(R, 16, &ln) || !rd_bits(R, 16, &nln) || (ln ^ 0xffff) != nln) { fb = true; break; }
            const uint32_t at = byte + 4;
            if (at + ln > clen || pos + ln > cap) { fb = true; break; }
            if (ln) {
                if (nrec >= a.reccap) { fb = true; break; }
                if (lane == 0)
                    recs[nrec] = REC_STORED | (uint64_t) pos | ((uint64_t) ln << 16) | ((uint64_t) at << 32);
                hasst = true;
                nrec++;
                pos += ln;
            }
            rd_init(R, at + ln);
            if (fin) { sawfin = 1; break; }
            continue;
        }
        if (type == 3) { fb = true; break; }
        if ((type == 1 ? build_static(s.t) : read_dynamic(s.t, R)) != E_OK) { fb = true; break; }
        const uint16_t* lt = s.t.lt;
        const uint16_t* dt = s.t.dt;

        const uint32_t B0 = (uint32_t) rd_pos(R);
        const uint32_t span = cbits > B0 ? cbits - B0 : 0;
        uint32_t nseg = span / 256;
        nseg = nseg < 1 ? 1 : nseg > 64 ? 64 : nseg;
        const uint32_t W = (span + nseg - 1) / nseg;
        const uint32_t sk = B0 + lane * W;
        /* a walk stops at its first token start at or past this (the last
         * segment's walks run to the end-of-block) */
        const uint32_t stopl = lane + 1 < nseg ? sk + W : 0xffffffffu;

        /* one walk per lane from `start` (if act): counts, end, flags */
        auto walk = [&](bool act, uint32_t start, uint32_t stop, uint32_t& e, uint32_t& oc,
                        uint32_t& fl) {
            bool dead = !act, eob = false;
            uint32_t o = 0, rc = 0;
            if (act) par_seek(s.ring, r, a.in, a.inlen, start, pre, lane);
            for (uint32_t it = 0;; it++) {
                const bool running = !dead && !eob && (uint32_t) p1_pos(r) < stop;
                PAR_BATCH(running)
                uint32_t kind, ln, off, nbits;
                const uint32_t p = (uint32_t) p1_pos(r);
                if (!par_tok(s.ring, r, a.in, a.inlen, lane, lt, dt, &kind, &v, &ln, &off, &nbits) ||
                    p + nbits > cbits) {
                    dead = true;
                    continue;
                }
                if (kind == 2) { eob = true; continue; }
                o += kind == 0 ? 1 : kind == 1 ? ln : 0;
                rc += kind == 1;
                /* following literals from the same refill, well inside the
                 * walk (two literals take at most 30 bits) */
                if (kind == 0 && p + 64 < min(stop, cbits)) o += par_lits(lt, r);
                if (o > 0x1ffffu || rc > 0x7fffu) dead = true;
            }
            e = act ? (uint32_t) p1_pos(r) : 0;
            oc = PACKC(o, rc);
            fl = (dead ? 1u : 0u) | (eob ? 2u : 0u);
        };

        /* A: MP_P phase walks per lane (lane 0 needs only phase 0) */
        for (uint32_t ph = 0; ph < MP_P; ph++) {
            const bool act = lane < nseg && (lane > 0 || ph == 0) && sk + ph < cbits;
            uint32_t e, oc, fl;
            walk(act, sk + ph, stopl, e, oc, fl);
            s.we[ph * 64 + lane] = e;
            s.wc[ph * 64 + lane] = oc;
            s.wf[ph * 64 + lane] = act ? fl : 1u;
        }
        __syncthreads();

        /* B: chain the true walks from the body start */
        uint32_t tstart = 0xffffffffu, slot = 0, endlane = 64;
        bool bad = false;
        {
            uint32_t t = B0;
            for (uint32_t i = 0; i < nseg; i++) {
                const uint32_t ski = B0 + i * W;
                const uint32_t ph = t - ski;
                uint32_t sl = ph;
                if (ph >= MP_P || (s.wf[ph * 64 + i] & 1)) {
                    /* a true start MP_P or more bits into the segment (or a
                     * walk that died there): lane i walks it now */
                    uint32_t e, oc, fl;
                    walk(lane == i, t, i + 1 < nseg ? ski + W : 0xffffffffu, e, oc, fl);
                    if (lane == i) {
                        s.we[MP_P * 64 + i] = e;
                        s.wc[MP_P * 64 + i] = oc;
                        s.wf[MP_P * 64 + i] = fl;
                    }
                    __syncthreads();
                    sl = MP_P;
                    if (s.wf[MP_P * 64 + i] & 1) { bad = true; break; }
                }
                if (lane == i) { tstart = t; slot = sl; }
                if (s.wf[sl * 64 + i] & 2) { endlane = i; break; }
                t = s.we[sl * 64 + i];
            }
            if (endlane >= 64) bad = true;
        }
        if (bad) { fb = true; break; }
        const bool live = lane <= endlane;
        const uint32_t mc = live ? s.wc[slot * 64 + lane] : 0;
        const uint32_t myo = mc & 0x1ffff, myr = mc >> 17;

        /* C: exclusive scan of the span counts */
        uint32_t so = myo, sr = myr;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t xo = (uint32_t) __shfl_up((int) so, d), xr = (uint32_t) __shfl_up((int) sr, d);
            if (lane >= d) { so += xo; sr += xr; }
        }
        const uint32_t tot_o = (uint32_t) __shfl((int) so, 63), tot_r = (uint32_t) __shfl((int) sr, 63);
        so -= myo;
        sr -= myr;
        if (pos + tot_o > cap || nrec + tot_r > a.reccap) { fb = true; break; }

        /* D: decode my span again, writing (to the next span's start, or
         * through the end-of-block on the last span) */
        const uint32_t endpos = live ? (lane < endlane ? s.we[slot * 64 + lane] : 0xffffffffu) : 0;
        bool err = false, eob = false;
        if (live) par_seek(s.ring, r, a.in, a.inlen, tstart, pre, lane);
        uint32_t op = pos + so, rp = nrec + sr;
        for (uint32_t it = 0;; it++) {
            const bool running = live && !err && !eob && (uint32_t) p1_pos(r) < endpos;
            PAR_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            uint32_t kind, ln, off, nbits;
            if (!par_tok(s.ring, r, a.in, a.inlen, lane, lt, dt, &kind, &v, &ln, &off, &nbits) ||
                p + nbits > cbits) {
                err = true;
                continue;
            }
            if (kind == 0) {
                out[op++] = (uint8_t) v;
                if (p + 64 < min(endpos, cbits)) {
#pragma unroll
                    for (int k2 = 0; k2 < 2; k2++) {
                        const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                        const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                        if (!(L3 != 0 && s3 < 256)) break;
                        p1_take(r, L3);
                        out[op++] = (uint8_t) s3;
                    }
                }
            } else if (kind == 1) {
                if (off > op) { err = true; continue; }
                recs[rp++] = (uint64_t) op | ((uint64_t) ln << 16) | ((uint64_t) off << 32);
                op += ln;
            } else if (kind == 2) {
                eob = true;
            }
        }
        if (__ballot(err)) { fb = true; break; }
        pos += tot_o;
        nrec += tot_r;
        /* the header reader continues after the end-of-block symbol */
        const uint32_t after = s.we[(uint32_t) __shfl((int) slot, (int) endlane) * 64 + endlane];
        rd_init(R, after >> 3);
        if (after & 7) rd_bits(R, after & 7, &v);
        __syncthreads();
        if (fin) { sawfin = 1; break; }
    }
    if (lane == 0 && !fb) {
        a.usize[b] = pos;
        a.err[b] = E_OK;
        a.nrec[b] = nrec | (hasst ? NREC_STORED : 0u);
        if (a.used) a.used[b] = (uint32_t) ((rd_pos(R) + 7) >> 3);
        if (a.fin) a.fin[b] = sawfin | ((rd_pos(R) & 7) ? 2u : 0u);
        a.fb[b] = 0;
    }
}


extern "C" int jdk_inflate_launch(const JdInflateLaunch* L)
{
    if (!L->nblocks) return 0;
    hipStream_t st = (hipStream_t) L->stream;
    const bool lanes = L->recs && L->nrec && L->fb && L->reccap && !L->require_final &&
                       L->bs <= 65536 && (L->bs & 15) == 0 && ((uintptr_t) L->out & 15) == 0;
    if (!lanes) {
        JdInflateLaunch a = *L;
        a.fb = nullptr;
        JDPROF_RUN(JDK_INFLATE, st, (k_inflate<<<L->nblocks, 64, 0, st>>>(a)));
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    /* chunks of L->chunk blocks share the record scratch */
    const uint32_t ch = L->chunk ? L->chunk : L->nblocks;
    for (uint32_t c0 = 0; c0 < L->nblocks; c0 += ch) {
        JdInflateLaunch a = *L;
        const uint32_t nb = min(ch, L->nblocks - c0);
        a.nblocks = nb;
        a.coff = L->coff + c0;
        a.csize = L->csize + c0;
        a.out = L->out + (uint64_t) c0 * L->bs;
        a.usize = L->usize + c0;
        a.err = L->err + c0;
        a.used = L->used ? L->used + c0 : nullptr;
        a.fin = L->fin ? L->fin + c0 : nullptr;
        JDPROF_RUN(JDK_INFLATE_P1, st, (k_inflate_par<<<nb, 64, 0, st>>>(a)));
        /* blocks P1 could not sync (incompressible data): multi-phase walks */
        JDPROF_RUN(JDK_INFLATE_MP, st, (k_inflate_mp<<<nb, 64, 0, st>>>(a)));
        JDPROF_RUN(JDK_INFLATE_P2, st, (k_inflate_resolve<<<nb, 64, 0, st>>>(a)));
        /* every block P1/P1b left flagged: the exact wave-per-block decoder */
        JDPROF_RUN(JDK_INFLATE, st, (k_inflate<<<nb, 64, 0, st>>>(a)));
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* ======================================================================== */
/* Parallel resume (JdRparLaunch): the drop-in inflator's decode of the span
 * it has in hand (inflator.c decodeblock :1330-1518 / decodefast :1530-1823
 * semantics), done by the 64 lanes of one wave with k_inflate_par's
 * self-synchronising walks instead of the one-wave serial decoder
 * (k_inflate_resume).  The differences from k_inflate_par:
 *   - the start is the resumable state (a block header, or inside a Huffman
 *     block whose tables the state holds), not a block's first byte;
 *   - the span's end is soft: the input may end inside a token, a header or
 *     a stored block.  Every lane remembers the end of its last token that
 *     ends at or before the input end; the chain stops on the lane whose walk
 *     reached the end without meeting a later lane, at that token end;
 *   - back-references may reach into the window (the <= 32 KiB before the
 *     output): window and output are one LDS buffer, resolved there;
 *   - the output room cuts the chain: the spans that fit are decoded whole,
 *     the first that does not is decoded token by token while the next token
 *     still fits (the serial decoder splits the last one, copybytes
 *     :1214-1290).
 * Anything it does not take (a flat literal code, an invalid code or a far
 * offset on the true path, too many end-of-block events in one walk) stops
 * it at the last clean point -- the block's header or its body's start --
 * with SERIAL, and the serial decoder continues with exact error semantics.
 * ======================================================================== */
#define RP_W  32768u
#define RP_OB (RP_W + JD_RP_OUT + 16u)

/* NW waves (T = 64 NW threads, one segment walk each): the header work is
 * done by every wave alike (the reader state is the same in all of them, so
 * their control flow agrees), the chain walk by every thread from LDS, the
 * scan and the reductions across waves through LDS, the resolve by wave 0 */
/* one record's copy in the LDS buffer, once its source is final */
__device__ static inline void rp_copy(uint8_t* ob, uint32_t d, uint32_t len, uint32_t off)
{
    if (!off) {
        for (uint32_t k = 0; k < len; k++) ob[d + k] = 0;
    } else if (off >= len) {
        for (uint32_t k = 0; k < len; k += 4) ob_put(ob, d + k, ob_word(ob, d - off + k), min(4u, len - k));
    } else if (off < 4) {
        const uint32_t pb = ob_word(ob, d - off);
        uint32_t ph = 0;
        for (uint32_t k = 0; k < len; k += 4) {
            uint32_t w = 0;
#pragma unroll
            for (uint32_t j = 0; j < 4; j++) {
                w |= ((pb >> (8 * ph)) & 0xff) << (8 * j);
                ph = ph + 1 == off ? 0 : ph + 1;
            }
            ob_put(ob, d + k, w, min(4u, len - k));
        }
    } else {
        for (uint32_t k = 0, km = 0; k < len;) {
            const uint32_t n = min(min(4u, len - k), off - km);
            ob_put(ob, d + k, ob_word(ob, d - off + km), n);
            k += n;
            km += n;
            if (km == off) km = 0;
        }
    }
}

template <uint32_t NW>
struct RpShared {
    static constexpr uint32_t T = 64 * NW;
    InfShared t;                          /* decode tables, header scratch   */
    uint32_t ring[P1_RING * T];           /* per-thread compressed-input ring */
    static constexpr uint32_t PW = PAR_WIN;   /* bits of a segment's start map */
    uint32_t bm[(PW / 32) * T];           /* [word][thread]                   */
    uint32_t ckp[PAR_NCK * T], ckc[PAR_NCK * T];
    uint32_t eps[PAR_NEOB * T], eo[PAR_NEOB * T];
    uint32_t lw[RD_LW];                   /* the header reader's input window */
    uint32_t y[T];                        /* each walk's sync point (the chain) */
    static constexpr uint32_t LV = NW == 1 ? 6 : NW == 2 ? 7 : NW <= 4 ? 8 : 9;   /* 2^(LV-1) >= T/2 */
    uint16_t jt[LV][T];                   /* jt[k][i]: 2^k-th successor of i (T: none) */
    uint32_t wo[NW], wr[NW];              /* per-wave totals of the scan      */
    uint32_t ctl[8];                      /* broadcast words                  */
};

template <uint32_t NW>
__global__ __launch_bounds__(64 * NW) void k_inflate_rpar(JdRparLaunch a)
{
    constexpr uint32_t T = 64 * NW;
    constexpr uint32_t OUTMAX = JD_RP_OUT;
    constexpr uint32_t PW = RpShared<NW>::PW;
    __shared__ RpShared<NW> s;
    __shared__ __attribute__((aligned(16))) uint8_t ob[RP_W + OUTMAX + 16u];
    uint32_t* const rin = s.ring;                 /* the walks' input */
    /* phase clocks (a -DRP_CLOCK build prints them per launch: tools/rpar_clock.py) */
#ifdef RP_CLOCK
    uint64_t rpc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, rpq = __builtin_amdgcn_s_memrealtime();
#define RPC_TICK(i_) do { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); rpc[i_] += t_ - rpq; rpq = t_; } while (0)
#else
#define RPC_TICK(i_) ((void) 0)
#endif
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    JdInfState* S = a.st;
    const uint32_t cbits = a.inlen * 8;
    uint32_t mode = S->mode, fin = S->fin;
    const uint32_t plen0 = S->plen, poff0 = S->poff;
    if (!(mode == JD_RS_HEADER || mode == JD_RS_HUFF) || (plen0 && mode != JD_RS_HUFF)) {
        /* a stored remainder: the serial decoder's */
        if (tid == 0) {
            S->status = JD_RST_SERIAL;
            S->bit = a.bitpos;
            S->produced = 0;
            head_to_host(S, a.hhead);
        }
        return;
    }
    /* window || output in LDS: the whole 32 KiB in front of out (the bytes
     * before the valid window are never referenced: such an offset is an
     * error, left to the serial decoder) */
    for (uint32_t o = tid * 16; o < RP_W; o += T * 16) *(uint4*) (ob + o) = *(const uint4*) (a.win + o);
    if (mode == JD_RS_HUFF) {
        for (uint32_t i = tid; i < LT_CAP; i += T) s.t.lt[i] = S->lt[i];
        for (uint32_t i = tid; i < DT_CAP; i += T) s.t.dt[i] = S->dt[i];
    }
    __syncthreads();
    const uint32_t wlo = RP_W - a.pos0;
    const uint32_t lim = RP_W + min(a.cap, OUTMAX);
    uint32_t pos = RP_W, nrec = 0, v = 0;
    uint32_t status = JD_RST_SERIAL;
    bool newtab = false;

    /* the last clean point: where the state is left */
    uint32_t cmode = mode, cfin = fin, cbit = a.bitpos, cpos = pos, cnrec = 0, csrem = 0;
    uint32_t cplen = 0, cpoff = 0;       /* a match split at a full target     */
    uint32_t fclean = 0;                 /* FULL where the serial decoder stops too */
    bool ctab = false;
    bool run = true;
    if (plen0) {
        /* the pending copy first (copybytes :1214-1290): every byte comes
         * from the window, period poff */
        const uint32_t n = min(plen0, lim - pos);
        for (uint32_t i = tid; i < n; i += T) ob[pos + i] = ob[pos - poff0 + (i % poff0)];
        __syncthreads();
        pos += n;
        cpos = pos;
        if (n < plen0) {
            cplen = plen0 - n;
            cpoff = poff0;
            status = JD_RST_FULL;
            fclean = 1;
            run = false;
        }
    }
    /* NEEDINPUT with nothing the serial decoder could add (a header, stored
     * block or valid token cut by the input's end), reported in `pad` */
    uint32_t clean = 0;

    Reader R;                      /* the same in every wave: headers */
    R.in = a.in;
    R.inlen = a.inlen;
    R.start = 0;
    R.clen = a.inlen;
    R.lw = s.lw;                   /* one load per 4 KiB of headers, not per dword */
    R.lwn = RD_LW;
    R.wa = ~0ull;
    rd_init(R, a.bitpos >> 3);
    if (a.bitpos & 7) rd_bits(R, a.bitpos & 7, &v);
    LReader r;                     /* per thread: bodies */
    r.clen = a.inlen;
    r.base = 0;
    r.sk = 0;
    uint32_t pre[P1_PRE];
#define RP_BATCH(running)                                                      \
    if ((it & (P1_K - 1)) == 0) {                                              \
        if (!__ballot(running)) break;                                         \
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                       \
        if (running) p1_batch<T>(s.ring, r, a.in, a.inlen, pre, tid);          \
    }                                                                          \
    if (!(running)) continue;

    bool marker = false;                 /* the last block was an empty stored one */
    if (run)
    for (;;) {
        if (mode == JD_RS_HEADER) {
            const uint32_t hb = (uint32_t) rd_pos(R);
            cmode = JD_RS_HEADER; cbit = hb; cpos = pos; cnrec = nrec; ctab = false;
            if (hb > a.bitpos) {
                /* the parallel rounds of the host take it from here */
                const uint64_t rest = (uint64_t) (a.inlen - (hb >> 3)) + a.extra;
                if ((a.hdrmin && rest >= a.hdrmin) || (marker && a.markmin && rest >= a.markmin)) {
                    status = JD_RST_MARKER;
                    break;
                }
            }
            marker = false;
            uint32_t hdr;
            if (!rd_bits(R, 3, &hdr)) { status = JD_RST_NEEDINPUT; clean = 1; break; }
            fin = hdr & 1;
            const uint32_t type = hdr >> 1;
            if (type == 0) {
                /* stored (decodestrd :931-1019): copied now, as far as the
                 * input and the room go */
                const uint32_t byte = (uint32_t) ((rd_pos(R) + 7) >> 3);
                rd_init(R, byte);
                uint32_t ln, nln;
                if (!rd_bits(R, 16, &ln) || !rd_bits(R, 16, &nln)) { status = JD_RST_NEEDINPUT; clean = 1; break; }
                if ((ln ^ 0xffff) != nln) break;                       /* SERIAL: the error */
                const uint32_t at = byte + 4;
                const uint32_t have = at < a.inlen ? a.inlen - at : 0;
                const uint32_t n = min(ln, min(have, lim - pos));
                for (uint32_t i = tid; i < n; i += T) {
                    JD_CHECK(a.in + at + i, 1, a.in + a.inlen);
                    ob[pos + i] = a.in[at + i];
                }
                pos += n;
                if (n < ln) {
                    cmode = JD_RS_STORED; cfin = fin; cbit = (at + n) * 8; cpos = pos; cnrec = nrec;
                    csrem = ln - n;
                    status = pos == lim ? JD_RST_FULL : JD_RST_NEEDINPUT;
                    clean = 1;
                    break;
                }
                rd_init(R, at + ln);
                if (fin) {
                    cmode = JD_RS_ENDED; cfin = 1; cbit = (uint32_t) rd_pos(R); cpos = pos; cnrec = nrec;
                    status = JD_RST_ENDED;
                    break;
                }
                marker = ln == 0;
                continue;
            }
            if (type == 3) break;                                         /* SERIAL */
            const uint32_t e2 = type == 1 ? build_static(s.t) : read_dynamic(s.t, R);
            if (e2 == E_INPUTEND) { status = JD_RST_NEEDINPUT; clean = 1; break; }
            if (e2) break;                                                /* SERIAL */
            mode = JD_RS_HUFF;
            newtab = true;
        }
        RPC_TICK(0);
        __syncthreads();

        /* ---- a Huffman body from B0: the clean point is its start ---- */
        const uint32_t B0 = (uint32_t) rd_pos(R);
        cmode = JD_RS_HUFF; cfin = fin; cbit = B0; cpos = pos; cnrec = nrec; ctab = newtab;
        const uint16_t* lt = s.t.lt;
        const uint16_t* dt = s.t.dt;
        {
            /* a flat literal code: walks may never fall into step (every
             * wave reduces the whole root table, so all of them agree) */
            uint32_t lmin = 15;
            for (uint32_t i = lane; i < (1u << LROOT); i += 64) {
                const uint32_t e = lt[i];
                if (!(e & E_SUB) && (e & 15) && ((e >> 4) & 0x1ff) < 256) lmin = min(lmin, e & 15);
            }
#pragma unroll
            for (uint32_t d = 32; d; d >>= 1) lmin = min(lmin, (uint32_t) __shfl_xor((int) lmin, (int) d));
            if (lmin >= 7) break;                                         /* SERIAL */
        }
        if (B0 >= cbits) { status = JD_RST_NEEDINPUT; clean = 1; break; }
        const uint32_t span = cbits - B0;
        uint32_t nseg = span / PW;
        nseg = nseg < 1 ? 1 : nseg > T ? T : nseg;
        const uint32_t W = (span + nseg - 1) / nseg;
        const bool act = tid < nseg;
        const uint32_t sk = B0 + tid * W;
        const uint32_t sk1 = B0 + (tid + 1) * W;

        /* a token at p is taken only if it ends at or before the input end;
         * near the end a failed or overlong decode is the end of the walk
         * (more input may complete it), not an error */
        uint32_t lend = 0xffffffffu, lo = 0, lr = 0;       /* last complete token end, counts */
        bool atend = false, aeclean = true;   /* clean: a valid token cut by the end */
        auto tok = [&](uint32_t p, uint32_t& kind, uint32_t& ln, uint32_t& off, uint32_t& nbits,
                       bool& dead, uint32_t cout, uint32_t crec) -> bool {
            const bool ok = par_tok<T>(rin, r, a.in, a.inlen, tid, lt, dt, &kind, &v, &ln, &off, &nbits);
            if (p + 48 > cbits && (!ok || p + nbits > cbits)) { atend = true; aeclean = ok; return false; }
            if (!ok) { dead = true; return false; }
            const uint32_t no = cout + (kind == 0 ? 1 : kind == 1 ? ln : 0);
            lend = p + nbits; lo = no; lr = crec + (kind == 1);
            return true;
        };

        /* A1: mark the token starts of the first PW bits */
        for (uint32_t w = 0; w < PW / 32; w++) s.bm[w * T + tid] = 0;
        uint32_t cout = 0, crec = 0, nbd = 0, nck = 0, neob = 0;
        bool dead = !act;
        if (act) par_seek<T>(rin, r, a.in, a.inlen, sk, pre, tid);
        if (act) { lend = sk; lo = 0; lr = 0; }
        const uint32_t winend = min(sk + PW, min(cbits, sk1));
        for (uint32_t it = 0;; it++) {
            const bool running = !dead && !atend && (uint32_t) p1_pos(r) < winend;
            RP_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            const uint32_t o = p - sk;
            atomicOr(&s.bm[(o >> 5) * T + tid], 1u << (o & 31));
            if (nbd >= nck * PAR_CK && nck < PAR_NCK) {
                const uint32_t c = nck * T + tid;
                s.ckp[c] = o;
                s.ckc[c] = PACKC(cout, crec);
                nck++;
            }
            nbd++;
            uint32_t kind, ln, off, nbits;
            if (!tok(p, kind, ln, off, nbits, dead, cout, crec)) continue;
            if (kind == 2 && neob < PAR_NEOB) {
                const uint32_t c = neob * T + tid;
                s.eps[c] = (p << 4) | nbits;
                s.eo[c] = PACKC(cout, crec);
                neob++;
            }
            cout += kind == 0 ? 1 : kind == 1 ? ln : 0;
            crec += kind == 1;
            if (kind == 0) {
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++) {
                    const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                    const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                    const uint32_t p3 = (uint32_t) p1_pos(r);
                    if (!(L3 != 0 && s3 < 256 && p3 < winend && p3 + L3 <= cbits)) break;
                    const uint32_t o3 = p3 - sk;
                    atomicOr(&s.bm[(o3 >> 5) * T + tid], 1u << (o3 & 31));
                    p1_take(r, L3);
                    nbd++;
                    cout++;
                    lend = p3 + L3; lo = cout; lr = crec;
                }
            }
        }
        __syncthreads();
        RPC_TICK(1);

        /* A2: continue to the first token start marked by a later thread */
        uint32_t nxt = T, y = 0xffffffffu, yout = 0, yrec = 0;
        bool synced = false;
        for (uint32_t it = 0;; it++) {
            const bool running = !dead && !synced && !atend && (uint32_t) p1_pos(r) < cbits;
            RP_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            if (p >= sk1) {
                uint32_t j = (p - B0) / W;
                j = j > nseg - 1 ? nseg - 1 : j;
                const uint32_t sj = B0 + j * W;
                if (j > tid && p - sj < PW) {
                    const uint32_t o = p - sj;
                    if ((s.bm[(o >> 5) * T + j] >> (o & 31)) & 1) {
                        nxt = j; y = p; yout = cout; yrec = crec;
                        synced = true;
                        continue;
                    }
                }
            }
            uint32_t kind, ln, off, nbits;
            if (!tok(p, kind, ln, off, nbits, dead, cout, crec)) continue;
            if (kind == 2 && neob < PAR_NEOB) {
                const uint32_t c = neob * T + tid;
                s.eps[c] = (p << 4) | nbits;
                s.eo[c] = PACKC(cout, crec);
                neob++;
            }
            cout += kind == 0 ? 1 : kind == 1 ? ln : 0;
            crec += kind == 1;
            if (kind == 0 && p + 64 < sk1 && p + 64 < cbits) {
                cout += par_lits(lt, r);
                lend = (uint32_t) p1_pos(r); lo = cout; lr = crec;
            }
        }
        /* a walk that reached the input end without a sync ends the chain */
        if ((uint32_t) p1_pos(r) >= cbits && !dead && !synced) atend = true;
        s.y[tid] = y;
        __syncthreads();
        RPC_TICK(2);

        /* B: chain the spans from the body start.  The chain is the path
         * 0 -> nx[0] -> ... (successors only increase): jump tables by
         * pointer doubling give every thread the last path node before it
         * (binary lifting), hence whether it is on the path and its true
         * start (that node's sync point); the first path node that stops
         * the chain (an end of block in its span, an invalid code or too
         * many end-of-block events on it, or no later thread met) is found
         * by a minimum over the threads. */
        s.jt[0][tid] = (uint16_t) nxt;
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k + 1 < RpShared<NW>::LV; k++) {
            const uint32_t j1 = s.jt[k][tid];
            const uint32_t j2 = j1 < T ? s.jt[k][j1] : T;
            s.jt[k + 1][tid] = (uint16_t) j2;
            __syncthreads();
        }
        uint32_t pn = 0;                           /* last path node before me */
        if (tid > 0) {
#pragma unroll
            for (int k = RpShared<NW>::LV - 1; k >= 0; k--) {
                const uint32_t jn = s.jt[k][pn];
                if (jn < tid) pn = jn;
            }
        }
        const bool member = tid == 0 || s.jt[0][pn] == tid;
        const uint32_t tme = tid == 0 ? B0 : s.y[pn];
        uint32_t found = PAR_NEOB;
        for (uint32_t i = 0; i < neob && found == PAR_NEOB; i++) {
            const uint32_t ep = s.eps[i * T + tid] >> 4;
            if (ep >= tme && ep < y) found = i;
        }
        const uint32_t code = found < PAR_NEOB ? 1u : (dead || neob >= PAR_NEOB) ? 2u
                            : nxt >= T ? (atend ? 3u : 2u) : 0u;
        if (tid == 0) s.ctl[6] = 0xffffffffu;
        __syncthreads();
        if (member && code) {
            atomicMin(&s.ctl[6], (tid << 2) | code);
        }
        __syncthreads();
        const uint32_t stop = s.ctl[6];
        const uint32_t endlane = stop == 0xffffffffu ? T : stop >> 2;
        const bool bad = stop == 0xffffffffu || (stop & 3) == 2;
        const bool trunc = (stop & 3) == 3;
        if (tid == endlane) s.ctl[7] = found | ((aeclean ? 1u : 0u) << 8);
        __syncthreads();
        if (bad) break;                                                   /* SERIAL */
        const uint32_t eobk = s.ctl[7] & 0xff;
        const uint32_t tclean = (s.ctl[7] >> 8) & 1;
        const uint32_t tstart = member ? tme : 0xffffffffu;
        const bool inchain = tstart != 0xffffffffu;

        /* counts at my true start (the last checkpoint before it, then
         * forward at most PAR_CK - 1 tokens) */
        uint32_t o0 = 0, r0 = 0;
        if (inchain) {
            uint32_t ci = 0;
            for (uint32_t i = 1; i < PAR_NCK; i++) {
                const uint32_t c = i * T + tid;
                if (i < nck && sk + s.ckp[c] <= tstart) ci = i;
            }
            const uint32_t c0 = ci * T + tid;
            o0 = s.ckc[c0] & 0x1ffff;
            r0 = s.ckc[c0] >> 17;
            par_seek<T>(rin, r, a.in, a.inlen, sk + s.ckp[c0], pre, tid);
            while ((uint32_t) p1_pos(r) < tstart) {
                uint32_t kind, ln, off, nbits;
                if (!par_tok<T>(rin, r, a.in, a.inlen, tid, lt, dt, &kind, &v, &ln, &off, &nbits)) {
                    o0 = 0xffffffffu;
                    break;
                }
                o0 += kind == 0 ? 1 : kind == 1 ? ln : 0;
                r0 += kind == 1;
                if (kind == 0) {
#pragma unroll
                    for (int k2 = 0; k2 < 2; k2++) {
                        const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                        const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                        if (!(L3 != 0 && s3 < 256 && (uint32_t) p1_pos(r) < tstart)) break;
                        p1_take(r, L3);
                        o0++;
                    }
                }
            }
        }
        if (tid == 0) s.ctl[0] = 0;
        __syncthreads();
        if (o0 == 0xffffffffu) s.ctl[0] = 1;
        __syncthreads();
        if (s.ctl[0]) break;                                              /* SERIAL */
        uint32_t endpos = y, o1 = yout, r1 = yrec;
        if (tid == endlane) {
            if (trunc) {
                endpos = lend; o1 = lo; r1 = lr;
            } else {
                const uint32_t c = eobk * T + tid;
                endpos = s.eps[c] >> 4;
                o1 = s.eo[c] & 0x1ffff;
                r1 = s.eo[c] >> 17;
            }
        }
        const bool live = inchain && tid <= endlane;
        const uint32_t myo = live ? o1 - o0 : 0, myr = live ? r1 - r0 : 0;

        RPC_TICK(3);
        /* C: exclusive scan of the span counts (thread order = chain order):
         * within the wave, then the totals of the waves before */
        uint32_t so = myo, sr = myr;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t xo = (uint32_t) __shfl_up((int) so, d), xr = (uint32_t) __shfl_up((int) sr, d);
            if (lane >= d) { so += xo; sr += xr; }
        }
        if (lane == 63) { s.wo[wv] = so; s.wr[wv] = sr; }
        __syncthreads();
        for (uint32_t w = 0; w < wv; w++) { so += s.wo[w]; sr += s.wr[w]; }
        so -= myo;
        sr -= myr;
        /* the room cuts the chain: spans that fit whole, then the first one
         * that does not, token by token */
        const uint32_t room = lim - pos, rroom = JD_RP_MAXREC - nrec;
        const bool fits = live && so + myo <= room && sr + myr <= rroom;
        if (tid == 0) s.ctl[1] = T;
        __syncthreads();
        if (live && !fits) atomicMin(&s.ctl[1], tid);
        __syncthreads();
        const uint32_t cutlane = s.ctl[1];
        const bool part = tid == cutlane;
        const bool wr = (live && fits) || part;

        /* D: decode my span again, writing literals into the buffer and
         * back-references as records */
        bool err = false;
        if (wr) par_seek<T>(rin, r, a.in, a.inlen, tstart, pre, tid);
        uint32_t op = pos + so, rp = nrec + sr;
        int32_t lastv = -1;
        uint32_t pstop = endpos;                  /* the part thread: where it stopped */
        uint32_t ppl = 0, ppo = 0, pfl = 0;       /* its split match, clean stop     */
        for (uint32_t it = 0;; it++) {
            const bool running = wr && !err && (uint32_t) p1_pos(r) < pstop;
            RP_BATCH(running)
            const uint32_t p = (uint32_t) p1_pos(r);
            uint32_t kind, ln, off, nbits;
            if (!par_tok<T>(rin, r, a.in, a.inlen, tid, lt, dt, &kind, &v, &ln, &off, &nbits) ||
                p + nbits > cbits) {
                err = true;
                continue;
            }
            if (part && (op + (kind == 1 ? ln : kind == 0 ? 1 : 0) > lim || rp + (kind == 1) > JD_RP_MAXREC)) {
                pstop = p;                        /* this token is the serial decoder's ... */
                if (kind == 0 && op >= lim) {
                    pfl = 1;                      /* ... which stops before it too */
                } else if (kind == 1 && op + ln > lim && rp + 1 <= JD_RP_MAXREC && off <= op - wlo) {
                    /* ... or split like copybytes: what fits now, the rest
                     * pending (its bits consumed) */
                    const uint32_t fit = lim - op;
                    if (fit) {
                        if (off == 1 && lastv >= 0) {
                            for (uint32_t k = 0; k < fit; k++) ob[op + k] = (uint8_t) lastv;
                            a.recs[rp++] = (uint64_t) op;
                        } else {
                            a.recs[rp++] = (uint64_t) op | ((uint64_t) fit << 17) | ((uint64_t) off << 32);
                        }
                    }
                    op = lim;
                    ppl = ln - fit;
                    ppo = off;
                    pfl = 1;
                    pstop = p + nbits;
                }
                continue;
            }
            if (kind == 0) {
                ob[op++] = (uint8_t) v;
                lastv = (int32_t) (v & 0xff);
#pragma unroll
                for (int k2 = 0; k2 < 2; k2++) {
                    const uint32_t e3 = p1_root(lt, LROOT, r.bb);
                    const uint32_t L3 = e3 & 15, s3 = (e3 >> 4) & 0xfff;
                    if (!(L3 != 0 && s3 < 256 && (uint32_t) p1_pos(r) < pstop && op < lim)) break;
                    p1_take(r, L3);
                    ob[op++] = (uint8_t) s3;
                    lastv = (int32_t) s3;
                }
            } else if (kind == 1) {
                if (off > op - wlo) { err = true; continue; }
                if (off == 1 && lastv >= 0) {
                    /* a fill: written now, its record slot left empty (the
                     * spans' record counts include it) */
                    for (uint32_t k = 0; k < ln; k++) ob[op + k] = (uint8_t) lastv;
                    a.recs[rp++] = (uint64_t) op;
                } else {
                    a.recs[rp++] = (uint64_t) op | ((uint64_t) ln << 17) | ((uint64_t) off << 32);
                    lastv = -1;
                }
                op += ln;
            }
        }
        /* the new end: the part thread's stop, or the last span's end */
        const uint32_t lastl = cutlane < T ? cutlane : endlane;
        if (tid == 0) s.ctl[2] = 0;
        __syncthreads();
        if (err) s.ctl[2] = 1;
        if (tid == lastl) { s.ctl[3] = op; s.ctl[4] = rp; s.ctl[5] = pstop; s.ctl[6] = ppl; s.ctl[7] = ppo | (pfl << 31); }
        __syncthreads();
        RPC_TICK(4);
        if (s.ctl[2]) break;                                              /* SERIAL */
        const uint32_t npos = s.ctl[3], nrp = s.ctl[4], nbit = s.ctl[5];
        const uint32_t nppl = s.ctl[6], nppo = s.ctl[7] & 0x7fffffffu, npfl = s.ctl[7] >> 31;
        __syncthreads();
        pos = npos;
        nrec = nrp;
        if (cutlane < T) {
            cmode = JD_RS_HUFF; cfin = fin; cbit = nbit; cpos = pos; cnrec = nrec; ctab = newtab;
            cplen = nppl; cpoff = nppo; fclean = npfl;
            status = JD_RST_FULL;
            break;
        }
        if (trunc) {
            cmode = JD_RS_HUFF; cfin = fin; cbit = nbit; cpos = pos; cnrec = nrec; ctab = newtab;
            status = JD_RST_NEEDINPUT;
            clean = tclean;
            break;
        }
        /* the header reader continues after the end-of-block symbol */
        const uint32_t ce = eobk * T + endlane;
        const uint32_t after = (s.eps[ce] >> 4) + (s.eps[ce] & 15);
        rd_init(R, after >> 3);
        if (after & 7) rd_bits(R, after & 7, &v);
        newtab = false;
        __syncthreads();
        if (fin) {
            cmode = JD_RS_ENDED; cfin = 1; cbit = after; cpos = pos; cnrec = nrec; ctab = false;
            status = JD_RST_ENDED;
            break;
        }
        mode = JD_RS_HEADER;
    }
#undef RP_BATCH
    /* the records are this workgroup's own global stores: every one must
     * have reached memory before the resolve's loads of them (other lanes) */
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    RPC_TICK(5);
    /* resolve the records before the clean point, 64 at a time, in LDS by
     * wave 0 (the rounds of k_inflate_resolve: a record waits for the
     * earlier records of its group whose destinations hold its source) */
    /* all waves (NW > 1): wave w takes groups w, w + NW, ...; the walks'
     * LDS (free now) holds every record's destination and length, so a
     * record's dependencies -- the records whose destinations overlap its
     * source -- are found by binary search over all of them: the ones in
     * its own group as in the one-wave rounds, the ones in earlier groups
     * through those groups' done flags (a group only waits on earlier
     * groups, and each wave takes its groups in order, so the earliest
     * unfinished group can always go on) */
    constexpr uint32_t RCAP = (PW / 32 + 2 * PAR_NCK + 2 * PAR_NEOB) * T;
    const bool allw = NW > 1 && cnrec <= RCAP &&
                      (cnrec + 63) / 64 <= RpShared<NW>::LV * T / 2;
    if (allw) {
        uint32_t* RD = s.bm;                          /* bm, ckp, ckc, eps, eo */
        uint32_t* GD = (uint32_t*) &s.jt[0][0];       /* group done flags      */
        const uint32_t ng = (cnrec + 63) / 64;
        for (uint32_t i = tid; i < cnrec; i += T) {
            const uint64_t rc = a.recs[i];
            RD[i] = ((uint32_t) rc & 0x1ffff) | ((((uint32_t) rc >> 17) & 0x1ff) << 17);
        }
        for (uint32_t i = tid; i < ng; i += T) GD[i] = 0;
        __syncthreads();
        for (uint32_t g = wv; g < ng; g += NW) {
            const uint32_t gb = g * 64, i = gb + lane;
            const bool m = i < cnrec;
            const uint32_t x = m ? RD[i] : 0;
            const uint32_t d = m ? x & 0x1ffff : 0xffffffffu;
            const uint32_t len = m ? x >> 17 : 0;
            const uint32_t off = m ? (uint32_t) (a.recs[i] >> 32) & 0xffff : 0;
            const uint32_t s0 = d - off, s1 = min(d, s0 + len);
            /* j0: first record ending after s0; j1: first starting at or after s1 */
            uint32_t j0 = 0, j1 = 0;
            if (m && off && len) {
                uint32_t lo2 = 0, hi2 = i;
                while (lo2 < hi2) {
                    const uint32_t md = (lo2 + hi2) >> 1, y2 = RD[md];
                    if ((y2 & 0x1ffff) + (y2 >> 17) <= s0) lo2 = md + 1; else hi2 = md;
                }
                j0 = lo2;
                hi2 = i;
                while (lo2 < hi2) {
                    const uint32_t md = (lo2 + hi2) >> 1;
                    if ((RD[md] & 0x1ffff) < s1) lo2 = md + 1; else hi2 = md;
                }
                j1 = lo2;
            }
            /* in this group: bits [max(j0, gb), min(j1, i)) - gb; earlier
             * groups: [j0 / 64, (min(j1, gb) - 1) / 64] */
            const uint32_t a0 = max(j0, gb), a1 = min(j1, i);
            const uint64_t dep = a0 < a1 ? (((a1 - gb) >= 64 ? ~0ull : ((1ull << (a1 - gb)) - 1)) &
                                            ~((1ull << (a0 - gb)) - 1)) : 0ull;
            const uint32_t ea = min(j1, gb);
            const uint32_t ga = j0 < ea ? j0 / 64 : 1u, gz = j0 < ea ? (ea - 1) / 64 : 0u;
            uint64_t U = __ballot(m && len);
            while (U) {
                bool inter = true;
                for (uint32_t k = ga; k <= gz; k++)
                    inter = inter && __hip_atomic_load(&GD[k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
                const bool ready = ((U >> lane) & 1) && !(U & dep) && inter;
                if (ready) rp_copy(ob, d, len, off);
                __builtin_amdgcn_s_waitcnt(0xc07f);      /* lgkmcnt(0) */
                __builtin_amdgcn_wave_barrier();
                const uint64_t R2 = __ballot(ready);
                if (!R2) __builtin_amdgcn_s_sleep(1);   /* an earlier group still runs */
                U &= ~R2;
            }
            if (lane == 0) __hip_atomic_store(&GD[g], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    uint64_t rnext = !allw && wv == 0 && lane < cnrec ? a.recs[lane] : 0;     /* the next group's records */
    if (!allw && wv == 0)
    for (uint32_t g = 0; g < cnrec; g += 64) {
        const uint32_t i = g + lane;
        const bool m = i < cnrec;
        const uint64_t rc = rnext;
        /* loaded one group ahead: the load overlaps this group's rounds */
        rnext = g + 64 + lane < cnrec ? a.recs[g + 64 + lane] : 0;
        const uint32_t d = m ? (uint32_t) rc & 0x1ffff : 0xffffffffu;
        const uint32_t len = m ? ((uint32_t) rc >> 17) & 0x1ff : 0;
        const uint32_t off = m ? (uint32_t) (rc >> 32) & 0xffff : 0;
        const uint32_t e = m ? d + len : 0xffffffffu;
        const uint32_t s0 = d - off, s1 = min(d, s0 + len);
        uint32_t j0 = 0, j1 = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1) {
            const uint32_t ej = (uint32_t) __shfl((int) e, (int) (j0 + step - 1));
            if (ej <= s0) j0 += step;
            const uint32_t dj = (uint32_t) __shfl((int) d, (int) (j1 + step - 1));
            if (dj < s1) j1 += step;
        }
        const uint32_t jend = min(j1, lane);
        const uint64_t dep = (m && off && j0 < jend)
            ? (((jend >= 64) ? ~0ull : ((1ull << jend) - 1)) & ~((1ull << j0) - 1)) : 0ull;
        uint64_t U = __ballot(m && len);
        while (U) {
            const bool ready = ((U >> lane) & 1) && !(U & dep);
            if (ready) {
                if (!off) {
                    for (uint32_t k = 0; k < len; k++) ob[d + k] = 0;
                } else if (off >= len) {
                    for (uint32_t k = 0; k < len; k += 4) ob_put(ob, d + k, ob_word(ob, d - off + k), min(4u, len - k));
                } else if (off < 4) {
                    const uint32_t pb = ob_word(ob, d - off);
                    uint32_t ph = 0;
                    for (uint32_t k = 0; k < len; k += 4) {
                        uint32_t w = 0;
#pragma unroll
                        for (uint32_t j = 0; j < 4; j++) {
                            w |= ((pb >> (8 * ph)) & 0xff) << (8 * j);
                            ph = ph + 1 == off ? 0 : ph + 1;
                        }
                        ob_put(ob, d + k, w, min(4u, len - k));
                    }
                } else {
                    for (uint32_t k = 0, km = 0; k < len;) {
                        const uint32_t n = min(min(4u, len - k), off - km);
                        ob_put(ob, d + k, ob_word(ob, d - off + km), n);
                        k += n;
                        km += n;
                        if (km == off) km = 0;
                    }
                }
            }
            __builtin_amdgcn_s_waitcnt(0xc07f);      /* lgkmcnt(0) */
            __builtin_amdgcn_wave_barrier();
            U &= ~__ballot(ready);
        }
    }
    __syncthreads();
    RPC_TICK(6);
    for (uint32_t o = RP_W + tid * 16; o < cpos; o += T * 16) *(uint4*) (a.out + (o - RP_W)) = *(const uint4*) (ob + o);
    RPC_TICK(7);
#ifdef RP_CLOCK
    if (tid == 0)
        printf("RPC in=%u out=%u rec=%u st=%u hdr=%.1f a1=%.1f a2=%.1f chain=%.1f write=%.1f rest=%.1f resolve=%.1f copy=%.1f\n",
               a.inlen, cpos - RP_W, cnrec, status, rpc[0] / 100.0, rpc[1] / 100.0, rpc[2] / 100.0, rpc[3] / 100.0,
               rpc[4] / 100.0, rpc[5] / 100.0, rpc[6] / 100.0, rpc[7] / 100.0);
#endif
#undef RPC_TICK
    if (tid == 0) {
        S->mode = cmode;
        S->fin = cfin;
        S->plen = cplen;
        S->poff = cpoff;
        S->srem = csrem;
        S->status = status;
        S->err = 0;
        S->pad = status == JD_RST_NEEDINPUT ? clean : status == JD_RST_FULL ? fclean : 0u;
        S->bit = cbit;
        S->produced = cpos - RP_W;
        head_to_host(S, a.hhead);
    }
    if (cmode == JD_RS_HUFF && ctab) {
        for (uint32_t i = tid; i < LT_CAP; i += T) S->lt[i] = s.t.lt[i];
        for (uint32_t i = tid; i < DT_CAP; i += T) S->dt[i] = s.t.dt[i];
    }
}

#undef PAR_BATCH

#ifndef JD_RP_NW
#define JD_RP_NW 4u                 /* waves of the parallel resume */
#endif
extern "C" int jdk_inflate_rpar_launch(const JdRparLaunch* L)
{
    hipStream_t st = (hipStream_t) L->stream;
    JdRparLaunch a = *L;
    JDPROF_RUN(JDK_INFLATE_RPAR, st, (k_inflate_rpar<JD_RP_NW><<<1, 64 * JD_RP_NW, 0, st>>>(a)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
