/*
 * jd_deflate.hip -- gfx950 deflate engine for independent blocks.
 *
 * Every block (<= 64 KiB) is compressed exactly as a fresh reference
 * deflator would compress it with DEFLT_FLUSH (DEFLT_END for the last block
 * of a stream): deflator_reset + deflator_deflate, deflator.c:455-786.
 *
 * The reference's sequential hot loop (compress2 :2767 -> getmatch2 :2606 ->
 * skipbytes2 :2730 -> flushblock :1725) is split into data-parallel stages:
 *
 *   k_chains<4>  hash-4 chain links for every position   (mhlist/mchain)
 *   k_chains<3>  hash-3 chain links for every position   (shlist/schain)
 *   k_match      chain walk for every position, both chain budgets and the
 *                3-byte candidate, all in LDS                (getmatch2)
 *   k_parse      the lazy / greedy parse + block-split heuristic, one lane
 *                per block, reading the match records      (compress2/1)
 *   k_emit       per deflate block: histogram, Huffman build, trees, and
 *                bit packing by a workgroup prefix scan     (flushblock)
 *   k_scan / k_compact  concatenate the per-block bitstreams
 *
 * Chains are a pure function of the data, which is
 * what makes k_chains/k_match order-independent.
 */
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "jd_device.h"
#include "jd_kernels.h"
#include "jd_prof.h"

/* the block pipeline's match stage: the lowest level that takes the slices
 * + k_match_sl (bit-exact) instead of the hash-4 links
 * + k_match.  JD_K2_SLICES=1 builds it for every level (the parity-test
 * library lib_sl). */
#ifndef JD_K2_SLICES
#define JD_K2_SLICES 0
#endif
#ifndef K2S_MINLEVEL
#define K2S_MINLEVEL 10
#endif
#define K2S_FROM (JD_K2_SLICES ? 1 : K2S_MINLEVEL)

/* ------------------------------------------------------------------------ */
/* helpers                                                                   */
/* ------------------------------------------------------------------------ */
__device__ static inline uint32_t blk_len(uint64_t n, uint32_t bs, uint32_t b)
{
    uint64_t base = (uint64_t) b * bs;
    uint64_t left = n - base;
    return left < bs ? (uint32_t) left : bs;
}

/* 4 bytes at block-local position p, zero past the block end (the reference
 * window is zeroed past inputend, deflator.c:499-502); returned as the
 * big-endian head of gethead :1931 */
__device__ static inline uint32_t head_be(const uint8_t* __restrict__ blk,
                                          uint32_t p, uint32_t len,
                                          const uint8_t* __restrict__ bufend)
{
    const uint8_t* a = blk + (p & ~3u);
    uint32_t v;
    if (p + 4 <= len && a + 8 <= bufend) {
        JD_CHECK(a, 8, bufend);
        uint32_t w0 = *(const uint32_t*) a;
        uint32_t w1 = *(const uint32_t*) (a + 4);
        v = __builtin_amdgcn_alignbyte(w1, w0, p & 3);
    } else {
        v = 0;
        for (uint32_t k = 0; k < 4; k++)
            if (p + k < len) {
                JD_CHECK(blk + p + k, 1, bufend);
                v |= (uint32_t) blk[p + k] << (8 * k);
            }
    }
    return __builtin_bswap32(v);
}

/* ------------------------------------------------------------------------ */
/* K1: chain links.  MODE 4: 16-bit hash of 4 bytes, output = distance to the
 * previous position in the same bucket (0 = none).  MODE 3: 14-bit hash of 3
 * bytes, output = that previous position itself (0 = none; position 0 reads
 * as empty exactly as shlist value 0 does, deflator.c:2681).
 * Position 0 is filed under bucket 0 in both (aux3/aux4 start at 0,
 * deflator.c:480-485).
 *
 * One workgroup per block walks it in batches of 1024 positions, in a
 * three-stage pipeline with one barrier per batch: all waves hash batch k+1,
 * wave 0 files batch k into the head table, all waves write the links of
 * batch k-1.  Filing is an atomic 16-bit exchange per position
 * (ds_mskor_rtn_b32 on the half-word of its bucket), 16 instructions per
 * batch issued by wave 0 in position order (LDS instructions of one wave
 * execute in issue order).  Within one instruction, lanes with the same
 * bucket are serialised by the LDS in an order the ISA does not specify, so
 * the result is checked, not assumed: the exchanges were applied in lane
 * order exactly when no lane got back its own or a higher lane's position
 * (a serialisation in which every lane receives an earlier position is
 * increasing).  The hardware measured does apply lane order (0 exceptions
 * in 5e7 lanes, scratch/xchg); a block that ever fails the check is filed
 * again serially, one position at a time (chains_serial), so the chains
 * equal the reference's serial insertion whatever the hardware does.
 * ------------------------------------------------------------------------ */

/* old 32-bit LDS word; bits `mask` replaced by `data` (16-bit exchange) */
__device__ static inline uint32_t lds_mskor_rtn(uint32_t addr, uint32_t mask, uint32_t data)
{
    uint32_t r;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=v"(r) : "v"(addr), "v"(mask), "v"(data) : "memory");
    return r;
}

/* old 32-bit LDS word; `data` added (the slices' 16-bit counts) */
__device__ static inline uint32_t lds_add_rtn(uint32_t addr, uint32_t data)
{
    uint32_t r;
    asm volatile("ds_add_rtn_u32 %0, %1, %2" : "=v"(r) : "v"(addr), "v"(data) : "memory");
    return r;
}

/* bytes < 16 in a word (exact per byte) */
__device__ static inline uint32_t low_bytes(uint32_t w)
{
    const uint32_t t = w & 0xf0f0f0f0u;
    const uint32_t y = ~(((t & 0x7f7f7f7fu) + 0x7f7f7f7fu) | t | 0x7f7f7f7fu);
    return __builtin_popcount(y);
}

/* Stream mode (single-window streams, deflator.c:1818-1911): blocks are
 * 32 KiB units of one stream.  MODE 4 first files the previous unit's
 * positions (warm-up, no links written): links reach back less than 32 KiB,
 * so the head table then holds exactly the reference's.  MODE 3 starts from
 * inc3, the latest position of every bucket before the unit (k_s3last /
 * k_s3scan): the 3-chain is read modulo 65536 at any distance (pos3 is a
 * uint16, deflator.c:2641-2643, 2681-2684).  Hash bytes past the stream end
 * read as zero, and only stream position 0 is filed under bucket 0. */
/* stream: the bucket a listed position is filed under instead (the stale
 * hashes of the positions around a mid-stream flush); HS = not filed */
template <int MODE>
__device__ static inline uint32_t ov_bucket(const JdOverride* ov, uint32_t nov, uint64_t gp, uint32_t h)
{
    constexpr uint32_t HS = MODE == 4 ? 65536u : 16384u;
    if (nov && gp >= ov[0].pos && gp <= ov[nov - 1].pos) {
        for (uint32_t i = 0; i < nov; i++) {
            if (ov[i].pos == gp) {
                const uint32_t v = MODE == 4 ? ov[i].h4 : ov[i].h3;
                return v == 0xffffffffu ? HS : v;
            }
        }
    }
    return h;
}

/* hash bucket of position p as k_chains files it (HS: not filed) */
template <int MODE>
__device__ static inline uint32_t chains_bucket(const uint8_t* blk, const uint8_t* bufend,
                                                uint64_t ws, uint32_t p, uint32_t len,
                                                uint32_t dlen, int stream, uint32_t dsz,
                                                const JdOverride* ov, uint32_t nov)
{
    constexpr uint32_t HS = MODE == 4 ? 65536u : 16384u;
    const uint64_t gp = ws + p;
    if (p >= len) return HS;
    if (stream && gp < dsz && gp + 4 > dsz) return ov_bucket<MODE>(ov, nov, gp, HS);
    if (stream ? gp == dsz : p == 0) return ov_bucket<MODE>(ov, nov, gp, 0);
    const uint32_t hd = head_be(blk, p, dlen, bufend);
    const uint32_t h = MODE == 4 ? (hd * 0x1e35a7bdu) >> 16 : ((hd >> 8) * 0x1e35a7bdu) >> 18;
    return stream ? ov_bucket<MODE>(ov, nov, gp, h) : h;
}

/* k_chains' filing done one position at a time by wave 0 (the reference's
 * serial insertion, deflator.c:2630-2645): the hashes of 64 positions are
 * computed at once, then lane i files position i after lane i-1 */
template <int MODE>
__device__ __attribute__((noinline)) static void chains_serial(
    uint16_t* head, const uint8_t* blk, const uint8_t* bufend, uint64_t ws, uint32_t len,
    uint32_t own, uint32_t dlen, uint16_t* dst, int stream, const uint32_t* inc3, uint32_t b,
    uint32_t dsz, uint32_t pbase, const JdOverride* ov, uint32_t nov)
{
    constexpr uint32_t HS = MODE == 4 ? 65536u : 16384u;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < HS; i += blockDim.x)
        head[i] = (uint16_t) (MODE == 3 ? ((inc3) ? inc3[(uint64_t) b * HS + i] : 0) : 0xffffu);
    __syncthreads();
    if (tid < 64) {
        for (uint32_t g = 0; g < len; g += 64) {
            const uint32_t p = g + tid;
            const uint32_t h = chains_bucket<MODE>(blk, bufend, ws, p, len, dlen, stream, dsz, ov, nov);
            for (uint32_t k = 0; k < 64; k++) {
                if (tid == k && h < HS) {
                    const uint32_t q = head[h];
                    head[h] = (uint16_t) ((pbase + p) & 0xffffu);
                    if (p >= own) {
                        uint32_t v = q;
                        if (MODE == 4) {
                            v = q == 0xffff ? 0 : p - q;
                            if (stream && v >= JD_WSIZE) v = 0;
                        }
                        dst[p] = (uint16_t) v;
                    }
                }
                __builtin_amdgcn_s_waitcnt(0);
            }
        }
    }
}

/* Block-mode slices (k_chains<4, false, true>, round 6).  A position's
 * hash-4 chain is exactly the earlier positions of its bucket, newest first
 * (SURVEY App. A 2), so with the block's positions sorted by (bucket,
 * position) -- S -- the chain of p is the contiguous slice S[r-1], S[r-2], ...
 * below p's own rank r.  k_match then loads its candidates 8 at a time with
 * no pointer chase (tests/support/decomp_emu.c models it, emu_slice).
 *
 * The sort is a counting sort done by the same pipeline: wave 0 files each
 * batch with 16 atomic adds in position order (ds_add_rtn on the bucket's
 * 16-bit count), so a position gets back c(p), the number of earlier
 * positions of its bucket; stage C stores (bucket, c) to W.  Then the counts
 * become bucket starts (a workgroup scan), r(p) = start + c(p), S is
 * scattered into the LDS table and written out, and each position's W becomes
 * r | n << 16 with n = its candidates within the 32 KiB window, capped at the
 * level's chain budget.  The order of same-bucket lanes inside one add is not
 * assumed: S must be increasing inside every bucket (S[r-1] < p wherever
 * c(p) > 0), and a block where it is not is sorted again by a serial filing
 * (never observed, as for the exchanges).  The hash-4 links the parser's rare
 * held-long walk reads (prev4) are p - S[r-1]. */
template <bool SL>
struct SlOut {
    uint16_t* s;            /* S, block-relative positions, bs per block     */
    uint32_t* w;            /* W, r | min(window candidates, chain) << 16    */
    uint32_t chain;
};

/* serial filing of the counts (the slices' fallback): lane k of wave 0 files
 * position g + k after lane k - 1, writing (bucket | c << 16) to W */
__device__ __attribute__((noinline)) static void slices_serial(
    uint16_t* head, const uint8_t* blk, const uint8_t* bufend, uint32_t len, uint32_t dlen,
    uint32_t* w, uint32_t* hlast_sh)
{
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 65536 + 8; i += blockDim.x) head[i] = 0;
    __syncthreads();
    if (tid < 64) {
        for (uint32_t g = 0; g < len; g += 64) {
            const uint32_t p = g + tid;
            const uint32_t h = chains_bucket<4>(blk, bufend, 0, p, len, dlen, 0, 0, nullptr, 0);
            for (uint32_t k = 0; k < 64; k++) {
                if (tid == k && h < 65536u) {
                    if (p == 65535u) {
                        *hlast_sh = h;
                    } else {
                        const uint32_t c = head[h];
                        head[h] = (uint16_t) (c + 1);
                        w[p] = h | (c << 16);
                    }
                }
                __builtin_amdgcn_s_waitcnt(0);
            }
        }
    }
    __threadfence();
    __syncthreads();
}


/* k_chains<4, false, true>'s tail: counts -> bucket starts -> ranks -> S,
 * W and the links, then the order check (see "Block-mode slices" above).
 * head: the 64 Ki 16-bit counts (LDS); W holds (bucket | c << 16) for every
 * position but 65535 (whose bucket is *hlast_sh, HS if none). */
__device__ static void k_chains_sl_tail(uint16_t* head, const uint8_t* blk, const uint8_t* bufend,
                                        uint32_t len, uint32_t dlen, uint32_t b, uint32_t bs,
                                        uint16_t* dst, const SlOut<true>& so, bool serial,
                                        uint32_t* hlast_sh)
{
    constexpr uint32_t HS = 65536u, NPT = 64;      /* positions (and buckets) per thread */
    __shared__ uint32_t wtot[16], bad_sh, clast_sh;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t* const wb = so.w + (uint64_t) b * bs;
    uint16_t* const sb = so.s + (uint64_t) b * bs;
    for (int attempt = serial ? 1 : 0; attempt < 2; attempt++) {
        if (attempt) slices_serial(head, blk, bufend, len, dlen, wb, hlast_sh);
        if (tid == 0) bad_sh = 0;
        __syncthreads();
        const uint32_t hl = *hlast_sh;
        if (tid == 0) clast_sh = hl < HS ? head[hl] : 0;
        /* exclusive scan of the counts: thread t owns buckets [64 t, 64 t + 64) */
        uint4 cv[8];
        uint32_t tot = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            cv[j] = ((const uint4*) head)[tid * 8 + j];
            tot += (cv[j].x & 0xffff) + (cv[j].x >> 16) + (cv[j].y & 0xffff) + (cv[j].y >> 16) +
                   (cv[j].z & 0xffff) + (cv[j].z >> 16) + (cv[j].w & 0xffff) + (cv[j].w >> 16);
        }
        uint32_t inc = tot;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t) __shfl_up((int) inc, d);
            if (lane >= (uint32_t) d) inc += y;
        }
        if (lane == 63) wtot[wv] = inc;
        __syncthreads();
        uint32_t run = inc - tot;
        for (uint32_t w = 0; w < wv; w++) run += wtot[w];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            uint32_t* x = (uint32_t*) &cv[j];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t lo = x[k] & 0xffff, hi = x[k] >> 16;
                x[k] = (run & 0xffff) | ((run + lo) << 16);
                run += lo + hi;
            }
        }
        __syncthreads();        /* every count read (and clast_sh) before the starts replace them */
#pragma unroll
        for (int j = 0; j < 8; j++) ((uint4*) head)[tid * 8 + j] = cv[j];
        __syncthreads();
        /* ranks: r = start + c (+1 past position 65535's bucket, which the
         * counts left out); W becomes r | c << 16 (each thread reads back
         * only the W words it wrote itself) */
#pragma unroll 2
        for (uint32_t i = 0; i < NPT; i++) {
            const uint32_t p = i * 1024 + tid;
            if (p < len) {
                uint32_t h, c;
                if (p == 65535u) { h = hl; c = clast_sh; }
                else { const uint32_t t = wb[p]; h = t & 0xffff; c = t >> 16; }
                const uint32_t r = head[h] + c + (p != 65535u && h > hl ? 1u : 0u);
                wb[p] = (r & 0xffff) | (c << 16);
            }
        }
        __syncthreads();        /* every start read before S overwrites them */
#pragma unroll 2
        for (uint32_t i = 0; i < NPT; i++) {
            const uint32_t p = i * 1024 + tid;
            if (p < len) head[wb[p] & 0xffff] = (uint16_t) p;
        }
        __syncthreads();
        /* links, W and the order check: S[r-1] < p wherever c > 0 */
        bool bad = false;
#pragma unroll 2
        for (uint32_t i = 0; i < NPT; i++) {
            const uint32_t p = i * 1024 + tid;
            if (p < len) {
                const uint32_t t = wb[p], r = t & 0xffff, c = t >> 16;
                uint32_t link = 0, nw = 0;
                if (c) {
                    const uint32_t q = head[r - 1];
                    bad |= q >= p;
                    link = p - q;
                    /* candidates within the window (p - q <= 32767), at most
                     * chain: the lowest index i in [r - m, r) with S[i] in reach */
                    const uint32_t m = c < so.chain ? c : so.chain;
                    const uint32_t lim = p > 32767u ? p - 32767u : 0u;
                    uint32_t lo = r - m;
                    if (head[lo] < lim) {
                        /* S[lo] out of reach, S[r - 1] within it (or none) */
                        uint32_t hi = r;
                        while (hi - lo > 1) {
                            const uint32_t mid = (lo + hi) >> 1;
                            if (head[mid] < lim) lo = mid; else hi = mid;
                        }
                        lo = hi;
                    }
                    nw = r - lo;
                }
                dst[p] = (uint16_t) link;
                wb[p] = r | (nw << 16);
            }
        }
        if (__ballot(bad) && lane == 0) bad_sh = 1;
        /* S out, 16 bytes per store */
        for (uint32_t i = tid; i * 8 < len; i += 1024) {
            if (i * 8 + 8 <= len) ((uint4*) sb)[i] = ((const uint4*) head)[i];
            else for (uint32_t k = i * 8; k < len; k++) sb[k] = head[k];
        }
        __syncthreads();
        if (!bad_sh) break;
    }
}


#ifndef CH_NPT
#define CH_NPT 2u               /* positions per thread per k_chains batch */
#endif

/* OV: the launch has an override list (a stream piece after a flush); the
 * check costs k_chains<3> its second workgroup per CU, so it is compiled
 * only where it is needed.  SL: block-mode slices (above). */
template <int MODE, bool OV = false, bool SL = false>
__global__ __launch_bounds__(1024) void k_chains(const uint8_t* __restrict__ in,
                                                 uint64_t n, uint32_t bs,
                                                 uint16_t* __restrict__ out,
                                                 uint32_t* __restrict__ dsg,
                                                 int stream, const uint32_t* __restrict__ inc3,
                                                 uint32_t dsz, const JdOverride* __restrict__ ov,
                                                 uint32_t nov, SlOut<SL> so = SlOut<SL>{})
{
    static_assert(!SL || (MODE == 4 && !OV), "slices: block-mode hash-4 chains only");
    constexpr int HB = MODE == 4 ? 16 : 14;
    constexpr uint32_t HS = 1u << HB;
    __shared__ __attribute__((aligned(16))) uint16_t head[HS + 8];   /* + dummy slot */
    /* batches of NPT x 1024 positions (NPT per thread), exchanged between
     * the pipeline stages through two buffers each: stage A writes batch
     * it's buckets while wave 0 reads batch it-1's, and wave 0 writes batch
     * it-1's results while stage C reads batch it-2's (a thread keeps its own
     * positions' buckets in registers for stage C).  Two positions per thread
     * halve the barriers and the loop's scalar work per position: k_chains<4>
     * 4.02 -> 3.70, k_chains<3> 2.43 -> 2.25 ms per GiB of text
     * (gpurun_out/r6v, r6zc) */
    constexpr uint32_t NPT = CH_NPT, BT = 1024 * NPT;
    /* MODE 4's dummy slot HS = 65536 needs 17 bits */
    using HashT = typename std::conditional<MODE == 4, uint32_t, uint16_t>::type;
    __shared__ HashT sh_h[2][BT];
    __shared__ uint16_t sh_r[2][BT];
    __shared__ uint32_t nlow_sh;
    __shared__ uint32_t order_bad;      /* an exchange left lane order   */
    __shared__ uint32_t hlast_sh;       /* SL: bucket of position 65535   */
    (void) hlast_sh;
    uint32_t hlast = HS;                /* MODE 4: bucket of position 65535 */
    /* stream bit 1: test hook, file serially (JD_CHAINS_SERIAL=1) */
    const bool force_serial = (stream & 2) != 0;
    stream &= 1;
    if (SL) stream = 0;
    if (SL && threadIdx.x == 0) hlast_sh = HS;

    const uint32_t b = blockIdx.x;
    /* positions [ws, ws + len) are filed; links are written from `own` on */
    const uint64_t ub = (uint64_t) b * bs;
    const uint32_t warm = (stream && MODE == 4) ? (ub >= JD_WSIZE ? JD_WSIZE : (uint32_t) ub) : 0;
    const uint64_t ws = ub - warm;
    const uint32_t len = warm + blk_len(n, bs, b), own = warm;
    /* bytes a hash may read: the block, or the rest of the stream */
    const uint64_t dl64 = stream ? n - ws : (uint64_t) len;
    const uint32_t dlen = dl64 > 0xffffffffull ? 0xffffffffu : (uint32_t) dl64;
    const uint8_t* blk = in + ws;
    const uint8_t* bufend = in + n;
    uint16_t* dst = out + ws;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    /* inputs under 4 bytes: no batches, the serial filing does it all */
    const uint32_t nbatch = n >= 4 ? (len + BT - 1) / BT : 0;
    /* MODE 3 stores positions modulo 65536 (0 = empty, as shlist 0) */
    const uint32_t pbase = (stream && MODE == 3) ? (uint32_t) (ws & 0xffff) : 0;

    if (MODE == 3) {
        for (uint32_t i = tid; i < HS + 8; i += 1024)
            head[i] = (uint16_t) ((inc3 && i < HS) ? inc3[(uint64_t) b * HS + i] : 0);
    } else if (SL) {
        /* bucket counts */
        for (uint32_t i = tid * 8; i < HS + 8; i += 1024 * 8) *(uint4*) &head[i] = make_uint4(0, 0, 0, 0);
    } else {
        for (uint32_t i = tid * 8; i < HS + 8; i += 1024 * 8)
            *(uint4*) &head[i] = make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
    }

    /* the 4 bytes of a position come from the two dwords around it; the
     * dwords of each 1024 positions are loaded JD_CHPF x 1024 positions
     * ahead (a batch iteration is shorter than one memory latency) */
#ifndef JD_CHPF
#define JD_CHPF 8
#endif
    /* k_chains<3> prefetches half as far: at 62 VGPRs it keeps two
     * workgroups per CU (8 waves per SIMD) */
#ifndef JD_CHPF3
#define JD_CHPF3 4
#endif
    constexpr uint32_t PF = MODE == 3 ? JD_CHPF3 : JD_CHPF;
    uint32_t nw0[PF], nw1[PF];
    /* each dword holding a byte of the buffer is loaded (one crossing the
     * buffer end as the buffer's last 4 bytes, shifted into place where the
     * words are used), so every position's hash comes from these two words
     * and the batch loop holds no other global load: the loads stay in
     * flight across batches (a byte-wise slow path for a block's last
     * positions made the compiler wait for all loads at every batch:
     * k_chains<4> 4.72 -> 3.90 ms, <3> 2.76 -> 2.36).  Inputs under 4 bytes
     * are filed serially. */
    /* a batch whose dwords all lie inside the buffer (every batch but the
     * buffer's last one or two) takes the plain loads; the choice is
     * wave-uniform */
    auto inside = [&](uint32_t base) { return blk + base + 1024 + 8 <= bufend; };
    auto fetch = [&](uint32_t bb, uint32_t& w0, uint32_t& w1) {
        const uint32_t p = bb + tid;
        const uint8_t* a = blk + (p & ~3u);
        w0 = w1 = 0;
        if (inside(bb)) {
            if (p < dlen) {
                JD_CHECK(a, 8, bufend);
                w0 = *(const uint32_t*) a;
                w1 = *(const uint32_t*) (a + 4);
            }
        } else {
            if (n >= 4 && p < dlen && a < bufend) {
                const uint8_t* a0 = a + 4 <= bufend ? a : bufend - 4;
                JD_CHECK(a0, 4, bufend);
                __builtin_memcpy(&w0, a0, 4);
            }
            if (n >= 4 && p < dlen && a + 4 < bufend) {
                const uint8_t* a1 = a + 8 <= bufend ? a + 4 : bufend - 4;
                JD_CHECK(a1, 4, bufend);
                __builtin_memcpy(&w1, a1, 4);
            }
        }
    };
#pragma unroll
    for (uint32_t d = 0; d < PF; d++) {
        nw0[d] = nw1[d] = 0;
        if (d * 1024 < len) fetch(d * 1024, nw0[d], nw1[d]);
    }
    uint32_t nlow = 0;                  /* MODE 3: bytes < 16 (doshort guess) */
    if (MODE == 3 && tid == 0) nlow_sh = 0;
    if (tid == 0) order_bad = (force_serial || (n < 4 && len)) ? 1u : 0u;
    const uint32_t headw = (uint32_t) (uintptr_t) head;     /* LDS byte address */
    static_assert(PF % NPT == 0, "the prefetch covers whole batches");
    constexpr uint32_t PFB = PF / NPT;          /* batches in flight */
    HashT hq1[NPT], hq2[NPT];                   /* my buckets of batches it-1, it-2 */
#pragma unroll
    for (uint32_t j = 0; j < NPT; j++) hq1[j] = hq2[j] = (HashT) HS;
    for (uint32_t it0 = 0; it0 < nbatch + 2; it0 += PFB)
#pragma unroll
    for (uint32_t d = 0; d < PFB; d++) {
        const uint32_t it = it0 + d;
        if (it >= nbatch + 2) break;
        HashT hcur[NPT];
#pragma unroll
        for (uint32_t j = 0; j < NPT; j++) hcur[j] = (HashT) HS;
        /* stage A: buckets of batch it (HS: past the block end, a dummy) */
        if (it < nbatch)
#pragma unroll
        for (uint32_t j = 0; j < NPT; j++) {
            const uint32_t sl = d * NPT + j;                /* prefetch slot */
            const uint32_t base = it * BT + j * 1024, p = base + tid;
            uint32_t w0 = nw0[sl], w1 = nw1[sl];
            if (base + PF * 1024 < len) fetch(base + PF * 1024, nw0[sl], nw1[sl]);
            if (!inside(base)) {
                /* the buffer's last dwords were read as its last 4 bytes */
                const uint8_t* a = blk + (p & ~3u);
                if (a + 8 > bufend) {
                    if (a + 4 > bufend) {
                        w1 = 0;
                        w0 = a < bufend ? w0 >> (8 * (uint32_t) (a + 4 - bufend)) : 0u;
                    } else {
                        w1 = a + 4 < bufend ? w1 >> (8 * (uint32_t) (a + 8 - bufend)) : 0u;
                    }
                }
            }
            if (MODE == 3 && (p & 3) == 0 && p + 4 <= len && blk + p + 8 <= bufend) nlow += low_bytes(w0);
            uint32_t h = HS;
            const uint64_t gp = ws + p;
            /* stream with a dictionary of dsz bytes (deflator_setdctnr
             * :2106-2167): its positions up to dsz-4 are filed with their own
             * hash, its last three not at all, and the parse start dsz takes
             * bucket 0 (aux3/aux4 are still 0 there) */
            if (p < len && !(stream && gp < dsz && gp + 4 > dsz)) {
                h = 0;
                if (stream ? gp != dsz : p != 0) {
                    uint32_t x4 = __builtin_amdgcn_alignbyte(w1, w0, p & 3);
                    /* bytes at or past dlen read as zero (the zeroed window,
                     * deflator.c:499-502); dlen - p is 1..3 here */
                    if (p + 4 > dlen) x4 &= 0xffffffffu >> (8 * (4 - (dlen - p)));
                    const uint32_t hd = __builtin_bswap32(x4);
                    if (MODE == 4) h = (hd * 0x1e35a7bdu) >> 16;
                    else h = ((hd >> 8) * 0x1e35a7bdu) >> 18;
                }
            }
            /* stream: positions around an earlier flush take their stale
             * buckets (the launch's override list) */
            if (OV && stream && p < len) h = ov_bucket<MODE>(ov, nov, gp, h);
            /* MODE 4: position 65535's value is the empty marker 0xFFFF, so
             * it is not exchanged (the order check could not tell the two
             * apart); as the last position it is linked after the loop */
            if (MODE == 4 && p == 65535u && h < HS) {
                hlast = h;
                if (SL) hlast_sh = h;       /* its count would overflow 16 bits */
                h = HS;
            }
            hcur[j] = (HashT) h;
            sh_h[it & 1][j * 1024 + tid] = (HashT) h;
        }
        /* stage B: wave 0 files batch it-1, its 16 NPT groups in position
         * order, 16 at a time */
        if (tid < 64 && it >= 1 && it - 1 < nbatch) {
            const uint32_t k = (it - 1) & 1, base = (it - 1) * BT;
#pragma unroll
            for (uint32_t hf = 0; hf < NPT; hf++) {
                uint32_t hv[16], old[16], sh[16];
#pragma unroll
                for (int w = 0; w < 16; w++) hv[w] = sh_h[k][(hf * 16 + w) * 64 + lane];
                /* all 16 reads land before the first exchange is issued, so
                 * the exchanges go out back to back (a compiler wait for a
                 * later read would also wait for the exchanges before it) */
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(hv[0]), "+v"(hv[1]), "+v"(hv[2]), "+v"(hv[3]),
                               "+v"(hv[4]), "+v"(hv[5]), "+v"(hv[6]), "+v"(hv[7]),
                               "+v"(hv[8]), "+v"(hv[9]), "+v"(hv[10]), "+v"(hv[11]),
                               "+v"(hv[12]), "+v"(hv[13]), "+v"(hv[14]), "+v"(hv[15])
                             :: "memory");
#pragma unroll
                for (int w = 0; w < 16; w++) {
                    sh[w] = (hv[w] & 1) * 16;
                    if (SL) {
                        /* count of the bucket; the dummy slot HS takes the rest */
                        old[w] = lds_add_rtn(headw + (hv[w] >> 1) * 4, 1u << sh[w]);
                    } else {
                        const uint32_t val = (pbase + base + (hf * 16 + w) * 64 + lane) & 0xffffu;
                        old[w] = lds_mskor_rtn(headw + (hv[w] >> 1) * 4, 0xffffu << sh[w], val << sh[w]);
                    }
                }
                /* one wait for the 16 exchanges; the results depend on it */
                asm volatile("s_waitcnt lgkmcnt(0)"
                             : "+v"(old[0]), "+v"(old[1]), "+v"(old[2]), "+v"(old[3]),
                               "+v"(old[4]), "+v"(old[5]), "+v"(old[6]), "+v"(old[7]),
                               "+v"(old[8]), "+v"(old[9]), "+v"(old[10]), "+v"(old[11]),
                               "+v"(old[12]), "+v"(old[13]), "+v"(old[14]), "+v"(old[15])
                             :: "memory");
#pragma unroll
                for (int w = 0; w < 16; w++) sh_r[k][(hf * 16 + w) * 64 + lane] = (uint16_t) (old[w] >> sh[w]);
            }
        }
        /* stage C: links of batch it-2 */
        if (it >= 2) {
            const uint32_t k = it & 1;                  /* (it - 2) & 1 */
#pragma unroll
            for (uint32_t j = 0; j < NPT; j++) {
                const uint32_t p = (it - 2) * BT + j * 1024 + tid;
                const uint32_t hb = hq2[j];
                /* lane order check of wave 0's exchange of this wave's 64
                 * positions: the value a lane got back must not be the
                 * position of a higher lane of the same bucket (nor its own:
                 * kk = 0 is the empty marker equal to it) */
                if (SL) {
                    /* (bucket, count) for the tail; the order is verified there */
                    if (p < len && p != 65535u) so.w[(uint64_t) b * bs + p] = hb | ((uint32_t) sh_r[k][j * 1024 + tid] << 16);
                } else {
                    const uint32_t got = sh_r[k][j * 1024 + tid];
                    const uint32_t kk = (got - ((pbase + p) & 0xffffu)) & 0xffffu;
                    const bool sus = hb < HS && kk - 1u < 63u - lane;
                    if (__ballot(sus)) {
                        /* rare: the value may also be an earlier position or
                         * the empty marker equal to it mod 65536; it came from
                         * that lane only if the lane shares the bucket */
                        const uint32_t jl = sus ? lane + kk : lane;
                        const bool bad = sus && (uint32_t) __shfl((int) hb, (int) jl) == hb;
                        if (__ballot(bad) && lane == 0) order_bad = 1;
                    }
                    if (p < len && p >= own && !(MODE == 4 && p == 65535u)) {
                        const uint32_t q = sh_r[k][j * 1024 + tid];
                        uint32_t v;
                        if (MODE == 4) {
                            v = q == 0xffff ? 0 : p - q;
                            /* stream: a link reaching 32 KiB or more ends the
                             * walk exactly as the window limit does
                             * (getmatch2 :2655) */
                            if (stream && v >= JD_WSIZE) v = 0;
                        } else {
                            v = q;
                        }
                        dst[p] = (uint16_t) v;
                    }
                }
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < NPT; j++) { hq2[j] = hq1[j]; hq1[j] = hcur[j]; }
        __syncthreads();
    }
    if constexpr (SL) {
        k_chains_sl_tail(head, blk, bufend, len, dlen, b, bs, dst, so, force_serial || (n < 4 && len),
                         &hlast_sh);
        return;
    }
    if (order_bad) {
        /* never observed; exact whatever the LDS serialisation was */
        chains_serial<MODE>(head, blk, bufend, ws, len, own, dlen, dst, stream, inc3, b, dsz, pbase,
                            ov, nov);
        __syncthreads();
    } else if (MODE == 4 && hlast < HS && 65535u >= own) {
        /* position 65535, the last of a full 64 KiB range: its link is the
         * head of its bucket after everything before it was filed */
        const uint32_t q = head[hlast];
        uint32_t v = q == 0xffff ? 0 : 65535u - q;
        if (stream && v >= JD_WSIZE) v = 0;
        dst[65535] = (uint16_t) v;
    }
    if (MODE == 3 && dsg) {
        /* the doshort value the split parse's lists assume: literals < 16
         * set it (:2934), so guess it from the share of such bytes */
        for (int d = 32; d >= 1; d >>= 1) nlow += (uint32_t) __shfl_xor((int) nlow, d);
        if (lane == 0) atomicAdd(&nlow_sh, nlow);
        __syncthreads();
        /* lists with doshort 0 (bit 0) and/or 1 (bit 1): doshort 0 alone
         * where such bytes are rare (text), both elsewhere (binary data
         * flips doshort at many checks) */
        if (tid == 0) dsg[b] = nlow_sh * 64 < len ? 1u : 3u;
    }
}

/* stream mode: latest position (+1) of every hash-3 bucket inside each unit */
__global__ __launch_bounds__(1024) void k_s3last(const uint8_t* __restrict__ in, uint64_t n,
                                                 uint32_t bs, uint32_t* __restrict__ last3,
                                                 uint32_t dsz, const JdOverride* __restrict__ ov,
                                                 uint32_t nov)
{
    __shared__ uint32_t t[16384];
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    for (uint32_t i = tid; i < 16384; i += 1024) t[i] = 0;
    __syncthreads();
    const uint64_t ub = (uint64_t) b * bs;
    const uint32_t len = blk_len(n, bs, b);
    const uint64_t rest = n - ub;
    const uint32_t dlen = rest > 0xffffffffull ? 0xffffffffu : (uint32_t) rest;
    const uint8_t* blk = in + ub;
    for (uint32_t p = tid; p < len; p += 1024) {
        const uint64_t gp = ub + p;
        uint32_t h = 0;
        if (gp < dsz && gp + 4 > dsz) h = 16384;      /* as k_chains */
        else if (gp != dsz) h = ((head_be(blk, p, dlen, in + n) >> 8) * 0x1e35a7bdu) >> 18;
        h = ov_bucket<3>(ov, nov, gp, h);
        if (h < 16384) atomicMax(&t[h], (uint32_t) gp + 1u);
    }
    __syncthreads();
    for (uint32_t i = tid; i < 16384; i += 1024) last3[(uint64_t) b * 16384 + i] = t[i];
}

/* in place: last3[u][h] becomes the latest position before unit u, as the
 * uint16 the reference's shlist holds (0 = empty); before the launch's first
 * position the table is init3 (NULL: empty) */
__global__ __launch_bounds__(256) void k_s3scan(uint32_t* __restrict__ last3, uint32_t nunits,
                                                const uint32_t* __restrict__ init3)
{
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    if (h >= 16384) return;
    const uint32_t i0 = init3 ? init3[h] : 0u;
    uint32_t run = 0;
    for (uint32_t u = 0; u < nunits; u++) {
        uint32_t* c = last3 + (uint64_t) u * 16384 + h;
        const uint32_t v = *c;
        *c = run ? ((run - 1) & 0xffffu) : i0;
        run = v > run ? v : run;
    }
}

/* ------------------------------------------------------------------------ */
/* K2: match records.  One workgroup per 16 Ki-position quarter of a block;
 * LDS holds the window [lo, lo + 48.5 KiB) and the hash-4 chain links of
 * [lo, hi).  For position p it walks the chain like getmatch2 :2650-2674
 * with the running threshold starting at 2: the first candidate reaching the
 * maximum length is kept, the walk stops at the first length >= nice, and
 * the state after half the budget (the `length >= 3` halving, :2650) is
 * recorded too.  A caller threshold L0 >= 2 only decides whether that result
 * beats L0, so one walk serves every call the parser can make.
 * ------------------------------------------------------------------------ */
#define K2_SR   16384u
#define K2_WLO  32768u
#ifndef K2_HOPS
#define K2_HOPS 4
#endif
#define K2_WIN  (K2_WLO + K2_SR + 512u)
#define K2_PV   (K2_WLO + K2_SR)


/* 4 window bytes from byte offset i (two aligned reads: unaligned LDS dword
 * reads are correct on gfx950 but made k_match 2x slower) */
__device__ static inline uint32_t lds_word(const uint32_t* w32, uint32_t i)
{
    const uint32_t a = w32[i >> 2], c = w32[(i >> 2) + 1];
    return __builtin_amdgcn_alignbyte(c, a, i);     /* uses i[1:0] only */
}

__device__ static inline uint64_t lds_dword2(const uint32_t* w32, uint32_t i)
{
    uint64_t v;
    __builtin_memcpy(&v, (const uint8_t*) w32 + i, 8);
    return v;
}

/* ML16: matchlen 16 bytes per step (levels 8-9, whose long budgets meet
 * long matches in repetitive data: 256 MiB of the mixed corpus at level 9,
 * k_match 48.9 -> 44.2 ms); 8 bytes per step elsewhere (text at level 6:
 * 23.4 vs 24.1 ms with 16) */
template <bool ML16>
__global__ __launch_bounds__(1024) void k_match(const uint8_t* __restrict__ in,
                                                uint64_t n, uint32_t bs,
                                                const uint16_t* __restrict__ prev4,
                                                const uint16_t* __restrict__ prev3,
                                                uint64_t* __restrict__ rec,
                                                uint32_t chain, uint32_t nice,
                                                uint32_t minlen, int use3)
{
    /* the window at LDS offset 0 and the links behind it: a link address
     * is then 2 q plus an immediate offset, a window address needs no base */
    struct MatchShared {
        __attribute__((aligned(16))) uint8_t win[K2_WIN];
        __attribute__((aligned(16))) uint16_t pv[K2_PV];
        uint32_t qnext;                        /* next unclaimed position    */
        uint32_t n3map[K2_SR / 32];            /* positions needing pass 2   */
    };
    __shared__ MatchShared ms;
    uint8_t* const win = ms.win;
    uint16_t* const pv = ms.pv;
    uint32_t& qnext = ms.qnext;
    uint32_t* const n3map = ms.n3map;

    const uint32_t nsub = (bs + K2_SR - 1) / K2_SR;
    /* workgroups are dealt round-robin to the 8 XCDs (blockIdx mod 8), each
     * with its own L2: the quarters of one block, whose windows overlap by
     * 32 KiB of bytes and links, go to the same XCD (b = 8 * group + xcd).
     * Measured 23.90 -> 23.57 ms per GiB (profiles/r02_variants.log). */
    uint32_t b, k;
    if (nsub == 4 && gridDim.x % 32 == 0) {
        const uint32_t x = blockIdx.x & 7, sidx = blockIdx.x >> 3;
        k = sidx & 3;
        b = (sidx >> 2) * 8 + x;
    } else {
        b = blockIdx.x / nsub;
        k = blockIdx.x % nsub;
    }
    const uint32_t len = blk_len(n, bs, b);
    const uint32_t k0 = k * K2_SR;
    if (k0 >= len) return;
    const uint32_t hi = min(len, k0 + K2_SR);
    const uint32_t lo = k0 >= K2_WLO ? k0 - K2_WLO : 0;
    const uint64_t base = (uint64_t) b * bs;
    const uint8_t* blk = in + base;
    const uint32_t tid = threadIdx.x;

    /* stage the window (zero past the block end) and the chain links: every
     * thread issues all of its 16-byte loads before the first LDS write, so
     * the ~145 KiB arrive in one memory latency */
    {
        const uint32_t wn = min(len, lo + K2_WIN) - lo;  /* valid window bytes */
        const uint32_t pn = hi - lo;                      /* chain links       */
        constexpr uint32_t WV = (K2_WIN / 16 + 1023) / 1024;       /* 4 */
        constexpr uint32_t PVV = (K2_PV / 8 + 1023) / 1024;        /* 6 */
        uint4 wv[WV], pvv[PVV];
        const uint16_t* psrc = prev4 + base + lo;
#pragma unroll
        for (uint32_t j = 0; j < WV; j++) {
            const uint32_t i = tid + j * 1024, o = i * 16;
            wv[j] = make_uint4(0, 0, 0, 0);
            if (o + 16 <= wn) {
                JD_CHECK(blk + lo + o, 16, in + n);
                wv[j] = *(const uint4*) (blk + lo + o);
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < PVV; j++) {
            const uint32_t i = tid + j * 1024, o = i * 8;
            pvv[j] = make_uint4(0, 0, 0, 0);
            if (o + 8 <= pn) pvv[j] = *(const uint4*) (psrc + o);
        }
        uint4* w4 = (uint4*) win;
        uint4* p4v = (uint4*) pv;
        /* an empty link (0) becomes 0xFFFF: the walk then ends on the same
         * distance test as the window limit */
#pragma unroll
        for (uint32_t j = 0; j < PVV; j++) {
            uint32_t* w = (uint32_t*) &pvv[j];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t x = w[k];
                w[k] = x | ((x & 0xffffu) ? 0u : 0xffffu) | ((x >> 16) ? 0u : 0xffff0000u);
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < WV; j++) {
            const uint32_t i = tid + j * 1024, o = i * 16;
            if (i < K2_WIN / 16) {
                if (o < wn && o + 16 > wn) {
                    uint8_t t[16];
                    for (uint32_t k = 0; k < 16; k++) {
                        if (o + k < wn) JD_CHECK(blk + lo + o + k, 1, in + n);
                        t[k] = o + k < wn ? blk[lo + o + k] : 0;
                    }
                    wv[j] = *(uint4*) t;
                }
                w4[i] = wv[j];
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < PVV; j++) {
            const uint32_t i = tid + j * 1024, o = i * 8;
            if (o < pn) {
                if (o + 8 > pn) {
                    for (uint32_t k = o; k < pn; k++) pv[k] = psrc[k] ? psrc[k] : 0xffff;
                } else {
                    p4v[i] = pvv[j];
                }
            }
        }
    }
    __syncthreads();

    if (tid == 0) qnext = 1024;
    for (uint32_t i = tid; i < K2_SR / 32; i += 1024) n3map[i] = 0;
    __syncthreads();
    const uint32_t* w32 = (const uint32_t*) win;
    const uint32_t half = chain >> 1;
    (void) minlen;          /* lengths are stored raw; the parser applies it */
    uint64_t* rb = rec + base;

    /* pass 1: one chain hop per iteration for whichever position each lane is
     * on; a finished position stores its record and the lane moves on, so the
     * loop holds no global loads and diverges only inside matchlen.
     * The hop is kept to a handful of VALU ops (the kernel is VALU-issue
     * bound): empty links were staged as 0xFFFF so one distance test ends
     * the walk (chain end or p - q >= 32768, getmatch2 :2655-2658); the
     * budget counts down; the next link loads together with the candidate
     * byte; the p-side byte at cl is cached; and the half-budget snapshot
     * (l24/o24) is taken only when an improvement happens at or after hop
     * `half` -- the best over hops < half is exactly the value before the
     * first such improvement.  (A phase-batched variant that ran matchlen
     * and record writes for many paused lanes at once measured 30% slower:
     * its ballots and extra iterations cost more VALU than the divergence
     * saved.) */
    uint32_t p = k0 + tid, need3 = 0;
    bool live = p < hi;
    /* window-local (minus lo); qmin >= 0: a wrong link that points before
     * the window ends the walk (valid chains never do) */
    int32_t q = 0, qmin = 0;
    /* quick reject: an improving candidate matches bytes [cl-3, cl] (bytes
     * [0, 2] while cl = 2), so the 4 bytes ending at cl are compared; the
     * p side (pw at offset pt, mask pm) changes only with cl */
    uint32_t cl = 2, co = 0, l24 = 0, o24 = 0, left = chain, pw = 0, pt = 0, pm = 0xffffffu;
    bool have24 = false;
    if (live) {
        q = (int32_t) (p - lo) - (int32_t) pv[p - lo];
        qmin = max((int32_t) (p - lo) - (int32_t) (JD_WSIZE - 1), 0);
        pw = lds_word(w32, p - lo) & pm;
    }

    while (live) {
        /* up to K2_HOPS quick-rejected hops per iteration: the matchlen and
         * finish blocks below run once per iteration, so fewer iterations
         * means fewer executions of them with only a few lanes active */
        /* A hop that hits (quick reject passed) or ends the walk leaves q
         * and left unchanged, so the remaining hops recompute the same
         * outcome: the lane is frozen without any per-hop flags.  The loads
         * are issued for every lane; a negative q (the walk has ended) reads
         * an LDS address whose value is discarded (LDS reads cannot fault). */
        bool endw = false, hit = false;
        uint32_t dn = 0;
#pragma unroll
        for (int u = 0; u < K2_HOPS; u++) {
            endw = left == 0 || q < qmin;
            const uint32_t iq = (uint32_t) q;
            dn = pv[iq];
            hit = ((lds_word(w32, iq + pt) ^ pw) & pm) == 0;
            const bool step = !endw && !hit;
            left -= step ? 1u : 0u;
            q -= step ? (int32_t) dn : 0;
        }
        bool fin = endw;
        const bool pass = !endw && hit;
        if (pass) {
            {
                /* getmatchlength :1978, capped at 258 */
                uint32_t m = 0;
                const uint32_t ip = p - lo, iq = (uint32_t) q;
                if (ML16) {
                while (m < JD_MAXMATCH) {
                    uint4 xa, xb;
                    __builtin_memcpy(&xa, (const uint8_t*) w32 + ip + m, 16);
                    __builtin_memcpy(&xb, (const uint8_t*) w32 + iq + m, 16);
                    const uint64_t x0 = ((uint64_t) (xa.y ^ xb.y) << 32) | (xa.x ^ xb.x);
                    const uint64_t x1 = ((uint64_t) (xa.w ^ xb.w) << 32) | (xa.z ^ xb.z);
                    if (x0 | x1) {
                        m += x0 ? __builtin_ctzll(x0) >> 3 : 8 + (__builtin_ctzll(x1) >> 3);
                        break;
                    }
                    m += 16;
                }
                } else {
                while (m < JD_MAXMATCH) {
                    const uint64_t x = lds_dword2(w32, ip + m) ^ lds_dword2(w32, iq + m);
                    if (x) { m += __builtin_ctzll(x) >> 3; break; }
                    m += 8;
                }
                }
                m = min(m, JD_MAXMATCH);
                if (m > cl) {
                    if (!have24 && half && chain - left >= half) { l24 = cl; o24 = co; have24 = true; }
                    cl = m;
                    co = p - lo - (uint32_t) q;
                    pt = cl - 3;
                    pm = 0xffffffffu;
                    pw = lds_word(w32, p - lo + pt);
                    fin = cl >= nice;
                }
            }
            left--;
            q -= (int32_t) dn;
        }
        if (fin) {
            if (!have24) { l24 = cl; o24 = co; }
            /* raw lengths (2 = no candidate); the parser clamps them to the
             * block end (getmatch2 :2717-2719) */
            /* a position without a chain match of length 3 gets its whole
             * record in pass 2, with its 3-byte candidate: every record is
             * stored once, never patched */
            if (use3 && cl < 3)
                atomicOr(&n3map[(p - k0) >> 5], 1u << ((p - k0) & 31));
            else
                *(uint2*) (rb + p) = make_uint2(cl | (co << 9) | (l24 << 24), (l24 >> 8) | (o24 << 1));
            /* positions are claimed from a workgroup counter, so lanes with
             * cheap positions take more of them and the waves finish
             * together (records are independent of the order) */
            p = k0 + atomicAdd(&qnext, 1u);
            live = p < hi;
            if (live) {
                cl = 2; co = 0; left = chain; have24 = false;
                q = (int32_t) (p - lo) - (int32_t) pv[p - lo];
                qmin = max((int32_t) (p - lo) - (int32_t) (JD_WSIZE - 1), 0);
                pt = 0;
                pm = 0xffffffu;
                pw = lds_word(w32, p - lo) & pm;
            }
        }
    }

    /* pass 2: 3-byte candidates, getmatch2 :2676-2711 (only reachable when no
     * chain candidate reached length 3); all of a lane's loads are issued
     * together.  Distances > 8192 are always dropped by the far-3 rule
     * (deflator.c:2829), so they are not recorded. */
    __syncthreads();
#pragma unroll
    for (int jj = 0; jj < K2_SR / 1024; jj++) {
        const uint32_t o = tid + jj * 1024;
        if ((n3map[o >> 5] >> (o & 31)) & 1) need3 |= 1u << jj;
    }
    if (need3) {
        constexpr int NJ = K2_SR / 1024;
        uint32_t n3[NJ], n3b[NJ];
#pragma unroll
        for (int jj = 0; jj < NJ; jj++) {
            n3[jj] = 0;
            if ((need3 >> jj) & 1) n3[jj] = prev3[base + k0 + tid + jj * 1024];
        }
#pragma unroll
        for (int jj = 0; jj < NJ; jj++) {
            n3b[jj] = 0;
            const uint32_t pp = k0 + tid + jj * 1024;
            /* schain[next3 & 0x3fff] as of position pp: written by the
             * latest r <= pp congruent to next3 (in a stream piece, the
             * carried heads can name a position before the launch buffer:
             * its ring entry is not here, and no parsed position needs it) */
            const uint32_t back = (pp - n3[jj]) & 16383u;
            if (n3[jj] && back <= pp) n3b[jj] = prev3[base + pp - back];
        }
#pragma unroll
        for (int jj = 0; jj < NJ; jj++) {
            if (!((need3 >> jj) & 1)) continue;
            const uint32_t pp = k0 + tid + jj * 1024;
            const uint32_t i0 = pp - lo;
            const uint32_t x0 = lds_word(w32, i0) & 0xffffff;
            uint32_t s3 = 0;
            uint32_t noff = (pp - n3[jj]) & 0xffff;
            if (n3[jj] && noff <= JD_WSIZE && noff != 0) {
                if ((lds_word(w32, i0 - noff) & 0xffffff) == x0) {
                    s3 = noff;
                } else if (n3b[jj]) {
                    noff = (pp - n3b[jj]) & 0xffff;
                    if (noff <= JD_WSIZE && noff != 0 && (lds_word(w32, i0 - noff) & 0xffffff) == x0)
                        s3 = noff;
                }
            }
            /* cl = l24 = 2 (no chain candidate, so no improvement and no
             * half-budget snapshot), s3 in the top 16 bits and also in the
             * offset field, which no reader uses below length 3 */
            if (s3 > 8192) s3 = 0;
            *(uint2*) (rb + pp) = make_uint2(2u | (s3 << 9) | (2u << 24), s3 << 16);
        }
    }
}


/* ------------------------------------------------------------------------ */
/* K2 over slices (block mode, round 6).  The records of k_match, with each
 * position's chain read as the slice S[r-1], S[r-2], ... that k_chains<4,
 * false, true> wrote (the block's positions sorted by (bucket, position),
 * W[p] = r | n << 16, n = candidates within the window, at most `chain`).
 * No candidate depends on the one before it, so a lane holds up to 16
 * upcoming candidates in registers (two 8-entry chunks, 16-byte loads) and
 * tests K2S_K of them per iteration with independent LDS reads, where
 * k_match waited on a dependent link read for every hop.  LDS holds only the
 * window, so two workgroups share a CU.  The walk itself -- quick reject on
 * the 4 bytes ending at the best length, matchlen, the half-budget snapshot,
 * the nice stop, the pass-2 3-byte candidate -- is k_match's (getmatch2
 * :2650-2711), and so are the records.
 * ------------------------------------------------------------------------ */
#ifndef K2S_K
#define K2S_K 8
#endif
#ifndef K2S_NT
#define K2S_NT 1024
#endif

/* a chunk of 8 slice entries ascending in memory, the next candidate in the
 * top half of .w: dropping the f next candidates is a 128-bit shift left */
__device__ static inline void sl_drop(uint4& a, uint32_t f)
{
    const uint64_t x = ((uint64_t) a.y << 32) | a.x, y = ((uint64_t) a.w << 32) | a.z;
    const uint32_t s = 16u * f;
    uint64_t nx, ny;
    if (s >= 64) {
        ny = s >= 128 ? 0 : x << (s - 64);
        nx = 0;
    } else {
        ny = s ? (y << s) | (x >> (64 - s)) : y;
        nx = x << s;
    }
    a = make_uint4((uint32_t) nx, (uint32_t) (nx >> 32), (uint32_t) ny, (uint32_t) (ny >> 32));
}

/* candidate u (0 = next) of a chunk */
__device__ static inline uint32_t sl_cand(const uint4& a, int u)
{
    const uint32_t d = u < 2 ? a.w : u < 4 ? a.z : u < 6 ? a.y : a.x;
    return (u & 1) ? (d & 0xffffu) : (d >> 16);
}

__device__ static inline uint4 sl_load(const uint16_t* p)
{
    uint4 v;
    __builtin_memcpy(&v, p, 16);       /* 2-byte aligned: one dwordx4 load */
    return v;
}

#ifndef K2S_W
#define K2S_W 8                 /* min waves per SIMD: 2 workgroups per CU */
#endif

template <bool ML16, uint32_t NT>
__global__ __launch_bounds__(NT, K2S_W) void k_match_sl(const uint8_t* __restrict__ in,
                                                 uint64_t n, uint32_t bs,
                                                 const uint16_t* __restrict__ S,
                                                 const uint32_t* __restrict__ W,
                                                 const uint16_t* __restrict__ prev3,
                                                 uint64_t* __restrict__ rec,
                                                 uint32_t chain, uint32_t nice, int use3)
{
    struct MatchShared {
        __attribute__((aligned(16))) uint8_t win[K2_WIN];
        uint32_t qnext;
        uint32_t n3map[K2_SR / 32];
    };
    __shared__ MatchShared ms;
    uint8_t* const win = ms.win;
    uint32_t& qnext = ms.qnext;
    uint32_t* const n3map = ms.n3map;

    const uint32_t nsub = (bs + K2_SR - 1) / K2_SR;
    uint32_t b, k;
    if (nsub == 4 && gridDim.x % 32 == 0) {
        const uint32_t x = blockIdx.x & 7, sidx = blockIdx.x >> 3;
        k = sidx & 3;
        b = (sidx >> 2) * 8 + x;
    } else {
        b = blockIdx.x / nsub;
        k = blockIdx.x % nsub;
    }
    const uint32_t len = blk_len(n, bs, b);
    const uint32_t k0 = k * K2_SR;
    if (k0 >= len) return;
    const uint32_t hi = min(len, k0 + K2_SR);
    const uint32_t lo = k0 >= K2_WLO ? k0 - K2_WLO : 0;
    const uint64_t base = (uint64_t) b * bs;
    const uint8_t* blk = in + base;
    const uint16_t* sb = S + base;
    const uint32_t* wb = W + base;
    const uint32_t tid = threadIdx.x;

    {
        const uint32_t wn = min(len, lo + K2_WIN) - lo;
        constexpr uint32_t WV = (K2_WIN / 16 + NT - 1) / NT;
        uint4 wv[WV];
#pragma unroll
        for (uint32_t j = 0; j < WV; j++) {
            const uint32_t i = tid + j * NT, o = i * 16;
            wv[j] = make_uint4(0, 0, 0, 0);
            if (o + 16 <= wn) {
                JD_CHECK(blk + lo + o, 16, in + n);
                wv[j] = *(const uint4*) (blk + lo + o);
            }
        }
        uint4* w4 = (uint4*) win;
#pragma unroll
        for (uint32_t j = 0; j < WV; j++) {
            const uint32_t i = tid + j * NT, o = i * 16;
            if (i < K2_WIN / 16) {
                if (o < wn && o + 16 > wn) {
                    uint8_t t[16];
                    for (uint32_t kk = 0; kk < 16; kk++) {
                        if (o + kk < wn) JD_CHECK(blk + lo + o + kk, 1, in + n);
                        t[kk] = o + kk < wn ? blk[lo + o + kk] : 0;
                    }
                    wv[j] = *(uint4*) t;
                }
                w4[i] = wv[j];
            }
        }
    }
    if (tid == 0) qnext = 3 * NT;
    for (uint32_t i = tid; i < K2_SR / 32; i += NT) n3map[i] = 0;
    __syncthreads();
    const uint32_t* w32 = (const uint32_t*) win;
    const uint32_t half = chain >> 1;
    uint64_t* rb = rec + base;

    /* lane state: position p (window index ip), its candidates A (next 8) and
     * B (the 8 after), na valid in A, nxt = slice index above the chunk to
     * load next, hop = candidates taken, nav = candidates in all.  Two
     * positions are claimed ahead: pn, whose W word wn has landed and whose
     * first 16 candidates (An, Bn) are in flight, and pnn, whose W word wnn
     * is in flight -- so a lane that moves on never waits on a load issued
     * in the iteration before (the wave would wait with it). */
    uint32_t p = k0 + tid, pn = k0 + NT + tid, pnn = k0 + 2 * NT + tid, wn = 0, wnn = 0;
    bool live = p < hi;
    uint32_t ip = 0, qmin = 0, nav = 0, hop = 0, na = 0, nxt = 0, navn = 0, rn = 0;
    uint4 A = make_uint4(0, 0, 0, 0), Bc = make_uint4(0, 0, 0, 0);
    uint4 An = make_uint4(0, 0, 0, 0), Bn = make_uint4(0, 0, 0, 0);
    uint32_t cl = 2, co = 0, l24 = 0, o24 = 0, pw = 0, pt = 0, pm = 0xffffffu;
    bool have24 = false;
    /* issue the first two chunks of pn (W word wn) */
    auto ahead = [&](uint32_t q) {              /* q: the position wn belongs to */
        rn = wn & 0xffffu;
        navn = min(min(wn >> 16, rn), chain);       /* never below the block's slice */
        if (q < hi && navn) An = sl_load(sb + rn - 8);
        if (q < hi && navn > 8) Bn = sl_load(sb + rn - 16);
    };
    /* p = pn: take its chunks */
    auto begin = [&]() {
        nav = navn;
        A = An;
        Bc = Bn;
        nxt = rn - 16;
        ip = p - lo;
        qmin = max((int32_t) ip - (int32_t) (JD_WSIZE - 1), 0);
        hop = 0;
        na = min(nav, 8u);
        cl = 2; co = 0; have24 = false;
        pt = 0;
        pm = 0xffffffu;
        pw = lds_word(w32, ip) & pm;
    };
    if (live) {
        wn = wb[p];
        ahead(p);                       /* p's own chunks, waited for at once */
        begin();
        wn = pn < hi ? wb[pn] : 0u;
        wnn = pnn < hi ? wb[pnn] : 0u;
        ahead(pn);
    }

    while (live) {
        constexpr int K = K2S_K;
        const uint32_t cnt = min(na, (uint32_t) K);
        uint32_t mp = 0, mb = 0, qv[K];
#pragma unroll
        for (int u = 0; u < K; u++) {
            /* window index of candidate u; one outside [qmin, ip) ends the
             * walk (only wrong slices have one) */
            const uint32_t iq = sl_cand(A, u) - lo;
            qv[u] = iq;
            const bool inr = iq - qmin < ip - qmin;
            const bool hit = ((lds_word(w32, iq + pt) ^ pw) & pm) == 0;
            mp |= ((uint32_t) u < cnt && inr && hit) ? 1u << u : 0u;
            mb |= ((uint32_t) u < cnt && !inr) ? 1u << u : 0u;
        }
        bool fin = false;
        const uint32_t mm = mp | mb;
        if (!mm) {
            hop += cnt;
            na -= cnt;
            sl_drop(A, cnt);
        } else {
            const uint32_t f = __builtin_ctz(mm);
            if ((mb >> f) & 1) {
                fin = true;
            } else {
                hop += f;
                uint32_t iq = qv[0];
#pragma unroll
                for (int u = 1; u < K; u++) iq = (uint32_t) u == f ? qv[u] : iq;
                uint32_t m = 0;
                if (ML16) {
                    while (m < JD_MAXMATCH) {
                        uint4 xa, xb;
                        __builtin_memcpy(&xa, (const uint8_t*) w32 + ip + m, 16);
                        __builtin_memcpy(&xb, (const uint8_t*) w32 + iq + m, 16);
                        const uint64_t x0 = ((uint64_t) (xa.y ^ xb.y) << 32) | (xa.x ^ xb.x);
                        const uint64_t x1 = ((uint64_t) (xa.w ^ xb.w) << 32) | (xa.z ^ xb.z);
                        if (x0 | x1) {
                            m += x0 ? __builtin_ctzll(x0) >> 3 : 8 + (__builtin_ctzll(x1) >> 3);
                            break;
                        }
                        m += 16;
                    }
                } else {
                    while (m < JD_MAXMATCH) {
                        const uint64_t x = lds_dword2(w32, ip + m) ^ lds_dword2(w32, iq + m);
                        if (x) { m += __builtin_ctzll(x) >> 3; break; }
                        m += 8;
                    }
                }
                m = min(m, JD_MAXMATCH);
                if (m > cl) {
                    if (!have24 && half && hop >= half) { l24 = cl; o24 = co; have24 = true; }
                    cl = m;
                    co = ip - iq;
                    pt = cl - 3;
                    pm = 0xffffffffu;
                    pw = lds_word(w32, ip + pt);
                    fin = cl >= nice;
                }
                hop++;
                na -= f + 1;
                sl_drop(A, f + 1);
            }
        }
        fin = fin || hop >= nav;
        if (!fin && na == 0) {
            A = Bc;
            na = min(nav - hop, 8u);
            if (nav - hop > 8) Bc = sl_load(sb + nxt - 8);
            nxt -= 8;
        }
        if (fin) {
            if (!have24) { l24 = cl; o24 = co; }
            if (use3 && cl < 3)
                atomicOr(&n3map[(p - k0) >> 5], 1u << ((p - k0) & 31));
            else
                *(uint2*) (rb + p) = make_uint2(cl | (co << 9) | (l24 << 24), (l24 >> 8) | (o24 << 1));
            p = pn;
            live = p < hi;
            if (live) {
                begin();
                pn = pnn;
                wn = wnn;
                ahead(pn);
                pnn = k0 + atomicAdd(&qnext, 1u);
                if (pnn < hi) wnn = wb[pnn];
            }
        }
    }

    /* pass 2: 3-byte candidates, as k_match (groups of 4 positions per
     * lane, their loads issued together) */
    __syncthreads();
    constexpr int NJ = K2_SR / NT, G = 4;
    for (int j0 = 0; j0 < NJ; j0 += G) {
        uint32_t need3 = 0;
#pragma unroll
        for (int jj = 0; jj < G; jj++) {
            const uint32_t o = tid + (j0 + jj) * NT;
            if ((n3map[o >> 5] >> (o & 31)) & 1) need3 |= 1u << jj;
        }
        if (!need3) continue;
        uint32_t n3[G], n3b[G];
#pragma unroll
        for (int jj = 0; jj < G; jj++) {
            n3[jj] = 0;
            if ((need3 >> jj) & 1) n3[jj] = prev3[base + k0 + tid + (j0 + jj) * NT];
        }
#pragma unroll
        for (int jj = 0; jj < G; jj++) {
            n3b[jj] = 0;
            const uint32_t pp = k0 + tid + (j0 + jj) * NT;
            const uint32_t back = (pp - n3[jj]) & 16383u;
            if (n3[jj] && back <= pp) n3b[jj] = prev3[base + pp - back];
        }
#pragma unroll
        for (int jj = 0; jj < G; jj++) {
            if (!((need3 >> jj) & 1)) continue;
            const uint32_t pp = k0 + tid + (j0 + jj) * NT;
            const uint32_t i0 = pp - lo;
            const uint32_t x0 = lds_word(w32, i0) & 0xffffff;
            uint32_t s3 = 0;
            uint32_t noff = (pp - n3[jj]) & 0xffff;
            if (n3[jj] && noff <= JD_WSIZE && noff != 0) {
                if ((lds_word(w32, i0 - noff) & 0xffffff) == x0) {
                    s3 = noff;
                } else if (n3b[jj]) {
                    noff = (pp - n3b[jj]) & 0xffff;
                    if (noff <= JD_WSIZE && noff != 0 && (lds_word(w32, i0 - noff) & 0xffffff) == x0)
                        s3 = noff;
                }
            }
            if (s3 > 8192) s3 = 0;
            *(uint2*) (rb + pp) = make_uint2(2u | (s3 << 9) | (2u << 24), s3 << 16);
        }
    }
}


/* ------------------------------------------------------------------------ */
/* K3: the parser.  One lane per block; the lane runs compress2 :2826-2949
 * (levels 6-9) or compress1 :2472-2505 (levels 1-5) over the match records,
 * writes one uint32 token per literal/match and closes a deflate block on
 * the token-list-full rule (:2910) and the split heuristic (:2927-2948).
 * ------------------------------------------------------------------------ */
struct ParseArgs {
    const uint64_t* rec;
    const uint16_t* prev4;
    const uint8_t* in;
    uint64_t n;
    uint32_t bs, nblocks;
    uint32_t* tokens;
    uint32_t* dbinfo;      /* per block: [ndb, (tokend, slots) x JD_MAXDB] */
    uint32_t good, lzcap, nice, half;
    int lazy;
};

/* byte of the block, zero past its end (the zeroed window, deflator.c:499) */
__device__ static inline uint32_t zbyte(const uint8_t* src, uint32_t x, uint32_t len)
{
    return x < len ? src[x] : 0;
}

/* 4 bytes at block position x, zero past the block end */
__device__ static inline uint32_t zword(const uint8_t* src, uint32_t x, uint32_t len,
                                        const uint8_t* bufend)
{
    const uint8_t* a = src + (x & ~3u);
    if (x + 4 <= len && a + 8 <= bufend) {
        JD_CHECK(a, 8, bufend);
        return __builtin_amdgcn_alignbyte(*(const uint32_t*) (a + 4), *(const uint32_t*) a, x & 3);
    }
    uint32_t v = 0;
    for (uint32_t k = 0; k < 4; k++) v |= zbyte(src, x + k, len) << (8 * k);
    return v;
}

/* Single-window stream view (deflator.c:1818-1897): bytes past the end are
 * what the reference's window buffer holds there -- the bytes an earlier
 * generation of the window (before a slide) left at that window offset and
 * no later one overwrote (JdWinState), else zero (the buffer is cleared by
 * deflator_reset :499-503, and the guard past windowend is never written). */
struct SView {
    const uint8_t* in;
    const uint16_t* prev4;     /* stream-global hash-4 links                */
    uint64_t n;
    uint64_t vbase;            /* launch offset of window[0]                */
    const uint64_t* gb;        /* earlier generations, newest first         */
    const uint32_t* gh;
    uint32_t ngen;
};

__device__ static inline uint32_t sv_byte(const SView& v, uint64_t x)
{
    if (x < v.n) return v.in[x];
    const uint64_t o = x - v.vbase;
    for (uint32_t g = 0; g < v.ngen; g++)
        if (o < v.gh[g]) return v.in[v.gb[g] + o];
    return 0;
}

/* Held step whose threshold L0 = held length - 1 reaches `nice`
 * (possible once an accept adopted a long match): the reference walk
 * (getmatch2 :2655-2674, half budget since L0 >= 3) then stops at the FIRST
 * candidate longer than L0, which the per-position records do not capture.
 * Rare (about one per 64 KiB of text at level 6), so it is walked here from
 * the global chain links. */
/* Every link walk stops at a link longer than its position (d > q): a valid
 * chain never has one, and a wrong one must give a wrong but in-bounds result
 * (the parity tests catch it), never a read before the buffer
 * (tests/test_gpu.py test_bad_links_never_fault). */
__device__ static void held_long(const uint8_t* src, uint32_t len, const uint8_t* bufend,
                                 const uint16_t* prev4, uint32_t cur, uint32_t L0,
                                 uint32_t half, uint32_t* ml, uint32_t* mo)
{
    uint32_t q = cur, it = 0;
    *ml = 0;
    *mo = 0;
    for (;;) {
        const uint32_t d = prev4[q];
        if (it >= half || d == 0 || d > q) break;
        q -= d;
        if (cur - q >= JD_WSIZE) break;
        if (zbyte(src, q + L0, len) == zbyte(src, cur + L0, len)) {
            uint32_t m = 0;
            while (m < JD_MAXMATCH) {
                const uint32_t x = zword(src, cur + m, len, bufend) ^ zword(src, q + m, len, bufend);
                if (x) { m += __builtin_ctz(x) >> 3; break; }
                m += 4;
            }
            m = min(m, JD_MAXMATCH);
            if (m > L0) {
                *ml = min(m, len - cur);
                *mo = cur - q;
                return;
            }
        }
        it++;
    }
}

/* held_long over the stream view (stream mode): positions are stream-global,
 * lengths truncate at the stream end, bytes past it are the window's */
__device__ static void held_long_s(const SView& v, uint64_t cur, uint32_t L0, uint32_t half,
                                   uint32_t* ml, uint32_t* mo)
{
    uint32_t it = 0;
    uint64_t q = cur;
    *ml = 0;
    *mo = 0;
    for (;;) {
        const uint32_t d = v.prev4[q];
        if (it >= half || d == 0 || d > q) break;
        q -= d;
        if (cur - q >= JD_WSIZE) break;
        if (sv_byte(v, q + L0) == sv_byte(v, cur + L0)) {
            uint32_t m = 0;
            while (m < JD_MAXMATCH && sv_byte(v, cur + m) == sv_byte(v, q + m)) m++;
            if (m > L0) {
                const uint64_t rest = v.n - cur;
                *ml = rest < m ? (uint32_t) rest : m;
                *mo = (uint32_t) (cur - q);
                return;
            }
        }
        it++;
    }
}

/* jd_lsym without branches */
__device__ static inline uint32_t lsym_bf(uint32_t len)
{
    const uint32_t x = len - 3;
    const uint32_t e = 29 - __builtin_clz(x | 4);
    const uint32_t big = 4 * e + 4 + ((x >> e) & 3);
    return len == 258 ? 28 : x < 8 ? x : big;
}

#define DBSTRIDE (1 + 2 * JD_MAXDB)

/* Per-lane LDS ring of the block's match records and bytes.  Each step
 * reads the record of the next position and of the jump target; from global
 * memory the step waits for the slowest of 64 lanes' gathers every time.
 * The ring is filled in 16-position chunks, two per batch, issued PR_K steps
 * before they are written to LDS, so the load latency overlaps the steps;
 * a position past the ring (a long jump) is read from global memory in a
 * rare wave-uniform branch. */
#define PR_W    256u                    /* positions per lane ring           */
#define PR_C    16u                     /* positions per chunk               */
#define PR_K    4u                      /* steps between batches             */
#define PR_RS   (PR_W * 8u + 16u)       /* rec ring row bytes (padded)       */
#define PR_SS   (PR_W + 16u)            /* byte ring row bytes (padded)      */
#define PR_VMCNT0 0x0f70                /* s_waitcnt vmcnt(0), gfx9 encoding  */

typedef uint32_t pr_v4 __attribute__((ext_vector_type(4)));
struct PrStage { pr_v4 a, b, c, d, e, f, g, h, s; };

struct ParseShared {
    uint8_t rr[64 * PR_RS];
    uint8_t sr[64 * PR_SS];
    uint32_t hist[32 * 64];             /* curr | prv << 16 per bucket       */
};

__global__ __launch_bounds__(64) void k_parse(ParseArgs a)
{
    __shared__ ParseShared sh;
    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x * 64 + lane;
    const bool on = b < a.nblocks;

    const uint32_t len = on ? blk_len(a.n, a.bs, b) : 0;
    const uint64_t base = (uint64_t) (on ? b : 0) * a.bs;
    const uint64_t* rec = a.rec + base;
    const uint16_t* prev4 = a.prev4 + base;
    const uint8_t* src = a.in + base;
    const uint8_t* bufend = a.in + a.n;
    uint32_t* tok = a.tokens + base;
    uint32_t* dbi = a.dbinfo + (uint64_t) (on ? b : 0) * DBSTRIDE;
    uint8_t* rr = sh.rr + lane * PR_RS;
    uint8_t* sr = sh.sr + lane * PR_SS;
    uint32_t* hist = sh.hist;

    for (int j = 0; j < 32; j++) hist[j * 64 + lane] = 0;
    uint32_t obscount = 0, newcount = 0, obstotal = 0;
    uint32_t cur = 0, nt = 0, slots = 0, ndb = 0;
    uint32_t hm = 0, hl = 0, ho = 0, ds = 0, lastc = 0;

#define RESETOBS() do { for (int j_ = 0; j_ < 32; j_++) hist[j_ * 64 + lane] = 0; obscount = newcount = obstotal = 0; } while (0)
#define CLOSEDB() do { if (ndb < JD_MAXDB) { dbi[1 + 2 * ndb] = nt; dbi[2 + 2 * ndb] = slots; } ndb++; slots = 0; } while (0)

    if (a.lazy) {
        /* ring: positions [.., rdy) are in LDS (those >= cur valid); np
         * chunks in flight in st0/st1 for [rdy, rdy + 16 np) */
        uint32_t rdy = 0, np = 0;
        PrStage st0, st1;
#define PR_LD(st_, q_)                                                                 \
        do {                                                                           \
            const pr_v4* g_ = (const pr_v4*) (rec + (q_));                             \
            st_.a = g_[0]; st_.b = g_[1]; st_.c = g_[2]; st_.d = g_[3];                \
            st_.e = g_[4]; st_.f = g_[5]; st_.g = g_[6]; st_.h = g_[7];                \
            st_.s = *(const pr_v4*) (src + (q_));                                      \
        } while (0)
#define PR_ST(st_, q_)                                                                 \
        do {                                                                           \
            const uint32_t w_ = (q_) & (PR_W - 1);                                     \
            pr_v4* d_ = (pr_v4*) (rr + w_ * 8);                                        \
            d_[0] = st_.a; d_[1] = st_.b; d_[2] = st_.c; d_[3] = st_.d;                \
            d_[4] = st_.e; d_[5] = st_.f; d_[6] = st_.g; d_[7] = st_.h;                \
            *(pr_v4*) (sr + w_) = st_.s;                                               \
        } while (0)
#define PR_ISSUE()                                                                     \
        do {                                                                           \
            np = 0;                                                                    \
            if (rdy + PR_C <= len && rdy + PR_C <= cur + PR_W) {                       \
                PR_LD(st0, rdy);                                                       \
                np = 1;                                                                \
                if (rdy + 2 * PR_C <= len && rdy + 2 * PR_C <= cur + PR_W) {           \
                    PR_LD(st1, rdy + PR_C);                                            \
                    np = 2;                                                            \
                }                                                                      \
            }                                                                          \
        } while (0)
#define PR_LAND()                                                                      \
        do {                                                                           \
            if (np >= 1) PR_ST(st0, rdy);                                              \
            if (np >= 2) PR_ST(st1, rdy + PR_C);                                       \
            rdy += np * PR_C;                                                          \
            if (rdy < (cur & ~(PR_C - 1))) rdy = cur & ~(PR_C - 1);                    \
        } while (0)
#define PR_RING(p_, r_, c_)                                                            \
        do {                                                                           \
            const uint32_t q_ = (p_) & (PR_W - 1);                                     \
            r_ = *(const uint64_t*) (rr + q_ * 8);                                     \
            c_ = sr[q_];                                                               \
        } while (0)
#define PR_MISS(p_, r_, c_)                                                            \
        do {                                                                           \
            if ((p_) >= rdy) {                                                         \
                r_ = rec[p_];                                                          \
                c_ = src[p_];                                                          \
            }                                                                          \
        } while (0)
        /* prime half the ring synchronously */
        for (uint32_t k = 0; k < PR_W / 2 / (2 * PR_C); k++) {
            PR_ISSUE();
            PR_LAND();
        }
        PR_ISSUE();
        uint32_t step = 0;
        uint64_t r = 0;
        uint32_t c = 0;
        if (len) {
            PR_RING(0u, r, c);
            PR_MISS(0u, r, c);
        }

        /* The next position is always cur + 1 or a target known from the
         * record before the step is decided (cur + l48 when a match reaches
         * `good`, cur + hl - 1 when the held match is emitted), so both
         * candidates' record and byte are read at the top of the step. */
        while (__ballot(cur < len)) {
            if (++step == PR_K) {
                step = 0;
                PR_LAND();
                PR_ISSUE();
            }
            if (cur < len) {
                /* records hold raw lengths; truncate to the block end here */
                const uint32_t rem = len - cur;
                const uint32_t raw48 = (uint32_t) r & 511;
                const uint32_t l48 = min(raw48, rem), o48 = (uint32_t) (r >> 9) & 0x7fff;
                const uint32_t n1 = cur + 1;
                /* selects, not branches (__builtin_unpredictable and the
                 * masks keep LLVM from turning them into divergent code) */
                const uint32_t nf = __builtin_unpredictable(l48 >= a.good) ? cur + l48 : n1;
                const uint32_t n2 = nf + ((cur + hl - 1 - nf) & (0u - hm));      /* hm ? .. : nf */
                /* a candidate at or past the block end is never stepped on */
                const uint32_t n1c = min(n1, len - 1), n2c = min(n2, len - 1);
                uint64_t r1, r2;
                uint32_t c1, c2;
                PR_RING(n1c, r1, c1);
                PR_RING(n2c, r2, c2);
                if (__ballot(n2c >= rdy)) {            /* n1c <= n2c */
                    PR_MISS(n1c, r1, c1);
                    PR_MISS(n2c, r2, c2);
                    /* wait here: a miss load left in flight would make every
                     * later ring read wait for the batch in flight */
                    __builtin_amdgcn_s_waitcnt(PR_VMCNT0);
                }
                /* one step of compress2 :2826-2906: the fresh step
                 * (getmatch2(2, shrt), far-3 rule, good) and the held step
                 * (getmatch2(prev-1, 0), accept rule) are both evaluated and
                 * one of their outcomes is kept */
                const bool H = hm != 0;
                const uint32_t s3 = (uint32_t) (r >> 48);
                const bool use3 = raw48 < 3 && ds && s3 && rem >= 3;
                uint32_t fml = use3 ? 3 : l48;
                const uint32_t fmo = use3 ? s3 : o48;
                fml = (fml == 3 && fmo > 8192) ? 2 : fml;
                const uint32_t l24 = min((uint32_t) (r >> 24) & 511, rem), o24 = (uint32_t) (r >> 33) & 0x7fff;
                uint32_t hml = hl >= 4 ? l24 : l48, hmo = hl >= 4 ? o24 : o48;
                if (__ballot(H && hl - 1 >= a.nice)) {
                    if (H && hl - 1 >= a.nice) held_long(src, len, bufend, prev4, cur, hl - 1, a.half, &hml, &hmo);
                }
                const int dl = (int) hml - (int) hl;
                const bool acc = __builtin_unpredictable(
                    H & (hml >= hl) & ((dl > 4) | ((dl * 4 + jd_ilog2(ho | 1) - jd_ilog2(hmo | 1)) >= 2)));
                const bool fm = !H & (fml >= 3);
                const bool emit_fresh = fm & (fml >= a.good);
                const bool hold = fm & (fml < a.good);
                const bool emit_held = H & !acc;
                const bool emit_match = __builtin_unpredictable(emit_fresh | emit_held);
                const bool emit_lit = (!H & (fml < 3)) | acc;
                const uint32_t mlen = H ? hl : fml, moff = H ? ho : fmo;
                const uint32_t lit = H ? lastc : c;
                /* emission without a branch: the token is stored at tok[nt]
                 * on every step and kept only when nt advances (a step that
                 * emits nothing is a hold, so nt < cur < len there) */
                const uint32_t em = (emit_match || emit_lit) ? 1u : 0u;
                tok[nt] = emit_match ? jd_tok_match(mlen, moff) : lit;
                nt += em;
                slots += emit_match ? 3u : em;
                const uint32_t mb = 16 + (lsym_bf(mlen) >> 1), lb = lit >> 4;
                const uint32_t bk = lb ^ ((mb ^ lb) & (0u - (uint32_t) emit_match));
                atomicAdd(&hist[bk * 64 + lane], em);
                newcount += em;
                obstotal += emit_match ? mlen : em;
                const uint32_t adv = emit_fresh ? fml : emit_held ? hl - 1 : 1;
                hm = (hold || acc) ? 1 : 0;
                hl = hold ? fml : acc ? hml : hl;
                ho = hold ? fmo : acc ? hmo : ho;
                cur += adv;
                lastc = c;
                r = cur == n1 ? r1 : r2;
                c = cur == n1 ? c1 : c2;
            }
            if (!__ballot(slots + 4 > a.lzcap || (newcount >= 512 && obstotal >= 4096))) continue;
            if (slots + 4 > a.lzcap) {
                CLOSEDB();
                RESETOBS();
            } else if (newcount >= 512 && obstotal >= 4096) {
                ds = (hist[0 * 64 + lane] & 0xffff) >= 16;
                /* shouldsplit :2557-2596 */
                bool split = false;
                if (obscount > 0) {
                    uint32_t delta = 0;
                    for (int j = 0; j < 32; j++) {
                        const uint32_t h = hist[j * 64 + lane];
                        const uint32_t x = h >> 16, y = h & 0xffff;
                        delta += x > y ? x - y : y - x;
                    }
                    split = delta >= 320 && obstotal >= 7168;
                }
                if (split) {
                    RESETOBS();
                    CLOSEDB();
                } else {
                    for (int j = 0; j < 32; j++) {
                        const uint32_t h = hist[j * 64 + lane];
                        hist[j * 64 + lane] = (((h >> 16) >> 1) + ((h & 0xffff) >> 1)) << 16;
                    }
                    obscount += newcount;
                    newcount = 0;
                }
            }
        }
#undef PR_LD
#undef PR_ST
#undef PR_ISSUE
#undef PR_LAND
#undef PR_RING
#undef PR_MISS
        if (!on) return;
    } else {
        if (!on) return;
        /* greedy parser, compress1 :2472-2505: a match needs length > 3 */
        while (cur < len) {
            const uint64_t r = rec[cur];
            const uint32_t l = min((uint32_t) r & 511, len - cur), o = (uint32_t) (r >> 9) & 0x7fff;
            if (l > 3) {
                tok[nt++] = jd_tok_match(l, o);
                slots += 3;
                cur += l - 1;
            } else {
                tok[nt++] = src[cur];
                slots += 1;
            }
            cur++;
            if (slots + 4 > a.lzcap) CLOSEDB();
        }
    }
    if (slots) CLOSEDB();
    dbi[0] = ndb;
#undef RESETOBS
#undef CLOSEDB
}

/* ------------------------------------------------------------------------ */
/* K3, split form (levels 6-9).  The serial lazy parse above is a chain of
 * ~30k dependent steps per block: one lane per block leaves 3 of 4 SIMDs
 * idle and every step waits on its own instruction latency.  Here:
 *   k_pspec   one lane per (block, segment): the lazy step walked from the
 *             segment start with nothing held and doshort = 0, past the
 *             segment end by a margin; every token goes to the segment's
 *             list with its start and whether the walk held nothing there.
 *             A lazy parse re-converges: two walks that reach the same
 *             position with nothing held continue identically.
 *   k_psync   one lane per segment boundary: the first token start past the
 *             boundary at which both neighbouring walks held nothing.
 *   k_pfinal  one lane per block: the exact parse.  It reads tokens from
 *             the lists (following sync points) and runs the block-split
 *             observer (:2910-2948) on them; where the lists cannot be used
 *             -- doshort became 1 (it changes which 3-byte matches count,
 *             :2826-2831), or a list ended without meeting the next -- it
 *             runs the lazy step itself until it stands with nothing held,
 *             doshort 0, at a position some list holds.
 * The token stream and block boundaries are those of k_parse.
 * ------------------------------------------------------------------------ */
struct PCtx {
    const uint64_t* rec;
    const uint16_t* prev4;
    const uint8_t* src;
    const uint8_t* bufend;
    uint32_t len, good, nice, half;
    uint32_t tlen;             /* lengths truncate here (block, or stream end) */
    int stream;
    int greedy;                /* levels 1-5: compress1 :2472-2505           */
    uint64_t gbase;            /* stream: block start in the stream          */
    SView v;
};

/* lazy-step state: position, held match, byte before, whether the held match
 * was taken at a step that held nothing (for the entry flags), whether it is
 * a 3-byte-chain match (doshort, :2826-2831), and the record and byte at cur */
struct PSt {
    uint32_t cur, hm, hl, ho, lastc, hfresh, h3;
    uint64_t r;
    uint32_t c;
};

/* list entry: x = token (a literal from an accept also carries the newly held
 * match: byte | hl << 8 | ho << 17), y = start | flags */
#define PE_H0    (1u << 16)     /* nothing was held at the start position   */
#define PE_ACC   (1u << 17)     /* literal emitted by an accept             */
#define PE_MATCH (1u << 18)
#define PE_D1    (1u << 19)     /* the step at the start position was fresh
                                   with a 3-byte-chain candidate, so doshort
                                   decides it (:2826-2831): walked with
                                   doshort 0 it emitted this literal, with
                                   doshort 1 it held the 3-byte match that
                                   this entry emits or replaces            */
#define PE_HS    (1u << 20)     /* a held step emitted this entry (its start
                                   is the step position - 1); stream mode
                                   tracks the window slides by it          */
#define PS_NONE  0xffffffffu

__device__ static inline void ps_load(const PCtx& x, uint32_t p, uint64_t& r, uint32_t& c)
{
    r = p < x.tlen ? x.rec[p] : 0;
    c = p < x.tlen ? (uint32_t) x.src[p] : 0;
}

/* the two positions a step can move to: cur + 1, or the jump target */
__device__ static inline void ps_targets(const PCtx& x, const PSt& s, uint32_t& n1, uint32_t& n2)
{
    const uint32_t l48 = min((uint32_t) s.r & 511, x.tlen - s.cur);
    n1 = s.cur + 1;
    const uint32_t nf = l48 >= x.good ? s.cur + l48 : n1;
    n2 = s.hm ? s.cur + s.hl - 1 : nf;
}

/* one step of compress2 :2826-2906 (the same selects as k_parse), given the
 * records and bytes at both targets; returns whether a token was emitted,
 * its list entry in ex/ey */
template <bool ST>
__device__ static inline bool ps_decide(const PCtx& x, PSt& s, uint32_t ds, uint32_t n1,
                                        uint64_t r1, uint32_t c1, uint64_t r2, uint32_t c2,
                                        uint32_t& ex, uint32_t& ey)
{
    const uint32_t cur = s.cur, rem = x.tlen - cur;
    const uint64_t r = s.r;
    if (ST && x.greedy) {
        /* compress1 :2472-2505: a match needs length > MINMATCH; x.good is 4
         * so ps_targets jumps over exactly these matches */
        const uint32_t l = min((uint32_t) r & 511, rem), o = (uint32_t) (r >> 9) & 0x7fff;
        const bool mt = l > 3;
        ex = mt ? jd_tok_match(l, o) : s.c;
        ey = cur | PE_H0 | (mt ? PE_MATCH : 0u);
        s.cur = cur + (mt ? l : 1u);
        s.lastc = s.c;
        s.r = s.cur == n1 ? r1 : r2;
        s.c = s.cur == n1 ? c1 : c2;
        return true;
    }
    const uint32_t raw48 = (uint32_t) r & 511;
    const uint32_t l48 = min(raw48, rem), o48 = (uint32_t) (r >> 9) & 0x7fff;
    const bool H = s.hm != 0;
    const uint32_t s3 = (uint32_t) (r >> 48);
    const bool c3 = raw48 < 3 && s3 && rem >= 3;       /* doshort decides   */
    const bool use3 = c3 && ds;
    uint32_t fml = use3 ? 3 : l48;
    const uint32_t fmo = use3 ? s3 : o48;
    fml = (fml == 3 && fmo > 8192) ? 2 : fml;
    const uint32_t l24 = min((uint32_t) (r >> 24) & 511, rem), o24 = (uint32_t) (r >> 33) & 0x7fff;
    uint32_t hml = s.hl >= 4 ? l24 : l48, hmo = s.hl >= 4 ? o24 : o48;
    if (H && s.hl - 1 >= x.nice) {
        if (ST && x.stream) held_long_s(x.v, x.gbase + cur, s.hl - 1, x.half, &hml, &hmo);
        else held_long(x.src, x.len, x.bufend, x.prev4, cur, s.hl - 1, x.half, &hml, &hmo);
    }
    const int dl = (int) hml - (int) s.hl;
    const bool acc = H && hml >= s.hl &&
                     (dl > 4 || (dl * 4 + jd_ilog2(s.ho | 1) - jd_ilog2(hmo | 1)) >= 2);
    const bool fm = !H && fml >= 3;
    const bool emit_fresh = fm && fml >= x.good;
    const bool hold = fm && fml < x.good;
    const bool emit_held = H && !acc;
    const bool emit_match = emit_fresh || emit_held;
    const bool emit_lit = (!H && fml < 3) || acc;
    const uint32_t mlen = H ? s.hl : fml, moff = H ? s.ho : fmo;
    const uint32_t lit = H ? s.lastc : s.c;
    ex = emit_match ? jd_tok_match(mlen, moff) : (lit | (acc ? (hml << 8) | (hmo << 17) : 0u));
    const bool d1 = H ? s.h3 != 0 : c3;
    /* the entry's start: a held step at a stream block's first position
     * (cur 0, the join carrying the state across blocks) emits for position
     * -1 of the block; only the 16 start bits may take it */
    ey = ((H ? cur - 1 : cur) & 0xffffu) | ((!H || s.hfresh) ? PE_H0 : 0u) | (acc ? PE_ACC : 0u) |
         (emit_match ? PE_MATCH : 0u) | (d1 ? PE_D1 : 0u) | (H ? PE_HS : 0u);
    const uint32_t adv = emit_fresh ? fml : emit_held ? s.hl - 1 : 1;
    s.hfresh = hold ? 1u : acc ? 0u : s.hfresh;
    s.h3 = hold ? (use3 ? 1u : 0u) : acc ? 0u : s.h3;
    s.hm = (hold || acc) ? 1 : 0;
    s.hl = hold ? fml : acc ? hml : s.hl;
    s.ho = hold ? fmo : acc ? hmo : s.ho;
    s.cur = cur + adv;
    s.lastc = s.c;
    s.r = s.cur == n1 ? r1 : r2;
    s.c = s.cur == n1 ? c1 : c2;
    return emit_match || emit_lit;
}

/* one step with its records read from global memory */
template <bool ST>
__device__ static inline bool ps_step(const PCtx& x, PSt& s, uint32_t ds, uint32_t& ex, uint32_t& ey)
{
    uint32_t n1, n2;
    ps_targets(x, s, n1, n2);
    uint64_t r1, r2;
    uint32_t c1, c2;
    ps_load(x, n1, r1, c1);
    ps_load(x, n2, r2, c2);
    return ps_decide<ST>(x, s, ds, n1, r1, c1, r2, c2, ex, ey);
}

/* the walk's margin past its segment: below half a segment, so a sync
 * point always lies inside the next segment's first half */
__host__ __device__ static inline uint32_t ps_margin(uint32_t seg)
{
    return seg / 2 < JD_PMARGIN ? seg / 2 : JD_PMARGIN;
}

struct PSplitArgs {
    const uint64_t* rec;
    const uint16_t* prev4;
    const uint8_t* in;
    uint64_t n;
    uint32_t bs, nblocks;
    uint32_t* tokens;
    uint32_t* dbinfo;
    uint32_t good, lzcap, nice, half;
    uint64_t* plist;
    uint32_t* pcount;
    uint32_t* psync;
    const uint32_t* dsg;    /* per block: the doshort value the lists assume */
    const uint32_t* perm;   /* block mode: k_pspec's block order (k_porder), or NULL */
    uint32_t pcap;
    /* stream mode (single-window stream cut into bs-byte blocks) */
    int stream;
    const uint16_t* prev3;  /* stream: hash-3 links (tail records)         */
    uint32_t* sdb;          /* stream: [ndb, (token end, slots) ...]       */
    uint32_t wend;          /* stream: window size of the level            */
    uint32_t chain;         /* stream: chain budget (tail records)         */
    int greedy;             /* levels 1-5 (stream): compress1, no observer */
    uint32_t pstart;        /* stream: parse start (the history's end)     */
    const uint64_t* cend;   /* stream: ends of the reference's calls       */
    uint32_t ncall;
    uint32_t tailchk;       /* stream: bytes past the end may be non-zero  */
    JdWinState w0;          /* stream: the window at pstart                */
    JdWinState* wout;       /* stream: the window at the end               */
};

__device__ static inline PCtx ps_ctx(const PSplitArgs& a, uint32_t b, uint32_t len)
{
    const uint64_t base = (uint64_t) b * a.bs;
    PCtx x;
    x.rec = a.rec + base;
    x.prev4 = a.prev4 + base;
    x.src = a.in + base;
    x.bufend = a.in + a.n;
    x.len = len;
    x.good = a.good;
    x.nice = a.nice;
    x.half = a.half;
    x.stream = a.stream;
    x.greedy = a.greedy;
    x.gbase = base;
    const uint64_t rest = a.n - base;
    x.tlen = a.stream ? (rest > 0xffffffffull ? 0xffffffffu : (uint32_t) rest) : len;
    x.v.in = a.in;
    x.v.prev4 = a.prev4;
    x.v.n = a.n;
    x.v.vbase = 0;
    x.v.gb = nullptr;
    x.v.gh = nullptr;
    x.v.ngen = 0;
    return x;
}

/* k_pspec: per-lane LDS ring of the segment's records and bytes (as in
 * k_parse, smaller: four waves share a CU), filled 16 positions per chunk,
 * two chunks issued every SP_K steps; a target past the ring is read from
 * global memory in a wave-uniform branch */
#ifndef SP_W
#define SP_W    64u
#endif
#define SP_C    16u
#ifndef SP_K
#define SP_K    4u
#endif
#define SP_RS   (SP_W * 8u + 16u)
#define SP_SS   (SP_W + 16u)

/* ST: stream mode (compiled out of the block-mode instantiation) */
template <bool ST>
__global__ __launch_bounds__(64) void k_pspec(PSplitArgs a)
{
    __shared__ uint8_t srr[64 * SP_RS];
    __shared__ uint8_t ssr[64 * SP_SS];
    const uint32_t lane = threadIdx.x;
    /* lane: set v (the doshort its walk assumes), block b, segment k; the
     * blocks are taken in k_porder's order (similar walks share a wave), the
     * list is (v, b, k)'s own slot g */
    const uint32_t NL = a.nblocks * JD_PSEG;
    const uint32_t gl = blockIdx.x * 64 + lane;
    const uint32_t v = gl / NL, ib = (gl % NL) / JD_PSEG, k = gl % JD_PSEG;
    const uint32_t b = a.perm ? a.perm[ib] : ib;
    const uint32_t g = v * NL + b * JD_PSEG + k;
    const bool on = v < 2 && ((a.dsg[b] >> v) & 1);
    const uint32_t len = on ? blk_len(a.n, a.bs, b) : 0;
    const uint32_t seg = a.bs / JD_PSEG, s0 = k * seg;
    const uint32_t lim = (!on || s0 >= len) ? 0 : k == JD_PSEG - 1 ? len : min(len, s0 + seg + ps_margin(seg));
    const PCtx x = ps_ctx(a, on ? b : 0, len);
    const uint32_t tlen = on ? x.tlen : 0;
    const uint32_t ds = v;
    const uint64_t* rec = x.rec;
    const uint8_t* src = x.src;
    uint8_t* rr = srr + lane * SP_RS;
    uint8_t* sr = ssr + lane * SP_SS;
    uint2* out = (uint2*) (a.plist + (uint64_t) (on ? g : 0) * a.pcap);
    uint32_t ne = 0;

    PSt s;
    s.cur = lim ? s0 : 0; s.hm = 0; s.hl = 0; s.ho = 0; s.lastc = 0; s.hfresh = 0; s.h3 = 0;
    s.r = 0; s.c = 0;
    /* the ring holds positions [vlo, rdy) in slots p mod SP_W; np chunks
     * from rdy on are in flight in st0/st1 */
    uint32_t rdy = s.cur & ~(SP_C - 1), vlo = rdy, np = 0;
    PrStage st0, st1;
#define SP_LD(st_, q_)                                                                 \
    do {                                                                               \
        const pr_v4* g_ = (const pr_v4*) (rec + (q_));                                 \
        st_.a = g_[0]; st_.b = g_[1]; st_.c = g_[2]; st_.d = g_[3];                    \
        st_.e = g_[4]; st_.f = g_[5]; st_.g = g_[6]; st_.h = g_[7];                    \
        st_.s = *(const pr_v4*) (src + (q_));                                          \
    } while (0)
#define SP_ST(st_, q_)                                                                 \
    do {                                                                               \
        const uint32_t w_ = (q_) & (SP_W - 1);                                         \
        pr_v4* d_ = (pr_v4*) (rr + w_ * 8);                                            \
        d_[0] = st_.a; d_[1] = st_.b; d_[2] = st_.c; d_[3] = st_.d;                    \
        d_[4] = st_.e; d_[5] = st_.f; d_[6] = st_.g; d_[7] = st_.h;                    \
        *(pr_v4*) (sr + w_) = st_.s;                                                   \
    } while (0)
#define SP_ISSUE()                                                                     \
    do {                                                                               \
        np = 0;                                                                        \
        if (rdy + SP_C <= tlen && rdy + SP_C <= s.cur + SP_W) {                        \
            SP_LD(st0, rdy);                                                           \
            np = 1;                                                                    \
            if (rdy + 2 * SP_C <= tlen && rdy + 2 * SP_C <= s.cur + SP_W) {            \
                SP_LD(st1, rdy + SP_C);                                                \
                np = 2;                                                                \
            }                                                                          \
        }                                                                              \
    } while (0)
#define SP_LAND()                                                                      \
    do {                                                                               \
        if (np >= 1) SP_ST(st0, rdy);                                                  \
        if (np >= 2) SP_ST(st1, rdy + SP_C);                                           \
        rdy += np * SP_C;                                                              \
        np = 0;                                                                        \
        vlo = max(vlo, rdy - min(rdy, SP_W));                                          \
        const uint32_t cb_ = s.cur & ~(SP_C - 1);                                      \
        if (rdy < cb_ || cb_ < vlo) rdy = vlo = cb_;                                   \
    } while (0)
#define SP_RING(p_, r_, c_)                                                            \
    do {                                                                               \
        const uint32_t q_ = (p_) & (SP_W - 1);                                         \
        r_ = *(const uint64_t*) (rr + q_ * 8);                                         \
        c_ = sr[q_];                                                                   \
    } while (0)
#define SP_MISS(p_, r_, c_)                                                            \
    do {                                                                               \
        if ((p_) >= rdy || (p_) < vlo) {                                               \
            r_ = rec[p_];                                                              \
            c_ = src[p_];                                                              \
        }                                                                              \
    } while (0)
    for (uint32_t j = 0; j < SP_W / 2 / (2 * SP_C); j++) {
        SP_ISSUE();
        SP_LAND();
    }
    SP_ISSUE();
    if (lim) {
        SP_RING(s.cur, s.r, s.c);
        SP_MISS(s.cur, s.r, s.c);
    }
    uint32_t step = 0;
    while (__ballot(s.cur < lim)) {
        if (++step == SP_K) {
            step = 0;
            SP_LAND();
            SP_ISSUE();
        }
        if (s.cur < lim) {
            uint32_t n1, n2;
            ps_targets(x, s, n1, n2);
            /* a target at or past the block (stream) end is never stepped on */
            const uint32_t n1c = min(n1, tlen - 1), n2c = min(n2, tlen - 1);
            uint64_t r1, r2;
            uint32_t c1, c2;
            SP_RING(n1c, r1, c1);
            SP_RING(n2c, r2, c2);
            const bool mis = n2c >= rdy || n1c < vlo;          /* n1c <= n2c */
            if (__ballot(mis)) {
                SP_MISS(n1c, r1, c1);
                SP_MISS(n2c, r2, c2);
                __builtin_amdgcn_s_waitcnt(PR_VMCNT0);
            }
            uint32_t ex, ey;
            if (ps_decide<ST>(x, s, ds, n1, r1, c1, r2, c2, ex, ey)) out[ne++] = make_uint2(ex, ey);
        }
    }
#undef SP_LD
#undef SP_ST
#undef SP_ISSUE
#undef SP_LAND
#undef SP_RING
#undef SP_MISS
    if (v < 2) a.pcount[g] = ne;
}

/* k_pspec's block order (block mode).  A wave of k_pspec walks 16 blocks'
 * segments in lockstep, so its time is that of its longest walk: on mixed
 * data a wave holding one incompressible block (a literal step at every
 * position) or one block of long jumps (every step a ring miss) held the
 * other 15 to its pace.  k_pweight classes each block by the share of
 * positions without a match of length 3 (every 256th match record, four
 * classes); k_porder lists the blocks class by class, heaviest first and in
 * block order within a class (a stable counting sort: blocks of one kind stay
 * neighbours in memory, and a uniform input keeps the launch order), so that
 * similar walks share waves and the long ones start first.  The lists keep
 * their (set, block, segment) slots: nothing downstream sees the order. */
#define PO_CLASSES 4u
__global__ __launch_bounds__(256) void k_pweight(const uint64_t* __restrict__ rec, uint64_t n, uint32_t bs,
                                                 uint32_t* __restrict__ w)
{
    __shared__ uint32_t cnt;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const uint32_t len = blk_len(n, bs, b);
    if (tid == 0) cnt = 0;
    __syncthreads();
    /* one sample per thread */
    const uint32_t stp = bs >= 65536 ? 256u : bs / 256u ? bs / 256u : 1u;
    const uint32_t p = tid * stp;
    uint32_t c = p < len ? (((uint32_t) rec[(uint64_t) b * bs + p] & 511) < 3) : 0u;
    for (int d = 32; d >= 1; d >>= 1) c += (uint32_t) __shfl_xor((int) c, d);
    if ((tid & 63) == 0) atomicAdd(&cnt, c);
    __syncthreads();
    const uint32_t ns = (len + stp - 1) / stp < 256 ? (len + stp - 1) / stp : 256u;
    /* class 0 = the heaviest (every sampled position without a match) */
    if (tid == 0) w[b] = ns ? (PO_CLASSES - 1) - min(cnt * PO_CLASSES / ns, PO_CLASSES - 1) : PO_CLASSES - 1;
}

__global__ __launch_bounds__(1024) void k_porder(const uint32_t* __restrict__ w, uint32_t nb,
                                                 uint32_t* __restrict__ perm)
{
    __shared__ uint32_t wsum[PO_CLASSES][16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t per = (nb + 1023) / 1024, i0 = tid * per, i1 = min(nb, i0 + per);
    uint32_t c[PO_CLASSES] = {0, 0, 0, 0};
    for (uint32_t i = i0; i < i1; i++) c[w[i]]++;
    /* per class: exclusive scan over the threads (block order) */
    uint32_t x[PO_CLASSES], tot[PO_CLASSES];
#pragma unroll
    for (uint32_t k = 0; k < PO_CLASSES; k++) {
        uint32_t v = c[k];
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = (uint32_t) __shfl_up((int) v, d);
            if (lane >= d) v += y;
        }
        x[k] = v - c[k];
        if (lane == 63) wsum[k][wv] = v;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < PO_CLASSES; k++) {
        uint32_t before = 0, all = 0;
        for (uint32_t j = 0; j < 16; j++) {
            before += j < wv ? wsum[k][j] : 0u;
            all += wsum[k][j];
        }
        x[k] += before;
        tot[k] = all;
    }
    uint32_t base = 0;
#pragma unroll
    for (uint32_t k = 0; k < PO_CLASSES; k++) {
        x[k] += base;
        base += tot[k];
    }
    for (uint32_t i = i0; i < i1; i++) {
        const uint32_t k = w[i];
        const uint32_t o = k == 0 ? x[0]++ : k == 1 ? x[1]++ : k == 2 ? x[2]++ : x[3]++;
        perm[o] = i;
    }
}

__global__ __launch_bounds__(64) void k_psync(PSplitArgs a)
{
    const uint32_t g = blockIdx.x * 64 + threadIdx.x;       /* list, as k_pspec */
    const uint32_t k = g % JD_PSEG;
    if (g >= 2 * a.nblocks * JD_PSEG) return;
    uint32_t ia = PS_NONE, jb = PS_NONE;
    const uint32_t na = a.pcount[g], nb2 = k + 1 < JD_PSEG ? a.pcount[g + 1] : 0;
    if (na && nb2) {
        const uint2* A = (const uint2*) (a.plist + (uint64_t) g * a.pcap);
        const uint2* B = A + a.pcap;
        const uint32_t s1 = (k + 1) * (a.bs / JD_PSEG);
        uint32_t lo = 0, hi = na;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((A[mid].y & 0xffff) < s1) lo = mid + 1; else hi = mid;
        }
        uint32_t i = lo, j = 0;
        while (i < na && j < nb2) {
            const uint32_t ya = A[i].y, yb = B[j].y;
            const uint32_t sa = ya & 0xffff, sb = yb & 0xffff;
            if (sa < sb) {
                i++;
            } else if (sa > sb) {
                j++;
            } else {
                if (ya & yb & PE_H0) { ia = i; jb = j; break; }
                i++;
                j++;
            }
        }
    }
    a.psync[2 * g] = ia;
    a.psync[2 * g + 1] = jb;
}

/* wave-wide inclusive prefix sum: row shifts 1, 2, 4, 8 inside each row of
 * 16 lanes, then row broadcasts of lanes 15 and 31 (DPP, no LDS traffic) */
__device__ static inline uint32_t wave_iscan(uint32_t v)
{
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x111, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x112, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x114, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x118, 0xf, 0xf, true);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x142, 0xa, 0xf, false);
    v += (uint32_t) __builtin_amdgcn_update_dpp(0, (int) v, 0x143, 0xc, 0xf, false);
    return v;
}

__device__ static inline uint32_t wave_sum(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += (uint32_t) __shfl_xor((int) v, d);
    return v;
}

/* Stream mode, the tail: a position whose match may read past the stream
 * end gets its record again over the window view (k_match and its 3-byte
 * pass, getmatch2 :2606-2721), walking the stream-global links */
__device__ static uint64_t srec_tail(const SView& v, const uint16_t* prev3, uint64_t p,
                                     uint32_t chain, uint32_t nice, bool use3)
{
    const uint32_t half = chain >> 1;
    uint32_t cl = 2, co = 0, l24 = 0, o24 = 0, left = chain;
    bool have24 = false;
    uint64_t q = p;
    for (;;) {
        const uint32_t d = v.prev4[q];
        if (!left || d == 0 || d > q) break;
        q -= d;
        if (p - q >= JD_WSIZE) break;
        if (sv_byte(v, q + cl) == sv_byte(v, p + cl)) {
            uint32_t m = 0;
            while (m < JD_MAXMATCH && sv_byte(v, p + m) == sv_byte(v, q + m)) m++;
            if (m > cl) {
                if (!have24 && half && chain - left >= half) { l24 = cl; o24 = co; have24 = true; }
                cl = m;
                co = (uint32_t) (p - q);
                if (cl >= nice) break;
            }
        }
        left--;
    }
    if (!have24) { l24 = cl; o24 = co; }
    uint32_t s3 = 0;
    if (use3 && cl < 3) {
        const uint32_t n3 = prev3[p], p32 = (uint32_t) p;
        auto eq3 = [&](uint32_t o) {
            return sv_byte(v, p - o) == sv_byte(v, p) && sv_byte(v, p - o + 1) == sv_byte(v, p + 1) &&
                   sv_byte(v, p - o + 2) == sv_byte(v, p + 2);
        };
        if (n3) {
            uint32_t noff = (p32 - n3) & 0xffff;
            if (noff <= JD_WSIZE && noff != 0) {
                if (eq3(noff)) {
                    s3 = noff;
                } else {
                    const uint32_t back = (p32 - n3) & 16383u;
                    const uint32_t n3b = back <= p ? prev3[p - back] : 0u;
                    noff = (p32 - n3b) & 0xffff;
                    if (n3b && noff <= JD_WSIZE && noff != 0 && eq3(noff)) s3 = noff;
                }
            }
        }
        if (s3 > 8192) s3 = 0;
    }
    return (uint64_t) cl | ((uint64_t) co << 9) | ((uint64_t) l24 << 24) | ((uint64_t) o24 << 33) |
           ((uint64_t) s3 << 48);
}

/* Stream mode, once the last window is known (after a slide): the hash of
 * position n-3 reads one byte past the end, so its chain head is found
 * again (the nearest earlier position in its bucket, a wave scanning 64
 * positions per step), then the records of the last positions are redone. */
__device__ static void stream_tail(const PSplitArgs& a, const SView& v, uint64_t from, uint32_t lane)
{
    const uint64_t n = a.n;
    uint16_t* prev4 = (uint16_t*) a.prev4;
    if (n >= 4) {
        const uint64_t p = n - 3;
        auto h4 = [](uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
            return (((b0 << 24) | (b1 << 16) | (b2 << 8) | b3) * 0x1e35a7bdu) >> 16;
        };
        const uint32_t hv = h4(a.in[p], a.in[p + 1], a.in[p + 2], sv_byte(v, n));
        const uint32_t hz = h4(a.in[p], a.in[p + 1], a.in[p + 2], 0);
        if (hv != hz) {
            uint32_t link = 0;
            for (uint64_t top = p; top > 0 && p - top < JD_WSIZE; top -= top < 64 ? top : 64) {
                const bool ok = top >= 1 + lane && p - (top - 1 - lane) < JD_WSIZE;
                const uint64_t q = ok ? top - 1 - lane : 0;
                const uint32_t h = !ok ? 0xffffffffu : q == 0 ? 0u : h4(a.in[q], a.in[q + 1], a.in[q + 2], a.in[q + 3]);
                const uint64_t m = __ballot(ok && h == hv);
                if (m) {
                    const uint32_t l = (uint32_t) __ffsll((unsigned long long) m) - 1;
                    link = (uint32_t) (p - (top - 1 - l));
                    break;
                }
            }
            if (lane == 0) prev4[p] = (uint16_t) link;
            __threadfence();
            __syncthreads();
        }
    }
    uint64_t* rec = (uint64_t*) a.rec;
    for (uint64_t p = from + lane; p < n; p += 64) rec[p] = srec_tail(v, a.prev3, p, a.chain, a.nice, !a.greedy);
    __threadfence();
    __syncthreads();
}

/* One wave per block joins the segment lists into the block's token stream
 * and runs the block-split observer (:2908-2948) over it, 64 tokens at a
 * time: each lane takes one token, a wave prefix sum of (slots, length)
 * gives every token's running counts, and the first token that closes a
 * deflate block (:2910) or reaches a check (newcount >= 512, obstotal >=
 * 4096) ends the batch; the check itself is evaluated by the wave.
 * A list set walked with doshort d is followed while doshort is d; while
 * doshort differs, up to the first entry flagged PE_D1 (there doshort
 * decides the step).  Where doshort changes to the value of another set the
 * block has, where a PE_D1 entry is reached, or where a list ends without
 * meeting the next, the lazy step runs serially (wave-uniform) from the
 * state at that point until it stands with nothing held at an entry of a
 * list, preferring the set walked with the current doshort.
 *
 * STREAM: one wave walks every block of a single-window stream in order; the
 * parse state, the observer, doshort and the open deflate block carry from
 * block to block (the join goes serial at a block end and rejoins the next
 * block's lists).  It also replays the reference's window slides
 * (fillwindow :1870-1897: a slide when the cursor passes the window end
 * minus MINLOOKAHEAD, by the cursor - 32 KiB rounded down to 8), and once the
 * last window is known redoes the tail records over the window's bytes
 * (stream_tail); from there the parse runs serially. */
#ifndef PJ_LSB
#define PJ_LSB 8192u
#endif
/* list entries per lane in a join batch (stream, block mode): a batch's cost
 * is mostly its ~500 wave instructions and ~60 branches, whatever its size */
#ifndef PJ_KS
#define PJ_KS 8u
#endif
#ifndef PJ_SU
#define PJ_SU 16u            /* stream: staging loads in flight per lane */
#endif
#ifndef PJ_KB
#define PJ_KB 2u
#endif
/* batch entry idx lives in lane idx / PK, slot idx % PK (lane-major order) */
template <uint32_t PK>
__device__ static inline uint32_t pj_first(const bool (&p)[PK])
{
    uint32_t lf = PK;
#pragma unroll
    for (int q = (int) PK - 1; q >= 0; q--)
        if (p[q]) lf = (uint32_t) q;
    const uint64_t m = __ballot(lf < PK);
    if (!m) return ~0u;
    const uint32_t l = (uint32_t) __ffsll((unsigned long long) m) - 1;
    return l * PK + (uint32_t) __builtin_amdgcn_readlane((int) lf, (int) l);
}
/* every slot read out of the lane, then a scalar select (a select among
 * the slots in registers became a dynamic index into scratch, whose load
 * waited for every store in flight) */
template <uint32_t PK>
__device__ static inline uint32_t pj_pick(const uint32_t (&v)[PK], uint32_t idx)
{
    const uint32_t q = idx % PK, l = idx / PK;
    uint32_t s = (uint32_t) __builtin_amdgcn_readlane((int) v[0], (int) l);
#pragma unroll
    for (uint32_t k = 1; k < PK; k++) {
        const uint32_t t = (uint32_t) __builtin_amdgcn_readlane((int) v[k], (int) l);
        s = q == k ? t : s;
    }
    return s;
}
#ifndef PJ_PF
#define PJ_PF 1
#endif
template <bool STREAM>
/* block mode: 78 VGPRs, 6 waves per SIMD (16,384 one-wave blocks; the walk
 * is latency-bound).  Held to 72 for 7 waves it spilled a little: 3.66 ->
 * 3.56 ms per GiB of text, 1.49 -> 1.38 per 256 MiB mixed at 6
 * (gpurun_out/r6zq, r6zr); at 64 VGPRs the entry and record caches spilled */
#ifndef PJ_WPE
#define PJ_WPE 6
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(STREAM ? 1 : PJ_WPE))) void k_pjoin(PSplitArgs a)
{
    __shared__ uint32_t curr[32], prv[32];
    __shared__ uint64_t sg_b[JD_NGEN];              /* stream: window generations */
    /* stream (one wave for the whole stream): the list being followed is
     * staged in LDS, PJ_LSB entries at a time (a list load per 64-entry batch
     * left one memory latency exposed per batch) */
    __shared__ uint2 lsb[STREAM ? PJ_LSB + 64 * PJ_SU : 1];
    /* block mode: a cache of list entries (the rest of the batch a doshort
     * stop cut, by list and index), and the records and bytes of the 64
     * positions from the stop: the serial steps, the rejoin probe and the
     * batch after the rejoin read them without a global load each */
    __shared__ uint2 wl[STREAM ? 1 : 64 * PJ_KB];
    __shared__ uint64_t wr[STREAM ? 1 : 64];
    __shared__ uint8_t wc8[STREAM ? 1 : 64];
    __shared__ uint32_t sg_h[JD_NGEN];
    const uint32_t lane = threadIdx.x;
    /* stream: the parse starts at pstart (after the dictionary or the
     * history of earlier segments), in its block */
    uint32_t b = STREAM ? a.pstart / a.bs : blockIdx.x;
    if (b >= a.nblocks) return;

    const uint32_t seg = a.bs / JD_PSEG;
    const uint32_t NL = a.nblocks * JD_PSEG;                /* lists per set  */
#define LIX(v_, k_) ((v_) * NL + b * JD_PSEG + (k_))
#define LIST(v_, k_) ((const uint2*) (a.plist + (uint64_t) LIX(v_, k_) * a.pcap))
#define PIECE_END(v_, k_) (((k_) + 1 < JD_PSEG && a.psync[2 * LIX(v_, k_)] != PS_NONE) \
                           ? a.psync[2 * LIX(v_, k_)] : a.pcount[LIX(v_, k_)])

    if (lane < 32) { curr[lane] = 0; prv[lane] = 0; }
    __syncthreads();
    uint32_t obscount = 0, newcount = 0, obstotal = 0;
    uint32_t nt = 0, slots = 0, ndb = 0, ds = STREAM ? a.w0.ds : 0;
    /* stream: the reference's window buffer (JdWinState: window[0] at sbase,
     * inputend at inend, earlier generations in sg_*), the limit of the
     * parse loop, the reference's call being served, the tail start */
    uint64_t sbase = a.w0.sbase, inend = a.w0.inend, lim = a.pstart;
    uint32_t ngen = STREAM ? min(a.w0.ngen, (uint32_t) JD_NGEN) : 0, callk = 0;
    uint32_t nslide = 0, tailed = 0, gerr = 0;
    if (STREAM && lane < JD_NGEN) { sg_b[lane] = a.w0.gb[lane]; sg_h[lane] = a.w0.gh[lane]; }
    const uint64_t tail0 = a.n > JD_MAXMATCH + 4 ? a.n - (JD_MAXMATCH + 4) : 0;
    const uint32_t LA = 261;        /* MINLOOKAHEAD, deflator.c:2328 */

#define RESETOBS() do { if (lane < 32) { curr[lane] = 0; prv[lane] = 0; } obscount = newcount = obstotal = 0; } while (0)
#define CLOSEDB() do { if (STREAM) { if (lane == 0) { a.sdb[1 + 2 * ndb] = nt; a.sdb[2 + 2 * ndb] = slots; } } \
                       else if (ndb < JD_MAXDB && lane == 0) { dbi[1 + 2 * ndb] = nt; dbi[2 + 2 * ndb] = slots; } \
                       ndb++; slots = 0; } while (0)

    PSt s;
    s.cur = 0; s.hm = 0; s.hl = 0; s.ho = 0; s.lastc = 0; s.hfresh = 0; s.h3 = 0; s.r = 0; s.c = 0;
    bool carry = false;
#ifdef JD_PJSTATS
#ifndef PJ_SEVERY
#define PJ_SEVERY 64
#endif
    const uint64_t st_k0 = __builtin_amdgcn_s_memrealtime();
    uint64_t st_in = 0;             /* stream: clocks inside the blocks' loops */
#endif
    __syncthreads();
    for (;;) {
    const uint32_t len = blk_len(a.n, a.bs, b);
    PCtx x = ps_ctx(a, b, len);
    if (STREAM) {
        x.v.vbase = sbase;
        x.v.gb = sg_b;
        x.v.gh = sg_h;
        x.v.ngen = ngen;
    }
    uint32_t* tok = STREAM ? a.tokens : a.tokens + (uint64_t) b * a.bs;
    uint32_t* dbi = a.dbinfo + (uint64_t) (STREAM ? 0 : b) * DBSTRIDE;
    const uint32_t mask = a.dsg[b];                         /* sets walked    */

    /* stream: the limit of compress2's parse loop from cursor c (parse_limit
     * :2806-2824; a call without a flush that runs out of input returns, and
     * the next call re-enters at the same cursor) */
    auto reloop = [&](uint64_t c) {
        for (;;) {
            const uint64_t srcleft = a.cend[callk] - inend;
            const bool fl = callk + 1 >= a.ncall;
            if (inend - c > LA + 1) { lim = inend - ((!fl || srcleft) ? LA : 0u); return; }
            if (srcleft) { lim = c; return; }
            if (!fl) { callk++; continue; }
            lim = inend;
            return;
        }
    };
    /* stream: fillwindow :1870-1897 each time the parse loop ends before a
     * step at cursor c (or compress2 re-enters there after a block flush):
     * slide when the call's remaining input does not fit and less than 1 KiB
     * is left (by the cursor - 32 KiB rounded down to 8, slidewindow
     * :1818-1862), copy what fits; once all input is in, the window is final
     * and the tail records are redone over it */
    auto fill_at = [&](uint64_t c, bool reentry) {
        if (reentry) reloop(c);
        while (c >= lim) {
            const uint64_t total = a.cend[callk] - inend;
            uint64_t il = inend - sbase;
            if (total > a.wend - il && a.wend - il < 0x400) {
                const uint64_t from = (c - sbase - JD_WSIZE) & ~7ull;
                /* the retired generation hides every older one it filled as far */
                uint64_t nb[JD_NGEN];
                uint32_t nh[JD_NGEN], m = 1;
                nb[0] = sbase;
                nh[0] = (uint32_t) il;
                for (uint32_t g = 0; g < ngen; g++) {
                    if (sg_h[g] > (uint32_t) il) {
                        if (m < JD_NGEN) { nb[m] = sg_b[g]; nh[m] = sg_h[g]; m++; }
                        else gerr = 1;
                    }
                }
                __syncthreads();
                if (lane < m) { sg_b[lane] = nb[lane]; sg_h[lane] = nh[lane]; }
                __syncthreads();
                ngen = m;
                sbase += from;
                il -= from;
                nslide++;
                x.v.vbase = sbase;
                x.v.ngen = ngen;
            }
            const uint64_t room = a.wend - il;
            const uint64_t cp = total < room ? total : room;
            inend += cp;
            if (cp == 0) {
                if (callk + 1 >= a.ncall) { lim = ~0ull; break; }
                callk++;
            }
            reloop(c);
            if (inend >= a.n && !tailed && ngen) {
                stream_tail(a, x.v, tail0, lane);
                tailed = 1;
            }
        }
    };

    /* list mode: entries [i, iend) of list kk of set cs; serial mode: s */
    uint32_t cs = (mask & 1) ? 0 : 1;
    const bool pst = STREAM && !carry && a.pstart;
    bool fast = len > 0 && !carry && !pst, done = len == 0;
    uint32_t kk = 0, i = 0, iend = fast ? PIECE_END(cs, 0) : 0;
    uint32_t lx = 0, ly = 0;                /* last list entry consumed        */
    if (pst) {
        /* after a dictionary or the history the parse starts at its end,
         * nothing held */
        s.cur = a.pstart - b * a.bs;
        carry = true;
    }
    if (carry && !done) {
        if (s.cur >= len) done = true;
        else ps_load(x, s.cur, s.r, s.c);
    }
    uint32_t jk = PS_NONE, jp = 0;          /* serial mode: rejoin search cursor */
    uint32_t pf_lid = PS_NONE, pf_i = 0;    /* list entries loaded ahead       */
    uint2 pfe = make_uint2(0, 0);
    uint32_t sb_lid = PS_NONE, sb_lo = 0, sb_hi = 0;   /* stream: entries in lsb */
    uint32_t wl_lid = PS_NONE, wl_i0 = 0, wl_n = 0;    /* block: entries in wl  */
    uint32_t w0 = 0x80000000u;                         /* block: wr/wc8 from w0 */
    uint32_t bl_i = 0, bl_n = 0;                       /* the batch: first entry, count */
    uint32_t jn2c = 0;                                 /* pcount of list jk      */
    /* a step's record and byte: the window, or global memory */
    auto wld = [&](uint32_t p_, uint64_t& r_, uint32_t& c_) {
        if (!STREAM && p_ - w0 < 64u) { r_ = wr[p_ - w0]; c_ = wc8[p_ - w0]; }
        else ps_load(x, p_, r_, c_);
    };
#ifdef JD_PJSTATS
    uint32_t st_serial = 0, st_d1 = 0, st_end = 0, st_batch = 0, st_ev = 0, st_rejoin = 0;
    uint64_t st_t0 = __builtin_amdgcn_s_memrealtime(), st_tq = st_t0, st_tk[6] = {0, 0, 0, 0, 0, 0};
#define PJS(x_) (x_)++
#define PJT(i_) do { const uint64_t t_ = __builtin_amdgcn_s_memrealtime(); st_tk[i_] += t_ - st_tq; st_tq = t_; } while (0)
#else
#define PJS(x_) ((void) 0)
#define PJT(i_) ((void) 0)
#endif
    /* serial mode from the state after the last consumed entry */
#define TO_SERIAL_AFTER_LAST()                                                          \
    do {                                                                                \
        fast = false;                                                                   \
        const uint32_t st_ = ly & 0xffff;                                               \
        if (ly & PE_ACC) {                                                              \
            s.cur = st_ + 2; s.hm = 1; s.hl = (lx >> 8) & 511; s.ho = lx >> 17;         \
            s.lastc = x.src[st_ + 1];                                                   \
        } else {                                                                        \
            s.cur = st_ + ((ly & PE_MATCH) ? (lx >> 16) & 511 : 1); s.hm = 0;           \
        }                                                                               \
        s.hfresh = 0; s.h3 = 0;                                                         \
        jk = PS_NONE;                                                                   \
        if (s.cur >= len) done = true;                                                  \
        else ps_load(x, s.cur, s.r, s.c);                                               \
    } while (0)

    constexpr uint32_t PK = STREAM ? PJ_KS : PJ_KB;
    while (!done) {
        uint32_t ex[PK], ey[PK], cnt;
#pragma unroll
        for (uint32_t q = 0; q < PK; q++) { ex[q] = 0; ey[q] = 0; }
        bool d1stop = false;
        if (fast) {
            if (i >= iend) {
                if (kk + 1 < JD_PSEG && a.psync[2 * LIX(cs, kk)] != PS_NONE) {
                    i = a.psync[2 * LIX(cs, kk) + 1];
                    kk++;
                    iend = PIECE_END(cs, kk);
                    continue;
                }
                /* the list ended without meeting the next */
                PJS(st_end);
                if (i == 0 && kk == 0) { fast = false; s.cur = 0; s.hm = 0; ps_load(x, 0, s.r, s.c); continue; }
                TO_SERIAL_AFTER_LAST();
                continue;
            }
            cnt = min(64u * PK, iend - i);
            PJS(st_batch);
            /* the batch's entries were usually loaded one batch ahead (a
             * batch consumes all of them unless an event or a d1 stop cuts
             * it); the next batch's are loaded now, so each batch's list load
             * overlaps the previous batch's observer work */
            const uint32_t lid = LIX(cs, kk);
            uint2 e = make_uint2(0, 0);
            if (STREAM) {
                if (lid != sb_lid || i < sb_lo || i + cnt > sb_hi) {
                    /* stage entries [i, i + PJ_LSB) of the list, PJ_SU loads
                     * per lane in flight; no lane skips a load or a store (a
                     * load left pending on a skipped path made the compiler
                     * wait for every earlier store at each batch) */
                    const uint2* src = LIST(cs, kk) + i;
                    const uint32_t hi = min(iend, i + PJ_LSB), nn = hi - i;
                    __syncthreads();
                    for (uint32_t o = 0; o < nn; o += 64 * PJ_SU) {
                        uint2 vu[PJ_SU];
#pragma unroll
                        for (uint32_t u = 0; u < PJ_SU; u++) vu[u] = src[min(o + u * 64 + lane, nn - 1)];
#pragma unroll
                        for (uint32_t u = 0; u < PJ_SU; u++) lsb[o + u * 64 + lane] = vu[u];
                    }
                    __syncthreads();
                    sb_lid = lid;
                    sb_lo = i;
                    sb_hi = hi;
                }
#pragma unroll
                for (uint32_t q = 0; q < PK; q++) {
                    const uint32_t ix = lane * PK + q;
                    if (ix < cnt) {
                        const uint2 e = lsb[i - sb_lo + ix];
                        ex[q] = e.x;
                        ey[q] = e.y;
                    }
                }
            } else if (PK == 1) {
                if (PJ_PF && pf_lid == lid && pf_i == i) e = pfe;
                else if (lane < cnt) e = LIST(cs, kk)[i + lane];
                pf_lid = lid;
                pf_i = i + cnt;
                if (PJ_PF && pf_i + lane < iend) pfe = LIST(cs, kk)[pf_i + lane];
                if (lane < cnt) {
                    ex[0] = e.x;
                    ey[0] = e.y;
                }
            } else {
                /* the entries a doshort stop staged, when the batch starts
                 * among them (it then ends with them) */
                const bool hit = lid == wl_lid && i - wl_i0 < wl_n;
                if (hit) cnt = min(cnt, wl_i0 + wl_n - i);
#pragma unroll
                for (uint32_t q = 0; q < PK; q++) {
                    const uint32_t ix = lane * PK + q;
                    if (ix < cnt) {
                        e = hit ? wl[i - wl_i0 + ix] : LIST(cs, kk)[i + ix];
                        ex[q] = e.x;
                        ey[q] = e.y;
                    }
                }
                bl_i = i;
                bl_n = cnt;
            }
            PJT(1);
            if (ds != cs) {
                bool pd[PK];
#pragma unroll
                for (uint32_t q = 0; q < PK; q++) pd[q] = lane * PK + q < cnt && (ey[q] & PE_D1);
                const uint32_t f = pj_first<PK>(pd);
                if (f != ~0u) { cnt = f; d1stop = true; }
            }
            if (STREAM && a.tailchk) {
                /* the entries' steps must not reach the tail: its records
                 * depend on the last window, redone before the serial parse
                 * runs there (steps at or past tail0 follow every slide) */
                bool pt[PK];
#pragma unroll
                for (uint32_t q = 0; q < PK; q++) {
                    const uint32_t stp = (ey[q] & 0xffff) + ((ey[q] & PE_HS) ? 1u : 0u);
                    pt[q] = lane * PK + q < cnt && x.gbase + stp >= tail0;
                }
                const uint32_t c2 = pj_first<PK>(pt);
                if (c2 != ~0u) {
                    if (c2 < cnt) { cnt = c2; d1stop = false; }
                    if (cnt == 0) {
                        if (i == 0 && kk == 0) { fast = false; s.cur = 0; s.hm = 0; ps_load(x, 0, s.r, s.c); }
                        else TO_SERIAL_AFTER_LAST();
                        continue;
                    }
                }
            }
        } else {
            /* block mode: the next step's records are loaded before the
             * rejoin probe, so the two loads share one memory latency */
            uint32_t sn1 = 0, sn2 = 0, sc1 = 0, sc2 = 0;
            uint64_t sr1 = 0, sr2 = 0;
            if (!STREAM) {
                ps_targets(x, s, sn1, sn2);
                wld(sn1, sr1, sc1);
                wld(sn2, sr2, sc2);
            }
            if (!s.hm && !(STREAM && tailed && x.gbase + s.cur + 1 >= tail0)) {
                /* nothing held: rejoin a list that stood here with nothing
                 * held, in the set walked with this doshort if there is one,
                 * else where doshort does not decide the entry's step (once
                 * the tail records are redone, only before the tail: the
                 * lists' entries there were made from the old records) */
                const uint32_t p = ((mask >> ds) & 1) ? ds : ds ^ 1;
                const uint32_t k2 = min(s.cur / seg, JD_PSEG - 1);
                const uint2* L2 = LIST(p, k2);
                const uint32_t plid = LIX(p, k2);
                const uint32_t n2c = (STREAM || p * JD_PSEG + k2 != jk) ? a.pcount[plid] : jn2c;
                /* the first entry starting at or after the cursor (entry
                 * starts increase along a list); the wave probes 64 entries
                 * per load round, so a search costs ~log64 of the list
                 * instead of log2 dependent loads */
                uint32_t lo, hi;
                if (p * JD_PSEG + k2 != jk) {
                    lo = 0;
                    hi = n2c;
                    jk = p * JD_PSEG + k2;
                    jn2c = n2c;
                } else {
                    lo = jp;
                    hi = n2c;
                }
                /* the first round probes the 64 entries from lo: the
                 * answer is usually among them (a serial episode advances
                 * the cursor a few entries at a time); block mode reads the
                 * staged entries first */
                bool near = true, found = false;
                if (!STREAM && plid == wl_lid && lo - wl_i0 < wl_n && lo < hi) {
                    const uint32_t m = min(min(64u, wl_i0 + wl_n - lo), hi - lo);
                    const bool below = lane < m && (wl[lo - wl_i0 + lane].y & 0xffff) < s.cur;
                    const uint32_t kb = (uint32_t) __builtin_popcountll(__ballot(below));
                    lo += kb;
                    found = kb < m;
                }
                while (!found && lo < hi) {
                    const uint32_t step = near ? 1u : (hi - lo + 63) >> 6;
                    near = false;
                    const uint32_t ix = lo + lane * step;
                    const bool below = ix < hi && (L2[ix].y & 0xffff) < s.cur;
                    const uint32_t kb = (uint32_t) __builtin_popcountll(__ballot(below));
                    if (step == 1) {
                        lo += kb;
                        if (kb < 64) break;
                        continue;
                    }
                    const uint32_t nhi = lo + kb * step;
                    if (kb) lo += (kb - 1) * step + 1;
                    if (nhi < hi) hi = nhi;
                }
                jp = lo;
                if (jp < n2c) {
                    const uint32_t y2 = (!STREAM && plid == wl_lid && jp - wl_i0 < wl_n) ? wl[jp - wl_i0].y : L2[jp].y;
                    const bool before_tail = !STREAM || !a.tailchk || x.gbase + s.cur + 1 < tail0;
                    if ((y2 & 0xffff) == s.cur && (y2 & PE_H0) && !(ds != p && (y2 & PE_D1)) && before_tail) {
                        PJS(st_rejoin);
                        fast = true;
                        /* block mode: the end of the list followed before is
                         * still known (a stream block entered with a carried
                         * parse has none yet) */
                        if (STREAM || !(p == cs && k2 == kk)) iend = PIECE_END(p, k2);
                        cs = p;
                        kk = k2;
                        i = jp;
                        continue;
                    }
                }
            }
            bool emitted = false;
            if (STREAM) {
                /* one step at a time: every cursor position can slide */
                for (;;) {
                    fill_at(x.gbase + s.cur, false);
                    if (tailed && x.gbase + s.cur >= tail0) ps_load(x, s.cur, s.r, s.c);
                    PJS(st_serial);
                    if (ps_step<STREAM>(x, s, ds, ex[0], ey[0])) { emitted = true; break; }
                    if (s.cur >= len) break;
                }
            } else {
                PJS(st_serial);
                if (!ps_decide<STREAM>(x, s, ds, sn1, sr1, sc1, sr2, sc2, ex[0], ey[0])) {
                    for (;;) {
                        PJS(st_serial);
                        ps_targets(x, s, sn1, sn2);
                        wld(sn1, sr1, sc1);
                        wld(sn2, sr2, sc2);
                        if (ps_decide<STREAM>(x, s, ds, sn1, sr1, sc1, sr2, sc2, ex[0], ey[0])) break;
                    }
                }
                emitted = true;
            }
            cnt = emitted ? 1 : 0;
        }

        PJT(2);
        /* the observer over tokens [0, cnt) of the batch: per token its
         * running (slots, length) sums, slots in bits 21+ (<= 3 per token),
         * lengths below (<= 258 per token, 64 * PK tokens) */
        static_assert(64 * PK * 3 < 2048 && 64 * PK * 258 < (1u << 21), "observer sums overflow");
        uint32_t tv[PK], pv[PK], run = 0;
        bool evq[PK];
#pragma unroll
        for (uint32_t q = 0; q < PK; q++) {
            const bool m = (ey[q] & PE_MATCH) != 0;
            const uint32_t ml = m ? (ex[q] >> 16) & 511 : 1;
            tv[q] = m ? ex[q] : (ex[q] & 0xff);
            run += lane * PK + q < cnt ? ((m ? 3u : 1u) << 21) | ml : 0u;
            pv[q] = run;
        }
        {
            const uint32_t base = wave_iscan(run) - run;
#pragma unroll
            for (uint32_t q = 0; q < PK; q++) {
                const uint32_t ix = lane * PK + q;
                pv[q] += base;
                evq[q] = ix < cnt && ((slots + (pv[q] >> 21) + 4 > a.lzcap) ||
                                      (!a.greedy && newcount + ix + 1 >= 512 && obstotal + (pv[q] & 0x1fffff) >= 4096));
            }
        }
        const uint32_t fe = pj_first<PK>(evq);
        const bool em = fe != ~0u;
        const uint32_t c = em ? fe + 1 : cnt;
#pragma unroll
        for (uint32_t q = 0; q < PK; q++) {
            const uint32_t ix = lane * PK + q;
            if (ix < c) {
                const bool m = (ey[q] & PE_MATCH) != 0;
                tok[nt + ix] = tv[q];
                atomicAdd(&curr[m ? 16 + (lsym_bf((ex[q] >> 16) & 511) >> 1) : tv[q] >> 4], 1u);
            }
        }
        if (c) {
            const uint32_t Pc = pj_pick<PK>(pv, c - 1);
            nt += c;
            slots += Pc >> 21;
            obstotal += Pc & 0x1fffff;
            newcount += c;
            PJT(3);
            if (fast) {
                lx = pj_pick<PK>(ex, c - 1);
                ly = pj_pick<PK>(ey, c - 1);
                i += c;
                if (STREAM) {
                    /* in order, every step of these entries at or past the
                     * loop limit (an entry's start, or the held step after
                     * it, PE_HS): the reference fills its window there.
                     * Entry starts increase with the lane, so the first step
                     * at or past a bound is the first lane with one (a
                     * ballot); the batch's last step, below the limit, rules
                     * out the whole batch at once (nearly every batch: the
                     * limit moves once per 32 KiB of input).  (A wave-wide
                     * minimum per batch instead cost 0.2-0.6 us of the
                     * ~1.8 us a stream batch takes.) */
                    const uint32_t sl = ly & 0xffff;
                    if (x.gbase + sl + 1 >= lim) {
                        uint64_t after = 0;
                        for (;;) {
                            const uint64_t lo = lim > after ? lim : after;
                            bool hit[PK];
                            uint32_t atv[PK];
#pragma unroll
                            for (uint32_t q = 0; q < PK; q++) {
                                const uint32_t st = ey[q] & 0xffff;
                                const bool vq = lane * PK + q < c;
                                const bool at = vq && x.gbase + st >= lo;
                                const bool ah = vq && (ey[q] & PE_HS) && x.gbase + st + 1 >= lo;
                                hit[q] = at || ah;
                                atv[q] = at ? 1u : 0u;
                            }
                            const uint32_t j = pj_first<PK>(hit);
                            if (j == ~0u) break;
                            const uint32_t sj = pj_pick<PK>(ey, j) & 0xffff;
                            const uint32_t aj = pj_pick<PK>(atv, j);
                            const uint32_t cand = aj ? sj : sj + 1;
                            fill_at(x.gbase + cand, false);
                            after = x.gbase + cand + 1;
                        }
                    }
                }
            }
        }
        PJT(4);
        if (em) {
            PJS(st_ev);
            __syncthreads();
            /* stream: the cursor after the event's step (compress2 returns
             * there to flush a block, and its re-entry can slide) */
            uint32_t ca = s.cur;
            if (STREAM && fast)
                ca = (ly & 0xffff) + ((ly & PE_MATCH) ? (lx >> 16) & 511 : (ly & PE_ACC) ? 2u : 1u);
            if (slots + 4 > a.lzcap) {
                CLOSEDB();
                RESETOBS();
                if (STREAM) fill_at(x.gbase + ca, true);
            } else {
                ds = curr[0] >= 16;
                uint32_t dl = 0;
                if (lane < 32) {
                    const uint32_t u = prv[lane], w = curr[lane];
                    dl = u > w ? u - w : w - u;
                }
                dl = wave_sum(dl);
                if (obscount > 0 && dl >= 320 && obstotal >= 7168) {
                    RESETOBS();
                    CLOSEDB();
                    if (STREAM) fill_at(x.gbase + ca, true);
                } else {
                    if (lane < 32) {
                        prv[lane] = (prv[lane] >> 1) + (curr[lane] >> 1);
                        curr[lane] = 0;
                    }
                    obscount += newcount;
                    newcount = 0;
                }
            }
            __syncthreads();
            /* doshort now matches another set this block has: move to it */
            if (fast && ds != cs && ((mask >> ds) & 1)) TO_SERIAL_AFTER_LAST();
        } else if (d1stop) {
            /* doshort decides the fresh step at entry i's start */
            PJS(st_d1);
            fast = false;
            s.hm = 0; s.hl = 0; s.ho = 0; s.lastc = 0; s.hfresh = 0; s.h3 = 0;
            /* a rejoin in this list lies at or after entry i */
            jk = cs * JD_PSEG + kk;
            jp = i;
            if (!STREAM && PK > 1) {
                /* entry i and the rest of the batch are in registers: staged
                 * for the rejoin probe and the batch after it, with the
                 * records of the 64 positions from the entry's start */
                const uint32_t f = i - bl_i;
#pragma unroll
                for (uint32_t q = 0; q < PK; q++) {
                    const uint32_t ix = lane * PK + q;
                    if (ix >= f && ix < bl_n) wl[ix - f] = make_uint2(ex[q], ey[q]);
                }
                wl_lid = LIX(cs, kk);
                wl_i0 = i;
                wl_n = bl_n - f;
                s.cur = pj_pick<PK>(ey, f) & 0xffff;
                const uint32_t pp = s.cur + lane;
                uint64_t r_;
                uint32_t c_;
                ps_load(x, pp, r_, c_);
                wr[lane] = r_;
                wc8[lane] = (uint8_t) c_;
                w0 = s.cur;
                jn2c = a.pcount[LIX(cs, kk)];
                __syncthreads();
                s.r = wr[0];
                s.c = wc8[0];
            } else {
                s.cur = LIST(cs, kk)[i].y & 0xffff;
                ps_load(x, s.cur, s.r, s.c);
                /* the rejoin probe reads jn2c whenever jk matches */
                if (!STREAM) jn2c = a.pcount[LIX(cs, kk)];
            }
            continue;
        }
        if (!fast && s.cur >= len) done = true;
        PJT(5);
    }
#ifdef JD_PJSTATS
    /* stream: every 64th block's counts and section clocks (us) */
    st_in += __builtin_amdgcn_s_memrealtime() - st_t0;
    if (STREAM && lane == 0 && b + 1 >= a.nblocks)
        printf("PJK blocks=%u kernel=%.1f us in-loops=%.1f us\n", a.nblocks,
               (__builtin_amdgcn_s_memrealtime() - st_k0) / 100.0, st_in / 100.0);
    if (STREAM && lane == 0 && (b % PJ_SEVERY) == 0)
        printf("PJS b=%u serial=%u d1=%u end=%u batch=%u ev=%u rejoin=%u all=%.1f load=%.1f pre=%.1f"
               " obs=%.1f fill=%.1f ev=%.1f us\n", b, st_serial, st_d1, st_end, st_batch, st_ev, st_rejoin,
               (__builtin_amdgcn_s_memrealtime() - st_t0) / 100.0, st_tk[1] / 100.0, st_tk[2] / 100.0,
               st_tk[3] / 100.0, st_tk[4] / 100.0, st_tk[5] / 100.0);
    if (!STREAM && lane == 0) {
        uint32_t* q = dbi + DBSTRIDE - 8;
        q[0] = st_serial; q[1] = st_d1; q[2] = st_end; q[3] = st_batch; q[4] = st_ev;
        q[5] = st_rejoin; q[6] = mask; q[7] = ds;
    }
#endif
#undef PJS
#undef PJT
#undef TO_SERIAL_AFTER_LAST
    if (!STREAM) {
        if (slots) CLOSEDB();
        if (lane == 0) dbi[0] = ndb;
        break;
    }
    if (b + 1 >= a.nblocks) {
        if (slots) CLOSEDB();
        if (lane == 0) {
            a.sdb[0] = ndb;
            JdWinState* w = a.wout;
            w->sbase = sbase;
            w->inend = inend;
            w->ngen = ngen;
            for (uint32_t g = 0; g < JD_NGEN; g++) {
                w->gb[g] = g < ngen ? sg_b[g] : 0;
                w->gh[g] = g < ngen ? sg_h[g] : 0;
            }
            w->ds = ds;
            w->err = gerr;
            w->nt = nt;
            w->nslide = nslide;
            w->tailed = tailed;
        }
        break;
    }
    /* the next block continues from the state at this block's end */
    s.cur -= len;
    b++;
    carry = true;
    }
#undef RESETOBS
#undef CLOSEDB
#undef PIECE_END
#undef LIST
#undef LIX
}

/* ------------------------------------------------------------------------ */
/* K4: emitter.  One 256-thread workgroup per block; its deflate blocks are
 * emitted in order (flushblock :1725-1805):
 *   histogram (LDS atomics) -> code lengths (rank sort in parallel,
 *   Moffat-Katajainen + cbloom limit on one lane, :934-1136) -> canonical
 *   codes -> precode RLE with the phantom zero (:1288-1354) -> header and
 *   trees (:1634-1722, one lane) -> tokens: per-token bit counts, a
 *   workgroup exclusive scan, then every lane ORs its bits into an LDS bit
 *   buffer that is streamed to the block's output slot.
 * ------------------------------------------------------------------------ */
#define EM_T       256u
#define EM_PER     8u
#define EM_CHUNK   (EM_T * EM_PER)
#define EM_WORDS   (EM_CHUNK * 48u / 32u + 256u)

struct EmitShared {
    uint32_t lf[288], df[32], cf[19];
    uint32_t lcode[288], dcode[32], pcode[19];
    uint16_t llen[290], dlen[34], plen[19];
    uint16_t map[288];
    uint32_t w[288];
    uint16_t rle[2][300];
    uint32_t nrle[2];
    uint32_t scan[EM_T];
    uint32_t bits[EM_WORDS];
    uint32_t used, lmax, dmax, cmax;
    uint32_t bp;          /* bit position inside bits[]      */
    uint32_t wout;        /* words already streamed out      */
};

/* serial bit append by one thread */
__device__ static inline void em_put(EmitShared& s, uint32_t v, uint32_t nb)
{
    if (!nb) return;
    const uint32_t w = s.bp >> 5, sh = s.bp & 31;
    s.bits[w] |= v << sh;
    if (sh + nb > 32) s.bits[w + 1] |= v >> (32 - sh);
    s.bp += nb;
}

/* serial bit writer of one thread over s.bits, starting at s.bp: bits
 * gather in a register and whole words are stored (em_put's LDS
 * read-modify-write per call is a dependent chain of LDS latencies) */
struct EmW {
    uint64_t acc;
    uint32_t n, w;
};

__device__ static inline EmW emw_begin(const EmitShared& s)
{
    EmW b;
    b.w = s.bp >> 5;
    b.n = s.bp & 31;
    b.acc = b.n ? (s.bits[b.w] & ((1u << b.n) - 1u)) : 0u;
    return b;
}

__device__ static inline void emw_put(EmitShared& s, EmW& b, uint32_t v, uint32_t nb)
{
    b.acc |= (uint64_t) v << b.n;
    b.n += nb;
    if (b.n >= 32) {
        s.bits[b.w++] = (uint32_t) b.acc;
        b.acc >>= 32;
        b.n -= 32;
    }
}

__device__ static inline void emw_end(EmitShared& s, const EmW& b)
{
    s.bits[b.w] = (uint32_t) b.acc;
    s.bp = b.w * 32 + b.n;
}

/* stream complete words to global and keep the partial one */
/* stream complete words to global and keep the partial one.  Words past
 * s.bp are zero (invariant): nothing is written beyond the word holding
 * bit bp - 1, so only the streamed words and the partial one are reset. */
__device__ static void em_flush(EmitShared& s, uint32_t* out, bool all)
{
    __syncthreads();
    const uint32_t bp = s.bp, wout = s.wout;
    const uint32_t full = all ? (bp + 31) >> 5 : bp >> 5;
    const uint32_t keep = all ? 0u : s.bits[full];
    for (uint32_t i = threadIdx.x; i < full; i += EM_T) {
        out[wout + i] = s.bits[i];
        if (!all) s.bits[i] = 0;
    }
    if (all) return;
    __syncthreads();
    if (threadIdx.x == 0) {
        if (full) {
            s.bits[0] = keep;
            s.bits[full] = 0;
        }
        s.bp = bp & 31;
        s.wout = wout + full;
    }
    __syncthreads();
}

/* code lengths for one alphabet (computelengths :1139 + setuptable
 * :1189-1285): f[] frequencies, len[] out, codes out as (len<<16)|revcode.
 * Returns last used symbol + 1 (in s.used scratch for broadcast). */
__device__ static uint32_t em_build(EmitShared& s, uint32_t* f, uint32_t nsym,
                                    uint32_t mlen, uint16_t* len, uint32_t* code)
{
    const uint32_t tid = threadIdx.x;
    __syncthreads();
    if (tid < 64) {
        /* used symbols, counted by wave 0 */
        uint32_t u = 0;
        for (uint32_t i0 = 0; i0 < nsym; i0 += 64)
            u += (uint32_t) __builtin_popcountll(__ballot(i0 + tid < nsym && f[i0 + tid] != 0));
        if (tid == 0) {
            if (u == 0) { f[0] = 1; f[1] = 1; u = 2; }
            else if (u == 1) { if (f[0]) f[1] = 1; else f[0] = 1; u = 2; }
            s.used = u;
        }
    }
    __syncthreads();
    /* rank = position in ascending (freq, symbol) order (heapsort :971) */
    for (uint32_t i = tid; i < nsym; i += EM_T) {
        len[i] = 0;
        const uint32_t fi = f[i];
        if (!fi) continue;
        uint32_t r = 0;
        for (uint32_t j = 0; j < nsym; j++) {
            const uint32_t fj = f[j];
            r += fj && (fj < fi || (fj == fi && j < i));
        }
        s.map[r] = (uint16_t) i;
    }
    __syncthreads();
    /* the sorted weights, gathered by every thread (one lane's gather was
     * two dependent LDS reads per symbol) */
    for (uint32_t r = tid; r < s.used; r += EM_T) s.w[r] = f[s.map[r]];
    __syncthreads();
    if (tid == 0) {
        const uint32_t u = s.used;
        const long nn = (long) u;
        uint32_t* a = s.w;
#ifdef EM_SKIPBUILD
        /* timing probe only (wrong output): no length computation */
        for (long i = 0; i < nn; i++) a[i] = 9;
#else
        /* Moffat-Katajainen phase 1 (katajainen :1047-1063), with the
         * heads of both queues held in registers: the next two leaf weights
         * (the leaves ahead of `leaf` are never overwritten before they are
         * taken: after step nx, leaf >= nx + 2) and the oldest unconsumed
         * internal node's weight; a[nx] is written once, at the step's end */
        long leaf = 0, root = 0;
        uint32_t aL = a[0], aL1 = nn > 1 ? a[1] : 0u, aR = 0;
        for (long nx = 0; nx < nn - 1; nx++) {
            uint32_t w = 0;
#pragma unroll
            for (int pick = 0; pick < 2; pick++) {
                if (leaf >= nn || (root < nx && aR < aL)) {
                    w += aR;
                    a[root++] = (uint32_t) nx;
                    aR = a[root];             /* stale if root == nx: fixed below */
                } else {
                    w += aL;
                    leaf++;
                    aL = aL1;
                    aL1 = leaf + 1 < nn ? a[leaf + 1] : 0u;
                }
            }
            a[nx] = w;
            if (root == nx) aR = w;
        }
        /* depth counting (:1065-1080); the parent index below root is read
         * one ahead */
        long top = nn - 2, lvl = 1, cap = 2, maxl = 0;
        root = nn - 2;
        for (long k = nn - 1; k > 0; lvl++) {
            long avail = 0;
            uint32_t c1 = root >= 1 ? a[root - 1] : 0u, c2 = root >= 2 ? a[root - 2] : 0u;
            while (root && (long) c1 >= top) {
                root--;
                avail++;
                c1 = c2;
                c2 = root >= 2 ? a[root - 2] : 0u;
            }
            if (cap - avail) maxl = lvl;
            for (long j = cap - avail; j; j--) a[k--] = (uint32_t) lvl;
            cap = avail * 2;
            top = root;
        }
        /* limitlengths :992-1028.  With no length over mlen it changes
         * nothing: the lengths of a Huffman tree meet Kraft's sum exactly
         * (kr = 0x8000), so neither adjustment loop runs; it is skipped then
         * (three serial passes of LDS reads) */
        if (maxl > (long) mlen) {
            long kr = 0;
            for (long i = 0; i < nn; i++) {
                if (a[i] > mlen) a[i] = mlen;
                kr += 0x8000L >> a[i];
            }
            for (long i = 0; i < nn; i++)
                while (a[i] < mlen && kr > 0x8000L) { a[i]++; kr -= 0x8000L >> a[i]; }
            for (long i = nn - 1; i >= 0; i--)
                while (kr + (0x8000L >> a[i]) <= 0x8000L) { kr += 0x8000L >> a[i]; a[i]--; }
        }
#endif
        s.used = u;
    }
    __syncthreads();
    const uint32_t nused = s.used;
    for (uint32_t r = tid; r < nused; r += EM_T) len[s.map[r]] = (uint16_t) s.w[r];
    __syncthreads();
    if (tid < 64) {
        /* canonical first codes per length (setuptable :1212-1227): wave 0
         * counts the codes of each length with ballots; lane l of the
         * result holds length l */
        uint32_t cnt = 0, last = 0;
        for (uint32_t i0 = 0; i0 < nsym; i0 += 64) {
            const uint32_t li = i0 + tid < nsym ? len[i0 + tid] : 0u;
            const uint64_t nz = __ballot(li != 0);
            if (nz) last = i0 + 63 - (uint32_t) __builtin_clzll(nz);
#pragma unroll
            for (uint32_t l = 1; l < 16; l++) {
                const uint32_t c = (uint32_t) __builtin_popcountll(__ballot(li == l));
                cnt += tid == l ? c : 0u;
            }
        }
        /* nxt[l] = (nxt[l-1] + cnt[l-1]) << 1, nxt[0] = 0: serial over 15
         * lengths through lane reads */
        uint32_t nx = 0;
#pragma unroll
        for (uint32_t l = 1; l < 16; l++) {
            nx = (nx + (uint32_t) __builtin_amdgcn_readlane((int) cnt, (int) l - 1)) << 1;
            if (tid == 0) s.w[l] = nx;
        }
        if (tid == 0) {
            s.w[0] = 0;
            s.used = last + 1;
        }
    }
    __syncthreads();
    for (uint32_t i = tid; i < nsym; i += EM_T) {
        const uint32_t l = len[i];
        if (!l) { code[i] = 0; continue; }
        uint32_t r = 0;
        for (uint32_t j = 0; j < i; j++) r += len[j] == l;
        code[i] = (l << 16) | jd_rev(s.w[l] + r, l);
    }
    __syncthreads();
    const uint32_t ret = s.used;
    __syncthreads();
    return ret;
}

/* run-length coding of code lengths (countprecodes :1288-1354) */
__device__ static void em_rle(const uint16_t* c, uint32_t size, uint32_t* cf,
                              uint16_t* outl, uint32_t* nout)
{
    uint32_t o = 0, run = 0, prev = 0xffff, maxrun = 0;
    uint32_t nxt = size ? c[0] : 0u;                 /* read one symbol ahead */
    for (uint32_t i = 0; i <= size; i++) {
        const uint32_t cur = i < size ? nxt : 0;     /* phantom zero at size */
        nxt = i + 1 < size ? c[i + 1] : 0u;
        bool capped = false;
        if (cur == prev) {
            run++;
            if (run < maxrun) continue;
            capped = true;
        }
        /* the counts go out as LDS adds whose results nobody waits for (an
         * increment was a read-modify-write on the lane's critical path) */
        if (run > 2) {
            const uint32_t sym = prev ? 16 : (run > 10 ? 18 : 17);
            atomicAdd(&cf[sym], 1u);
            outl[o++] = (uint16_t) sym;
            outl[o++] = (uint16_t) run;
            if (capped) { run = 0; continue; }
        } else if (run) {
            atomicAdd(&cf[prev], run);
            for (; run; run--) outl[o++] = (uint16_t) prev;
        }
        atomicAdd(&cf[cur], 1u);
        maxrun = cur ? 6 : 136;
        outl[o++] = (uint16_t) cur;
        prev = cur;
        run = 0;
    }
    *nout = o - 1;    /* the phantom's slot becomes the terminator */
}

__device__ static inline void tok_bits(const EmitShared& s, uint32_t t,
                                       uint64_t* v, uint32_t* nb)
{
    if (!(t & JD_TOK_MATCH)) {
        const uint32_t c = s.lcode[t & 0xff];
        *v = c & 0xffff;
        *nb = c >> 16;
        return;
    }
    const uint32_t ln = (t >> 16) & 0x1ff, off = t & 0xffff;
    const uint32_t ls = jd_lsym(ln), dsy = jd_dsym(off);
    const uint32_t lc = s.lcode[257 + ls], dc = s.dcode[dsy];
    const uint32_t le = jd_lextra(ls), de = jd_dextra(dsy);
    uint64_t x = lc & 0xffff;
    uint32_t k = lc >> 16;
    x |= (uint64_t) (ln - jd_lbase(ls)) << k; k += le;
    x |= (uint64_t) (dc & 0xffff) << k; k += dc >> 16;
    x |= (uint64_t) (off - jd_dbase(dsy)) << k; k += de;
    *v = x;
    *nb = k;
}

__device__ static inline void or_bits(uint32_t* bits, uint32_t pos, uint64_t v,
                                      uint32_t nb)
{
    if (!nb) return;
    const uint32_t w = pos >> 5, sh = pos & 31;
    const uint64_t lo = v << sh;
    atomicOr(&bits[w], (uint32_t) lo);
    if (sh + nb > 32) atomicOr(&bits[w + 1], (uint32_t) (lo >> 32));
    if (sh + nb > 64) atomicOr(&bits[w + 2], (uint32_t) (v >> (64 - sh)));
}

struct EmitArgs {
    const uint32_t* tokens;
    const uint32_t* dbinfo;
    uint64_t n;
    uint32_t bs, nblocks, slotcap;
    int level;
    uint32_t fixed;
    uint32_t lastfinal;   /* 1: the last block ends with BFINAL=1 (END) */
    uint8_t* stage;
    uint32_t* csize;
    /* stream mode: one workgroup per deflate block of the list sdb
     * ([ndb, (token end, slots) ...]); its bits go to the stage at
     * sslot(b), their count to csize[b]; no terminator */
    const uint32_t* sdb;
};

/* stream mode: stage slot of deflate block b (8 B per token: tokens take at
 * most 48 bits; 1 KiB per block for the header, trees and end code) */
__host__ __device__ static inline uint64_t sslot(uint32_t t0, uint32_t b)
{
    return (uint64_t) t0 * 8u + (uint64_t) b * 1024u;
}

#ifndef EM_WPE
#define EM_WPE 7
#endif
__global__ __launch_bounds__(EM_T) __attribute__((amdgpu_waves_per_eu(EM_WPE))) void k_emit(EmitArgs a)
{
    __shared__ EmitShared s;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    const bool stream = a.sdb != nullptr;
    if (stream && b >= a.sdb[0]) return;
    const uint64_t base = stream ? 0 : (uint64_t) b * a.bs;
    const uint32_t* tok = a.tokens + base;
    const uint32_t* dbi = stream ? a.sdb : a.dbinfo + (uint64_t) b * DBSTRIDE;
    const uint32_t sb = stream ? b : 0;                   /* first list entry */
    const uint32_t ndb = stream ? 1 : min(dbi[0], JD_MAXDB);
    const uint32_t st0 = (stream && b) ? dbi[1 + 2 * (b - 1)] : 0;
    uint32_t* out = (uint32_t*) (a.stage + (stream ? sslot(st0, b) : (uint64_t) b * a.slotcap));

    for (uint32_t i = tid; i < EM_WORDS; i += EM_T) s.bits[i] = 0;
    if (tid == 0) { s.bp = 0; s.wout = 0; }
    __syncthreads();

    uint32_t t0 = st0;
    for (uint32_t db = sb; db < sb + ndb; db++) {
        const uint32_t t1 = dbi[1 + 2 * db], slots = dbi[2 + 2 * db];
        const bool dyn = !(a.level == 1 || a.fixed || slots < 0x400);
        for (uint32_t i = tid; i < 288; i += EM_T) s.lf[i] = 0;
        if (tid < 32) s.df[tid] = 0;
        if (tid < 19) s.cf[tid] = 0;
        __syncthreads();
        if (dyn) {
            /* EM_PER tokens per thread loaded together: one memory latency
             * per EM_CHUNK tokens instead of one per EM_T */
            for (uint32_t i0 = t0 + tid; i0 < t1; i0 += EM_CHUNK) {
                uint32_t tv[EM_PER];
#pragma unroll
                for (uint32_t k = 0; k < EM_PER; k++) {
                    const uint32_t i = i0 + k * EM_T;
                    tv[k] = i < t1 ? tok[i] : 0u;
                }
#pragma unroll
                for (uint32_t k = 0; k < EM_PER; k++) {
                    if (i0 + k * EM_T >= t1) break;
                    const uint32_t t = tv[k];
                    if (t & JD_TOK_MATCH) {
                        atomicAdd(&s.lf[257 + jd_lsym((t >> 16) & 0x1ff)], 1u);
                        atomicAdd(&s.df[jd_dsym(t & 0xffff)], 1u);
                    } else {
                        atomicAdd(&s.lf[t], 1u);
                    }
                }
            }
            __syncthreads();
            if (tid == 0) s.lf[256]++;
            __syncthreads();
            const uint32_t lmax = em_build(s, s.lf, 288, 15, s.llen, s.lcode);
            const uint32_t dmax = em_build(s, s.df, 32, 15, s.dlen, s.dcode);
            if (tid == 0) {
                s.lmax = lmax;
                s.dmax = dmax;
                em_rle(s.llen, lmax, s.cf, s.rle[0], &s.nrle[0]);
                em_rle(s.dlen, dmax, s.cf, s.rle[1], &s.nrle[1]);
            }
            __syncthreads();
            em_build(s, s.cf, 19, 7, s.plen, s.pcode);
            /* the precode's codes in wave 0's lanes: lane 0 reads them with
             * readlane, not by a dependent LDS read per tree symbol */
            uint32_t pcv = tid < 19 ? s.pcode[tid] : 0u;
            /* materialised in every lane of wave 0 here, in uniform control
             * flow: the readlane below runs with lane 0 alone active, so the
             * load must not be sunk into that branch */
            asm volatile("" : "+v"(pcv));
            if (tid == 0) {
                const uint8_t order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
                int i;
                for (i = 18; i >= 3; i--) if (s.plen[order[i]]) break;
                s.cmax = (uint32_t) i + 1;
                /* block header + trees (flushblock :1776-1783, emittrees) */
                EmW bw = emw_begin(s);
                emw_put(s, bw, 0, 1);
                emw_put(s, bw, 2, 2);
                emw_put(s, bw, s.lmax - 257, 5);
                emw_put(s, bw, s.dmax - 1, 5);
                emw_put(s, bw, s.cmax - 4, 4);
                for (uint32_t j = 0; j < s.cmax; j++) emw_put(s, bw, s.plen[order[j]], 3);
                for (int t = 0; t < 2; t++) {
                    const uint16_t* l = s.rle[t];
                    const uint32_t nr = s.nrle[t];
                    uint32_t e0 = nr ? l[0] : 0u, e1 = nr > 1 ? l[1] : 0u;   /* two entries ahead */
                    for (uint32_t k = 0; k < nr;) {
                        const uint32_t sym = e0;
                        const uint32_t pc = (uint32_t) __builtin_amdgcn_readlane((int) pcv, (int) sym);
                        emw_put(s, bw, pc & 0xffff, pc >> 16);
                        if (sym >= 16) {
                            const uint32_t nb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
                            const uint32_t bb = sym == 18 ? 11 : 3;
                            emw_put(s, bw, e1 - bb, nb);
                            k += 2;
                            e0 = k < nr ? l[k] : 0u;
                            e1 = k + 1 < nr ? l[k + 1] : 0u;
                        } else {
                            k += 1;
                            e0 = e1;
                            e1 = k + 1 < nr ? l[k + 1] : 0u;
                        }
                    }
                }
                emw_end(s, bw);
            }
        } else {
            for (uint32_t i = tid; i < 288; i += EM_T) s.lcode[i] = jd_static_lit(i);
            if (tid < 32) s.dcode[tid] = jd_static_dist(tid);
            if (tid == 0) { em_put(s, 0, 1); em_put(s, 1, 2); }
        }
        em_flush(s, out, false);

        /* tokens, EM_CHUNK at a time */
        for (uint32_t c0 = t0; c0 < t1; c0 += EM_CHUNK) {
            const uint32_t mine = c0 + tid * EM_PER;
            uint64_t v[EM_PER];
            uint32_t nb[EM_PER], tv[EM_PER], sum = 0;
            /* the thread's tokens are loaded together, then coded (a load
             * per token followed by its table reads cost one memory latency
             * per token) */
#pragma unroll
            for (uint32_t j = 0; j < EM_PER; j++) tv[j] = mine + j < t1 ? tok[mine + j] : 0u;
#pragma unroll
            for (uint32_t j = 0; j < EM_PER; j++) {
                nb[j] = 0; v[j] = 0;
                if (mine + j < t1) { tok_bits(s, tv[j], &v[j], &nb[j]); sum += nb[j]; }
            }
            /* exclusive scan of the per-thread bit counts: inclusive scan
             * inside each wave, then the wave totals through LDS (one
             * barrier instead of two per doubling step) */
            const uint32_t lane = tid & 63, wid = tid >> 6;
            uint32_t inc = sum;
#pragma unroll
            for (uint32_t d = 1; d < 64; d <<= 1) {
                const uint32_t y = (uint32_t) __shfl_up((int) inc, d);
                if (lane >= d) inc += y;
            }
            if (lane == 63) s.scan[wid] = inc;
            __syncthreads();
            uint32_t before = 0, total = 0;
#pragma unroll
            for (uint32_t w = 0; w < EM_T / 64; w++) {
                const uint32_t x = s.scan[w];
                before += w < wid ? x : 0u;
                total += x;
            }
            uint32_t pos = s.bp + before + inc - sum;
#pragma unroll
            for (uint32_t j = 0; j < EM_PER; j++) { or_bits(s.bits, pos, v[j], nb[j]); pos += nb[j]; }
            __syncthreads();
            if (tid == 0) s.bp += total;
            em_flush(s, out, false);
        }
        if (tid == 0) {
            const uint32_t e = s.lcode[256];
            em_put(s, e & 0xffff, e >> 16);
        }
        __syncthreads();
        t0 = t1;
    }
    if (stream) {
        __syncthreads();
        const uint32_t bits = s.wout * 32 + s.bp;
        em_flush(s, out, true);
        if (tid == 0) a.csize[b] = bits;
        return;
    }
    /* endstream :610-654: empty stored block, BFINAL per flush mode */
    if (tid == 0) {
        const bool last = b + 1 == a.nblocks;
        em_put(s, (last && a.lastfinal) ? 1 : 0, 1);
        em_put(s, 0, 2);
        s.bp = (s.bp + 7) & ~7u;
        em_put(s, 0x0000, 16);
        em_put(s, 0xffff, 16);
    }
    __syncthreads();
    const uint32_t bytes = s.wout * 4 + s.bp / 8;
    em_flush(s, out, true);
    if (tid == 0) a.csize[b] = bytes;
}

/* ------------------------------------------------------------------------ */
/* stored blocks (level 0, compress0 :796-926), one workgroup per block      */
/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(256) void k_stored(const uint8_t* __restrict__ in,
                                                uint64_t n, uint32_t bs,
                                                uint32_t nblocks, uint32_t lastfinal,
                                                uint8_t* __restrict__ stage,
                                                uint32_t slotcap,
                                                uint32_t* __restrict__ csize)
{
    const uint32_t b = blockIdx.x;
    const uint32_t len = blk_len(n, bs, b);
    const uint8_t* src = in + (uint64_t) b * bs;
    uint8_t* dst = stage + (uint64_t) b * slotcap;
    /* pieces of at most 0xffff bytes, each: 3 header bits (byte aligned, so
     * one 0x00 byte), LEN, NLEN, data */
    uint32_t o = 0;
    for (uint32_t s0 = 0; s0 < len; s0 += 0xffff) {
        const uint32_t run = min(len - s0, 0xffffu);
        if (threadIdx.x == 0) {
            dst[o] = 0;
            dst[o + 1] = (uint8_t) run; dst[o + 2] = (uint8_t) (run >> 8);
            dst[o + 3] = (uint8_t) ~run; dst[o + 4] = (uint8_t) (~run >> 8);
        }
        for (uint32_t i = threadIdx.x; i < run; i += 256) dst[o + 5 + i] = src[s0 + i];
        o += 5 + run;
    }
    if (threadIdx.x == 0) {
        const bool last = b + 1 == nblocks;
        dst[o] = (last && lastfinal) ? 1 : 0;
        dst[o + 1] = 0; dst[o + 2] = 0; dst[o + 3] = 0xff; dst[o + 4] = 0xff;
        csize[b] = o + 5;
    }
}

/* ------------------------------------------------------------------------ */
/* K5: concatenation                                                         */
/* ------------------------------------------------------------------------ */
__global__ __launch_bounds__(1024) void k_scan(const uint32_t* __restrict__ sz,
                                               uint32_t nb, uint64_t* __restrict__ off,
                                               uint64_t* __restrict__ total,
                                               const uint64_t* __restrict__ base)
{
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x;
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t s0 = min(nb, tid * per), s1 = min(nb, s0 + per);
    uint64_t acc = 0;
    for (uint32_t i = s0; i < s1; i++) acc += sz[i];
    part[tid] = acc;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint64_t x = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    const uint64_t b0 = base ? *base : 0;
    uint64_t run = b0 + part[tid] - acc;
    for (uint32_t i = s0; i < s1; i++) { off[i] = run; run += sz[i]; }
    __syncthreads();
    if (tid == 1023) *total = b0 + part[1023];
}

__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ stage,
                                                 uint32_t slotcap,
                                                 const uint32_t* __restrict__ sz,
                                                 const uint64_t* __restrict__ off,
                                                 uint8_t* __restrict__ out,
                                                 uint64_t outcap)
{
    const uint32_t b = blockIdx.x;
    const uint32_t n = sz[b];
    const uint64_t o = off[b];
    if (o + n > outcap) return;
    const uint8_t* s = stage + (uint64_t) b * slotcap;
    uint8_t* d = out + o;
    /* align the destination, then 4-byte stores assembled from 4-byte loads */
    const uint32_t head = (uint32_t) ((4 - ((uintptr_t) d & 3)) & 3);
    const uint32_t h = min(head, n);
    if (threadIdx.x < h) d[threadIdx.x] = s[threadIdx.x];
    const uint32_t body = (n - h) / 4;
    const uint32_t* s32 = (const uint32_t*) s;
    uint32_t* d32 = (uint32_t*) (d + h);
    for (uint32_t i = threadIdx.x; i < body; i += 256) {
        const uint32_t bo = h + i * 4;
        const uint32_t w0 = s32[bo >> 2], w1 = s32[(bo >> 2) + 1];
        JD_CHECK(d32 + i, 4, out + outcap);
        d32[i] = __builtin_amdgcn_alignbyte(w1, w0, bo & 3);
    }
    const uint32_t tail0 = h + body * 4;
    if (threadIdx.x < n - tail0) d[tail0 + threadIdx.x] = s[tail0 + threadIdx.x];
}

/* ------------------------------------------------------------------------ */
/* Stream mode concatenation: deflate blocks follow each other bit by bit
 * (flushblock :1725-1805 writes into one bit buffer), then endstream
 * (:610-654) adds the empty stored block.  k_sscan: bit offsets of the
 * blocks, and the terminator as one more "block" of 3 + pad + 32 bits.
 * k_sbits: byte j of the output belongs to the block holding its bit 8j,
 * which also takes the first bits of the next block. */
__global__ __launch_bounds__(1024) void k_sscan(const uint32_t* __restrict__ sdb,
                                                uint32_t* __restrict__ bl,
                                                uint64_t* __restrict__ bo,
                                                uint32_t* __restrict__ tslot,
                                                uint32_t final, uint64_t* __restrict__ total)
{
    __shared__ uint64_t part[1024];
    const uint32_t tid = threadIdx.x, nb = sdb[0];
    const uint32_t per = (nb + 1023) / 1024;
    const uint32_t s0 = min(nb, tid * per), s1 = min(nb, s0 + per);
    uint64_t acc = 0;
    for (uint32_t i = s0; i < s1; i++) acc += bl[i];
    part[tid] = acc;
    __syncthreads();
    for (uint32_t o = 1; o < 1024; o <<= 1) {
        const uint64_t x = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    uint64_t run = part[tid] - acc;
    for (uint32_t i = s0; i < s1; i++) { bo[i] = run; run += bl[i]; }
    if (tid == 0) {
        const uint64_t T = part[1023];
        const uint32_t pad = (uint32_t) ((8u - ((T + 3) & 7u)) & 7u);
        const uint64_t tv = (uint64_t) (final ? 1u : 0u) | (0xffffull << (3 + pad + 16));
        tslot[0] = (uint32_t) tv;
        tslot[1] = (uint32_t) (tv >> 32);
        tslot[2] = 0;
        bo[nb] = T;
        bl[nb] = 3 + pad + 32;
        *total = (T + 3 + pad + 32) >> 3;
    }
}

__device__ static inline uint32_t bits8(const uint32_t* w, uint64_t pos)
{
    const uint64_t i = pos >> 5;
    const uint32_t sh = (uint32_t) (pos & 31);
    const uint64_t v = ((uint64_t) w[i + 1] << 32) | w[i];
    return (uint32_t) (v >> sh) & 0xffu;
}

__global__ __launch_bounds__(256) void k_sbits(const uint32_t* __restrict__ sdb,
                                               const uint8_t* __restrict__ stage,
                                               const uint32_t* __restrict__ tslot,
                                               const uint32_t* __restrict__ bl,
                                               const uint64_t* __restrict__ bo,
                                               uint8_t* __restrict__ out, uint64_t outcap)
{
    const uint32_t k = blockIdx.x, nb = sdb[0];
    if (k > nb) return;
    auto slot = [&](uint32_t j) -> const uint32_t* {
        if (j == nb) return tslot;
        const uint32_t t0 = j ? sdb[1 + 2 * (j - 1)] : 0;
        return (const uint32_t*) (stage + sslot(t0, j));
    };
    const uint32_t* me = slot(k);
    const uint32_t* nx = k < nb ? slot(k + 1) : nullptr;
    const uint64_t o = bo[k], e = o + bl[k];
    const uint64_t j0 = (o + 7) >> 3, j1 = (e + 7) >> 3;
    for (uint64_t j = j0 + threadIdx.x; j < j1; j += 256) {
        const uint64_t p = 8 * j;
        const uint32_t mine = e - p < 8 ? (uint32_t) (e - p) : 8u;
        uint32_t v = bits8(me, p - o) & ((1u << mine) - 1);
        if (mine < 8 && nx) v |= (bits8(nx, 0) << mine) & 0xffu;
        if (j < outcap) out[j] = (uint8_t) v;
    }
}

/* stream mode, level 0 (compress0 :796-926 with the whole input given):
 * stored blocks of 65535 bytes, then endstream */
__global__ __launch_bounds__(256) void k_sstored(const uint8_t* __restrict__ in, uint64_t n,
                                                 uint32_t final, uint8_t* __restrict__ out)
{
    const uint64_t nblk = (n + 65534) / 65535;
    const uint64_t j = blockIdx.x;
    if (j < nblk) {
        const uint64_t s0 = j * 65535, run = n - s0 < 65535 ? n - s0 : 65535;
        uint8_t* d = out + j * 65540;
        if (threadIdx.x == 0) {
            d[0] = 0;
            d[1] = (uint8_t) run; d[2] = (uint8_t) (run >> 8);
            d[3] = (uint8_t) ~run; d[4] = (uint8_t) (~run >> 8);
        }
        for (uint64_t i = threadIdx.x; i < run; i += 256) d[5 + i] = in[s0 + i];
    } else if (threadIdx.x == 0) {
        uint8_t* d = out + nblk * 5 + n;
        d[0] = final ? 1 : 0;
        d[1] = 0; d[2] = 0; d[3] = 0xff; d[4] = 0xff;
    }
}

/* ------------------------------------------------------------------------ */
/* launch sequence                                                           */
/* ------------------------------------------------------------------------ */
/* k_chains' `stream` argument; JD_CHAINS_SERIAL=1 (tests) forces the
 * serial filing path */
static int jd_chains_flag(int stream)
{
    const char* e = getenv("JD_CHAINS_SERIAL");
    return stream | ((e && *e == '1') ? 2 : 0);
}

/* Test hook (JD_TEST_BADLINKS=1, tests/test_gpu.py
 * test_bad_links_never_fault): about half of the hash-4 links are replaced by
 * links longer than their position.  Every walk must then stay in bounds
 * (k_match ends on the window test, the global walks on d > q) and the output
 * must still be a valid encoding of the input (every match is verified
 * against the bytes). */
__global__ __launch_bounds__(256) void k_badlinks(uint16_t* __restrict__ prev4, uint32_t* __restrict__ slw,
                                                   uint32_t chain, uint64_t n, uint32_t bs)
{
    const uint64_t g = (uint64_t) blockIdx.x * 256 + threadIdx.x;
    if (g >= n) return;
    uint32_t h = (uint32_t) g * 0x9e3779b1u;
    h ^= h >> 15;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    if (h & 1) return;
    const uint32_t p = (uint32_t) (g % bs);
    prev4[g] = (uint16_t) (p < 32766 ? p + 1 + (h >> 8) % (32767 - p) : 65535 - ((h >> 8) & 255));
    /* block mode: a slice rank and candidate count anywhere in range, so
     * k_match_sl walks slices of other buckets and positions (its window
     * test must keep every candidate in [p - 32767, p)) */
    if (slw) slw[g] = ((h >> 4) & 0xffffu) | ((((h >> 20) * 7u) % (chain + 1)) << 16);
}

static bool test_badlinks()
{
    const char* e = getenv("JD_TEST_BADLINKS");
    return e && *e == '1';
}

/* bytes of L->chains per input position the block pipeline needs */
extern "C" uint32_t jdk_chains_bytes(int level)
{
    return level >= K2S_FROM ? 10u : 4u;
}

extern "C" int jdk_deflate_launch(const JdDeflateLaunch* L)
{
    hipStream_t st = (hipStream_t) L->stream;
    const uint32_t nb = L->nblocks;
    if (!nb) return 0;
    if (L->level == 0) {
        JDPROF_RUN(JDK_STORED, st, (k_stored<<<nb, 256, 0, st>>>(L->in, L->n, L->bs, nb, L->lastfinal,
                                                                 L->stage, L->slotcap, L->csize)));
    } else {
        const JdLevel lv = jd_level(L->level);
        const bool lazy = L->level >= 6;
        uint16_t* prev4 = L->chains;
        uint16_t* prev3 = L->chains + L->nslots;
        if (L->level < K2S_FROM) {
        /* the hash-4 links and k_match's link walk (the slice walk below
         * measured slower at level 6: DESIGN.md §9 round 6) */
        JDPROF_RUN(JDK_CHAINS4, st, (k_chains<4><<<nb, 1024, 0, st>>>(L->in, L->n, L->bs, prev4, nullptr, jd_chains_flag(0), nullptr, 0,
                                                                          nullptr, 0)));
        if (test_badlinks()) k_badlinks<<<(uint32_t) ((L->n + 255) / 256), 256, 0, st>>>(prev4, nullptr, 0, L->n, L->bs);
        if (lazy)
            JDPROF_RUN(JDK_CHAINS3, st, (k_chains<3><<<nb, 1024, 0, st>>>(L->in, L->n, L->bs, prev3, L->dsg, jd_chains_flag(0), nullptr, 0,
                                                                          nullptr, 0)));
        {
            const uint32_t nsub = (L->bs + K2_SR - 1) / K2_SR;
            /* greedy levels use getmatch1 :2335: initial threshold MINMATCH, so
             * a record only matters when longer than 3 */
            if (L->level >= 8)
                JDPROF_RUN(JDK_MATCH, st, (k_match<true><<<nb * nsub, 1024, 0, st>>>(L->in, L->n, L->bs, prev4, prev3,
                                                                                     L->rec, lv.chain, lv.nice,
                                                                                     lazy ? 3 : 4, lazy ? 1 : 0)));
            else
                JDPROF_RUN(JDK_MATCH, st, (k_match<false><<<nb * nsub, 1024, 0, st>>>(L->in, L->n, L->bs, prev4, prev3,
                                                                                      L->rec, lv.chain, lv.nice,
                                                                                      lazy ? 3 : 4, lazy ? 1 : 0)));
        }
        } else {
        /* the slices: S after 16 entries of padding (a chunk load may start
         * below a block's first entry), W 4-byte aligned after it */
        uint16_t* sl_s = L->chains + 2 * L->nslots + 16;
        uint32_t* sl_w = (uint32_t*) (L->chains + 3 * L->nslots + 32);
        SlOut<true> so;
        so.s = sl_s; so.w = sl_w; so.chain = lv.chain;
        JDPROF_RUN(JDK_CHAINS4, st, (k_chains<4, false, true><<<nb, 1024, 0, st>>>(L->in, L->n, L->bs, prev4, nullptr,
                                                                                  jd_chains_flag(0), nullptr, 0,
                                                                                  nullptr, 0, so)));
        if (test_badlinks())
            k_badlinks<<<(uint32_t) ((L->n + 255) / 256), 256, 0, st>>>(prev4, sl_w, lv.chain, L->n, L->bs);
        if (lazy)
            JDPROF_RUN(JDK_CHAINS3, st, (k_chains<3><<<nb, 1024, 0, st>>>(L->in, L->n, L->bs, prev3, L->dsg, jd_chains_flag(0), nullptr, 0,
                                                                          nullptr, 0)));
        const uint32_t nsub = (L->bs + K2_SR - 1) / K2_SR;
        if (L->level >= 8)
            JDPROF_RUN(JDK_MATCH, st, (k_match_sl<true, K2S_NT><<<nb * nsub, K2S_NT, 0, st>>>(
                                          L->in, L->n, L->bs, sl_s, sl_w, prev3, L->rec, lv.chain, lv.nice,
                                          lazy ? 1 : 0)));
        else
            JDPROF_RUN(JDK_MATCH, st, (k_match_sl<false, K2S_NT><<<nb * nsub, K2S_NT, 0, st>>>(
                                          L->in, L->n, L->bs, sl_s, sl_w, prev3, L->rec, lv.chain, lv.nice,
                                          lazy ? 1 : 0)));
        }
        ParseArgs pa;
        pa.rec = L->rec; pa.prev4 = prev4; pa.in = L->in; pa.n = L->n; pa.bs = L->bs;
        pa.nblocks = nb; pa.tokens = L->tokens;
        pa.dbinfo = L->dbinfo; pa.good = lv.good; pa.lzcap = lv.lzcap;
        pa.nice = lv.nice; pa.half = lv.chain >> 1; pa.lazy = lazy;
        if (lazy && L->plist) {
            PSplitArgs ps;
            memset(&ps, 0, sizeof(ps));
            ps.rec = L->rec; ps.prev4 = prev4; ps.in = L->in; ps.n = L->n; ps.bs = L->bs;
            ps.nblocks = nb; ps.tokens = L->tokens; ps.dbinfo = L->dbinfo;
            ps.good = lv.good; ps.lzcap = lv.lzcap; ps.nice = lv.nice; ps.half = lv.chain >> 1;
            ps.plist = L->plist; ps.pcount = L->pcount; ps.psync = L->psync; ps.pcap = L->pcap;
            ps.dsg = L->dsg;
            if (L->pord && nb > 16) {
                JDPROF_RUN(JDK_PORDER, st, (k_pweight<<<nb, 256, 0, st>>>(L->rec, L->n, L->bs, L->pord)));
                JDPROF_RUN(JDK_PORDER, st, (k_porder<<<1, 1024, 0, st>>>(L->pord, nb, L->pord + nb)));
                ps.perm = L->pord + nb;
            }
            const uint32_t ng = (2 * nb * JD_PSEG + 63) / 64;
            JDPROF_RUN(JDK_PSPEC, st, (k_pspec<false><<<ng, 64, 0, st>>>(ps)));
            JDPROF_RUN(JDK_PSYNC, st, (k_psync<<<ng, 64, 0, st>>>(ps)));
            JDPROF_RUN(JDK_PJOIN, st, (k_pjoin<false><<<nb, 64, 0, st>>>(ps)));
        } else {
            JDPROF_RUN(JDK_PARSE, st, (k_parse<<<(nb + 63) / 64, 64, 0, st>>>(pa)));
        }
        EmitArgs ea;
        ea.tokens = pa.tokens; ea.dbinfo = L->dbinfo; ea.n = L->n; ea.bs = L->bs;
        ea.nblocks = nb; ea.slotcap = L->slotcap; ea.level = L->level;
        ea.fixed = L->flags & 1u; ea.lastfinal = L->lastfinal;
        ea.stage = L->stage; ea.csize = L->csize; ea.sdb = nullptr;
        JDPROF_RUN(JDK_EMIT, st, (k_emit<<<nb, EM_T, 0, st>>>(ea)));
    }
    JDPROF_RUN(JDK_SCAN, st, (k_scan<<<1, 1024, 0, st>>>(L->csize, nb, L->coff, L->total, L->base)));
    if (L->out)
        JDPROF_RUN(JDK_COMPACT, st, (k_compact<<<nb, 256, 0, st>>>(L->stage, L->slotcap, L->csize,
                                                                    L->coff, L->out, L->outcap)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

/* Single-window stream: chains over 32 KiB units, match records over the
 * whole stream as one block, segment lists per 64 KiB block, one wave
 * joining them in order (window slides, tail), then every deflate block
 * emitted on its own and the bits concatenated. */
extern "C" int jdk_deflate_stream_launch(const JdStreamLaunch* L)
{
    hipStream_t st = (hipStream_t) L->stream;
    const uint64_t n = L->n;
    const uint32_t final = L->final ? 1u : 0u;
    if (L->level == 0) {
        /* deflator_setdctnr has no effect at level 0 (:2112) */
        const uint64_t nd = n - L->dsize;
        const uint64_t nblk = (nd + 65534) / 65535;
        JDPROF_RUN(JDK_STORED, st, (k_sstored<<<(uint32_t) (nblk + 1), 256, 0, st>>>(L->in + L->dsize, nd,
                                                                                      final, L->out)));
        const uint64_t tot = nblk * 5 + nd + 5;
        if (hipMemcpyAsync(L->total, &tot, 8, hipMemcpyHostToDevice, st) != hipSuccess) return -1;
        return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
    }
    if (L->level < 1 || L->level > 9 || n >= (1ull << 32) - 65536) return -1;
    const JdLevel lv = jd_level(L->level);
    const bool lazy = L->level >= 6;
    const uint64_t maxdb = jdk_stream_maxdb(n);
    if (hipMemsetAsync(L->sdb, 0, 4, st) != hipSuccess) return -1;
    if (n) {
        const uint32_t unit = 32768, bs = 65536;
        const uint32_t nunits = (uint32_t) ((n + unit - 1) / unit);
        const uint32_t nb = (uint32_t) ((n + bs - 1) / bs);
        uint16_t* prev4 = L->chains;
        uint16_t* prev3 = L->chains + n;
        if (L->nov)
            JDPROF_RUN(JDK_CHAINS4, st, (k_chains<4, true><<<nunits, 1024, 0, st>>>(L->in, n, unit, prev4, nullptr, jd_chains_flag(1), nullptr,
                                                                                    L->dsize, L->ov, L->nov)));
        else
            JDPROF_RUN(JDK_CHAINS4, st, (k_chains<4><<<nunits, 1024, 0, st>>>(L->in, n, unit, prev4, nullptr, jd_chains_flag(1), nullptr,
                                                                              L->dsize, nullptr, 0)));
        if (test_badlinks() && n < 65536) k_badlinks<<<(uint32_t) ((n + 255) / 256), 256, 0, st>>>(prev4, nullptr, 0, n, 65536);
        if (lazy) {
            JDPROF_RUN(JDK_CHAINS3, st, (k_s3last<<<nunits, 1024, 0, st>>>(L->in, n, unit, L->last3, L->dsize, L->ov, L->nov)));
            JDPROF_RUN(JDK_CHAINS3, st, (k_s3scan<<<64, 256, 0, st>>>(L->last3, nunits, L->inc3)));
            if (L->nov)
                JDPROF_RUN(JDK_CHAINS3, st, (k_chains<3, true><<<nunits, 1024, 0, st>>>(L->in, n, unit, prev3, nullptr, jd_chains_flag(1),
                                                                                        L->last3, L->dsize, L->ov, L->nov)));
            else
                JDPROF_RUN(JDK_CHAINS3, st, (k_chains<3><<<nunits, 1024, 0, st>>>(L->in, n, unit, prev3, nullptr, jd_chains_flag(1),
                                                                                  L->last3, L->dsize, nullptr, 0)));
        }
        const uint32_t nsub = (uint32_t) ((n + K2_SR - 1) / K2_SR);
        if (L->level >= 8)
            JDPROF_RUN(JDK_MATCH, st, (k_match<true><<<nsub, 1024, 0, st>>>(L->in, n, (uint32_t) n, prev4, prev3,
                                                                            L->rec, lv.chain, lv.nice,
                                                                            lazy ? 3 : 4, lazy ? 1 : 0)));
        else
            JDPROF_RUN(JDK_MATCH, st, (k_match<false><<<nsub, 1024, 0, st>>>(L->in, n, (uint32_t) n, prev4, prev3,
                                                                             L->rec, lv.chain, lv.nice,
                                                                             lazy ? 3 : 4, lazy ? 1 : 0)));
        /* lazy: lists for both doshort values; greedy: doshort plays no part */
        if (hipMemsetD32Async((hipDeviceptr_t) L->dsg, lazy ? 3 : 1, nb, st) != hipSuccess) return -1;
        PSplitArgs ps;
        memset(&ps, 0, sizeof(ps));
        ps.rec = L->rec; ps.prev4 = prev4; ps.in = L->in; ps.n = n; ps.bs = bs;
        ps.nblocks = nb; ps.tokens = L->tokens; ps.dbinfo = L->dbinfo;
        ps.good = lv.good; ps.lzcap = lv.lzcap; ps.nice = lv.nice; ps.half = lv.chain >> 1;
        ps.plist = L->plist; ps.pcount = L->pcount; ps.psync = L->psync; ps.pcap = L->pcap;
        ps.dsg = L->dsg;
        ps.stream = 1; ps.prev3 = prev3; ps.sdb = L->sdb; ps.chain = lv.chain;
        ps.wend = lazy ? 1u << 17 : 1u << 16;          /* kwbits: getmeminfo :210-230 */
        ps.greedy = lazy ? 0 : 1;
        ps.pstart = L->pstart;
        ps.cend = L->cend;
        ps.ncall = L->ncall;
        ps.w0 = L->w0;
        ps.wout = L->wout;
        ps.tailchk = (L->w0.ngen > 0 || n > L->w0.sbase + ps.wend) ? 1u : 0u;
        if (!lazy) ps.good = 4;
        const uint32_t ng = (2 * nb * JD_PSEG + 63) / 64;
        JDPROF_RUN(JDK_PSPEC, st, (k_pspec<true><<<ng, 64, 0, st>>>(ps)));
        JDPROF_RUN(JDK_PSYNC, st, (k_psync<<<ng, 64, 0, st>>>(ps)));
        JDPROF_RUN(JDK_PJOIN, st, (k_pjoin<true><<<1, 64, 0, st>>>(ps)));
        EmitArgs ea;
        memset(&ea, 0, sizeof(ea));
        ea.tokens = L->tokens; ea.dbinfo = L->dbinfo; ea.n = n; ea.bs = bs;
        ea.nblocks = nb; ea.slotcap = 0; ea.level = L->level;
        ea.fixed = L->flags & 1u; ea.lastfinal = 0;
        ea.stage = L->stage; ea.csize = L->bl; ea.sdb = L->sdb;
        JDPROF_RUN(JDK_EMIT, st, (k_emit<<<(uint32_t) maxdb, EM_T, 0, st>>>(ea)));
    }
    JDPROF_RUN(JDK_SCAN, st, (k_sscan<<<1, 1024, 0, st>>>(L->sdb, L->bl, L->bo, L->tslot, final, L->total)));
    JDPROF_RUN(JDK_COMPACT, st, (k_sbits<<<(uint32_t) (maxdb + 1), 256, 0, st>>>(L->sdb, L->stage, L->tslot,
                                                                                 L->bl, L->bo, L->out, L->outcap)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
