/*
 * jd_check.hip -- gfx950 CRC-32 and Adler-32 of independent blocks
 * (the zstrm container's checksums as parallel
 * per-block scans, combined afterwards).
 *
 * Semantics follow the reference's zstrm_crc32update (zstrm.c:1449-1527:
 * the reflected CRC-32 register, polynomial 0xEDB88320, no pre/post
 * inversion) and zstrm_adler32update (zstrm.c:1347-1405, modulus 65521).
 * Per block b the kernel writes out[3b] = CRC register of the block from 0,
 * and out[3b+1], out[3b+2] = the block's Adler sums from (0, 0):
 *     A_b = sum(x_i) mod 65521,  B_b = sum((L - i) x_i) mod 65521.
 * Running values are combined on the host (jd_crc.c): the CRC register is
 * linear, R(r, D) = shift(r, |D|) ^ R(0, D), with shift by a byte count a
 * product of GF(2) matrices for its set bits (crc32_ncombine :1428-1446);
 * Adler: a += A_b, b += L_b * a_before + B_b.
 *
 * One 256-thread workgroup per block: each thread scans a 16-byte-aligned
 * piece with slice-by-4 tables in LDS (built per workgroup), then the piece
 * CRCs are joined by a tree of shifts and the Adler sums by a weighted sum.
 * HBM-bound: the block is read once (16-byte loads).
 */
#include "jd_device.h"
#include "jd_kernels.h"
#include "jd_prof.h"

#define CK_T 256u

/* GF(2) matrix (column j = image of bit j) times vector */
__device__ static inline uint32_t gf2_times(const uint32_t* m, uint32_t v)
{
    uint32_t r = 0;
#pragma unroll 8
    for (int j = 0; j < 32; j++) r ^= (v >> j) & 1 ? m[j] : 0u;
    return r;
}

/* the CRC register advanced over len zero bytes (sm[k]: 2^k bytes) */
__device__ static inline uint32_t crc_shift(const uint32_t (*sm)[32], uint32_t c, uint32_t len)
{
    for (int k = 0; len; k++, len >>= 1)
        if (len & 1) c = gf2_times(sm[k], c);
    return c;
}

/* one little-endian word: slice-by-4 CRC step, and the Adler sums of its
 * 4 bytes (s += b0..b3 in turn, w += s after each: w gains
 * 4s + 4b0 + 3b1 + 2b2 + b3) */
__device__ static inline void ck_word(const uint32_t (*tab)[256], uint32_t& crc, uint32_t& s,
                                      uint32_t& w, uint32_t x)
{
    const uint32_t c = crc ^ x;
    crc = tab[3][c & 0xff] ^ tab[2][(c >> 8) & 0xff] ^ tab[1][(c >> 16) & 0xff] ^ tab[0][c >> 24];
    w = __builtin_amdgcn_udot4(x, 0x01020304u, w + 4 * s, false);
    s = __builtin_amdgcn_sad_u8(x, 0u, s);
}

__global__ __launch_bounds__(256) void k_checksum(const uint8_t* __restrict__ in, uint64_t n,
                                                  uint32_t bs, const uint32_t* __restrict__ shiftm,
                                                  uint32_t* __restrict__ out)
{
    __shared__ uint32_t tab[4][256];
    __shared__ uint32_t sm[17][32];
    __shared__ uint32_t pc[CK_T];
    __shared__ uint64_t pa[CK_T], pb[CK_T];
    const uint32_t tid = threadIdx.x, b = blockIdx.x;
    const uint64_t base = (uint64_t) b * bs;
    const uint32_t len = (uint32_t) min((uint64_t) bs, n - base);
    const uint8_t* blk = in + base;

    /* this thread's piece: P bytes, a multiple of 16.  A full 256-byte
     * piece (every piece of a 64 KiB block) is loaded into registers before
     * the tables are built, so the HBM latency overlaps the table setup */
    const uint32_t P = ((bs + CK_T - 1) / CK_T + 15) & ~15u;
    const uint32_t p0 = min(len, tid * P), p1 = min(len, p0 + P);
    const bool full = P == 256u && p1 - p0 == 256u;
    uint4 v[16];
    if (full) {
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = *(const uint4*) (blk + p0 + 16 * k);
    }

    /* slice-by-4 tables: tab[0] is the byte table, tab[k][i] advances
     * tab[k-1][i] over one more zero byte */
    {
        uint32_t c = tid;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xedb88320u & (0u - (c & 1)));
        tab[0][tid] = c;
    }
    for (uint32_t i = tid; i < 17 * 32; i += CK_T) sm[i >> 5][i & 31] = shiftm[i];
    __syncthreads();
    for (int k = 1; k < 4; k++) {
        const uint32_t c = tab[k - 1][tid];
        tab[k][tid] = (c >> 8) ^ tab[0][c & 0xff];
        __syncthreads();
    }

    uint32_t crc = 0, s = 0, w = 0;
    uint32_t i = p0;
    if (full) {
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const uint32_t x[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int q = 0; q < 4; q++) ck_word(tab, crc, s, w, x[q]);
        }
        i = p1;
    }
    for (; i + 16 <= p1; i += 16) {
        const uint4 u = *(const uint4*) (blk + i);
        const uint32_t x[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int q = 0; q < 4; q++) ck_word(tab, crc, s, w, x[q]);
    }
    for (; i < p1; i++) {
        const uint32_t x = blk[i];
        crc = (crc >> 8) ^ tab[0][(crc ^ x) & 0xff];
        s += x;
        w += s;
    }
    /* Adler: the piece's weighted sum counts positions to the piece end;
     * every byte of the piece is also weighted by the bytes after it */
    pc[tid] = crc;
    pa[tid] = s;
    pb[tid] = (uint64_t) w + (uint64_t) s * (len - p1);
    __syncthreads();
    /* CRC tree: group g of 2^(l+1) pieces = left half, shifted over the
     * right half's bytes, xor right half */
    for (uint32_t h = 1; h < CK_T; h <<= 1) {
        if ((tid & (2 * h - 1)) == 0) {
            const uint32_t r0 = min(len, (tid + h) * P), r1 = min(len, (tid + 2 * h) * P);
            pc[tid] = crc_shift(sm, pc[tid], r1 - r0) ^ pc[tid + h];
        }
        __syncthreads();
    }
    for (uint32_t h = CK_T / 2; h; h >>= 1) {
        if (tid < h) {
            pa[tid] += pa[tid + h];
            pb[tid] += pb[tid + h];
        }
        __syncthreads();
    }
    if (tid == 0) {
        out[3 * (uint64_t) b] = pc[0];
        out[3 * (uint64_t) b + 1] = (uint32_t) (pa[0] % 65521u);
        out[3 * (uint64_t) b + 2] = (uint32_t) (pb[0] % 65521u);
    }
}

/* ------------------------------------------------------------------------ */
/* Sync markers of FLUSH-joined streams (index-free):
 * every block of a FLUSH-joined stream ends with the byte-aligned empty
 * stored block 00 00 FF FF (endstream, deflator.c:610-654).  For each
 * 64 KiB chunk of the compressed bytes, the offsets just past every
 * 00 00 FF FF whose end is <= region are written in increasing order
 * (cnt[c] = count, 0xFFFFFFFF when more than MK_MAX).  A false match (the
 * pattern inside coded data) only costs the caller its fast path: the block
 * decoder rejects a segment that does not end on a block boundary. */
#define MK_CH  65536u
#define MK_MAX 64u

__global__ __launch_bounds__(256) void k_markers(const uint8_t* __restrict__ in, uint64_t region,
                                                 uint32_t* __restrict__ cnt, uint32_t* __restrict__ off)
{
    __shared__ uint32_t part[256];
    const uint32_t tid = threadIdx.x, c = blockIdx.x;
    const uint64_t s0 = (uint64_t) c * MK_CH + (uint64_t) tid * (MK_CH / 256);
    uint32_t found[4], nf = 0;
    /* pattern start positions s in [s0, s0 + 256) with s + 4 <= region */
    for (uint32_t k = 0; k < MK_CH / 256; k++) {
        const uint64_t st = s0 + k;
        if (st + 4 > region) break;
        if (in[st] == 0 && in[st + 1] == 0 && in[st + 2] == 0xff && in[st + 3] == 0xff) {
            if (nf < 4) found[nf] = (uint32_t) (st + 4);
            nf++;
        }
    }
    part[tid] = nf;
    __syncthreads();
    /* exclusive scan of the per-thread counts */
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t x = tid >= o ? part[tid - o] : 0;
        __syncthreads();
        part[tid] += x;
        __syncthreads();
    }
    const uint32_t tot = part[255], base = part[tid] - nf;
    const bool over = tot > MK_MAX || __syncthreads_or(nf > 4);
    if (!over)
        for (uint32_t k = 0; k < nf; k++) off[(uint64_t) c * MK_MAX + base + k] = found[k];
    if (tid == 0) cnt[c] = over ? 0xffffffffu : tot;
}

extern "C" int jdk_markers_launch(const uint8_t* in, uint64_t region, uint32_t* cnt, uint32_t* off,
                                  void* stream)
{
    hipStream_t st = (hipStream_t) stream;
    const uint64_t nc = (region + MK_CH - 1) / MK_CH;
    if (!nc) return 0;
    k_markers<<<(uint32_t) nc, 256, 0, st>>>(in, region, cnt, off);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int jdk_checksum_launch(const uint8_t* in, uint64_t n, uint32_t bs,
                                   const uint32_t* shiftm, uint32_t* out, void* stream)
{
    hipStream_t st = (hipStream_t) stream;
    const uint64_t nb = n ? (n + bs - 1) / bs : 0;
    if (!nb) return 0;
    if (nb > 0xffffffffull) return -1;
    JDPROF_RUN(JDK_CHECKSUM, st, (k_checksum<<<(uint32_t) nb, CK_T, 0, st>>>(in, n, bs, shiftm, out)));
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
