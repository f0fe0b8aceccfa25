/*
 * jd_device.h -- shared device-side definitions for the gfx950 deflate /
 * inflate kernels.  Everything here is integer/byte arithmetic; no MFMA.
 *
 * Reference semantics are cited as deflator.c:LINE / inflator.c:LINE
 * (Jpn666/jdeflate 0.4.0).
 */
#ifndef JD_DEVICE_H
#define JD_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

/* Debug build only (make EXTRA=-DJD_BOUNDS): every global access of a
 * caller's buffer near its end is checked against that buffer's end, and a
 * violation is printed (tests/test_bounds.py runs the GPU suite on this
 * build and fails on any such line).  Compiled out of the shipped library. */
#ifdef JD_BOUNDS
#include <stdio.h>
#define JD_CHECK(ptr, width, end)                                                    \
    do {                                                                             \
        if ((uintptr_t) (ptr) + (width) > (uintptr_t) (end))                         \
            printf("JD_BOUNDS %s:%d %p + %u > %p\n", __FILE__, __LINE__,             \
                   (const void*) (ptr), (unsigned) (width), (const void*) (end));    \
    } while (0)
#else
#define JD_CHECK(ptr, width, end) ((void) 0)
#endif

#define JD_MAXBLOCK   65536u   /* independent block size (north_star)       */
#define JD_WSIZE      32768u   /* LZ77 window, deflator.c:30                */
#define JD_MAXMATCH   258u
#define JD_MAXDB      32u      /* deflate blocks per data block (<= 11 used) */
#define JD_EMPTY16    0xffffu

/* per-level parameters, deflator.c:242-263 and getmeminfo :210-230 */
struct JdLevel {
    uint32_t good, nice, chain, lzcap;
};

__host__ __device__ static inline JdLevel jd_level(int level)
{
    switch (level) {
        case 1: return JdLevel{8, 4, 2, 1u << 14};
        case 2: return JdLevel{8, 8, 8, 1u << 15};
        case 3: return JdLevel{8, 16, 16, 1u << 15};
        case 4: return JdLevel{8, 32, 32, 1u << 15};
        case 5: return JdLevel{8, 64, 128, 1u << 15};
        case 6: return JdLevel{16, 16, 48, 1u << 16};
        case 7: return JdLevel{32, 64, 128, 1u << 16};
        case 8: return JdLevel{64, 128, 320, 1u << 17};
        case 9: return JdLevel{192, 256, 512, 1u << 17};
        default: return JdLevel{0, 0, 0, 0};
    }
}

/* RFC 1951 length/distance symbol of a match (getlsymbol :2281,
 * getdsymbol :2237), computed instead of looked up */
__device__ static inline uint32_t jd_lsym(uint32_t len)
{
    uint32_t x = len - 3;
    if (len == 258) return 28;
    if (x < 8) return x;
    uint32_t e = 29 - __builtin_clz(x);       /* floor(log2 x) - 2 */
    return 4 * e + 4 + ((x >> e) & 3);
}

__device__ static inline uint32_t jd_dsym(uint32_t d)
{
    uint32_t x = d - 1;
    if (x < 4) return x;
    uint32_t e = 30 - __builtin_clz(x);       /* floor(log2 x) - 1 */
    return 2 * e + 2 + ((x >> e) & 1);
}

__device__ static inline uint32_t jd_lbase(uint32_t s)
{
    if (s == 28) return 258;
    if (s < 8) return s + 3;
    uint32_t e = (s - 4) >> 2;
    return 3 + ((4 + (s & 3)) << e);
}

__device__ static inline uint32_t jd_lextra(uint32_t s)
{
    return (s < 8 || s == 28) ? 0 : ((s - 4) >> 2);
}

__device__ static inline uint32_t jd_dbase(uint32_t s)
{
    if (s < 4) return s + 1;
    uint32_t e = (s - 2) >> 1;
    return 1 + ((2 + (s & 1)) << e);
}

__device__ static inline uint32_t jd_dextra(uint32_t s)
{
    return s < 4 ? 0 : ((s - 2) >> 1);
}

__device__ static inline uint32_t jd_rev(uint32_t code, uint32_t len)
{
    return __builtin_bitreverse32(code) >> (32 - len);
}

/* fixed Huffman codes, RFC 1951 3.2.6 (slitcodes_ :2987, sdstcodes_ :3094):
 * returns (length << 16) | reversed code */
__device__ static inline uint32_t jd_static_lit(uint32_t s)
{
    if (s < 144) return (8u << 16) | jd_rev(0x30 + s, 8);
    if (s < 256) return (9u << 16) | jd_rev(0x190 + s - 144, 9);
    if (s < 280) return (7u << 16) | jd_rev(s - 256, 7);
    return (8u << 16) | jd_rev(0xc0 + s - 280, 8);
}

__device__ static inline uint32_t jd_static_dist(uint32_t s)
{
    return (5u << 16) | jd_rev(s, 5);
}

/* floor(log2 x), x > 0 (ctb_u32log2, assumed floor) */
__device__ static inline int jd_ilog2(uint32_t x)
{
    return 31 - __builtin_clz(x);
}

/* token encoding between the parser and the emitter */
#define JD_TOK_MATCH 0x80000000u
__device__ static inline uint32_t jd_tok_match(uint32_t len, uint32_t off)
{
    return JD_TOK_MATCH | (len << 16) | off;
}

/* match record written by the match finder for every position:
 *   bits  0- 8  best length with the full chain budget, RAW: not truncated
 *               to the block end (2 = no candidate); the parser applies
 *               the truncation of getmatch2 :2717-2719
 *   bits  9-23  its distance
 *   bits 24-32  best length with half the chain budget (deflator.c:2650), raw
 *   bits 33-47  its distance
 *   bits 48-63  3-byte candidate distance (deflator.c:2676-2711), 0 = none;
 *               written only when the full-budget length is < 3
 */

#endif
