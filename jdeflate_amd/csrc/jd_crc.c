/*
 * jd_crc.c -- host-side checksum algebra for combining per-block values
 * (no data passes through here: the bytes are scanned on the GPU by
 * k_checksum, jd_check.hip).
 *
 * The CRC-32 register of the reference (zstrm_crc32update, zstrm.c:1449;
 * reflected, polynomial 0xEDB88320, no pre/post inversion) is linear over
 * GF(2): advancing it over k zero bytes is a 32x32 matrix, and
 *     R(r, A || B) = Z(|B|) R(r, A) ^ R(0, B).
 * Z(2^i) are built by repeated squaring of the one-byte operator; Z(len) is
 * the product of those for the set bits of len, as crc32_ncombine does with
 * its precomputed crc32_combinetable (zstrm.c:1411-1446).
 */
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <jdeflate/config/config.h>
#include "jd_crc.h"

static uint32_t zmat[64][32];            /* zmat[i]: 2^i zero bytes */
static pthread_once_t zonce = PTHREAD_ONCE_INIT;
static uint32_t btab[256];               /* the register over one byte  */

static uint32_t gf2_times(const uint32_t* m, uint32_t v)
{
    uint32_t r = 0;
    int j;
    for (j = 0; v; j++, v >>= 1)
        if (v & 1) r ^= m[j];
    return r;
}

static void gf2_square(uint32_t* dst, const uint32_t* m)
{
    int j;
    for (j = 0; j < 32; j++) dst[j] = gf2_times(m, m[j]);
}

static void zinit(void)
{
    uint32_t one[32];
    int j, k, i;
    /* one zero byte: eight steps of the reflected shift register */
    for (j = 0; j < 32; j++) {
        uint32_t c = 1u << j;
        for (k = 0; k < 8; k++) c = (c >> 1) ^ (0xedb88320u & (0u - (c & 1)));
        one[j] = c;
    }
    memcpy(zmat[0], one, sizeof one);
    for (i = 1; i < 64; i++) gf2_square(zmat[i], zmat[i - 1]);
    for (j = 0; j < 256; j++) btab[j] = gf2_times(one, (uint32_t) j);
}

/* Short inputs (and the utility entry points without a device) are scanned
 * here, a byte at a time: a device round trip costs more than the scan below
 * ~64 KiB.  Bulk data goes through k_checksum. */
uint32_t jdcrc_bytes(uint32_t crc, const uint8_t* p, uint64_t n)
{
    uint64_t i;
    pthread_once(&zonce, zinit);
    for (i = 0; i < n; i++) crc = (crc >> 8) ^ btab[(crc ^ p[i]) & 0xffu];
    return crc;
}

uint32_t jdadler_bytes(uint32_t adler, const uint8_t* p, uint64_t n)
{
    uint32_t a = adler & 0xffffu, s = adler >> 16;
    while (n) {
        /* 5552 bytes keep s below 2^32 before the reduction (RFC 1950) */
        uint64_t k = n < 5552 ? n : 5552;
        n -= k;
        while (k--) {
            a += *p++;
            s += a;
        }
        a %= 65521u;
        s %= 65521u;
    }
    return (s << 16) | a;
}

const uint32_t* jdcrc_zero_matrices(void)
{
    pthread_once(&zonce, zinit);
    return &zmat[0][0];
}

uint32_t jdcrc_shift(uint32_t crc, uint64_t len)
{
    int i;
    pthread_once(&zonce, zinit);
    for (i = 0; len; i++, len >>= 1)
        if (len & 1) crc = gf2_times(zmat[i], crc);
    return crc;
}

uint32_t jdcrc_join(uint32_t crc, const uint32_t* blocks, uint64_t n, uint32_t bs)
{
    uint64_t b, nb = n ? (n + bs - 1) / bs : 0;
    for (b = 0; b < nb; b++) {
        const uint64_t len = n - b * bs < bs ? n - b * bs : bs;
        crc = jdcrc_shift(crc, len) ^ blocks[3 * b];
    }
    return crc;
}

uint32_t jdadler_join(uint32_t adler, const uint32_t* blocks, uint64_t n, uint32_t bs)
{
    uint64_t a = adler & 0xffffu, s = adler >> 16, b, nb = n ? (n + bs - 1) / bs : 0;
    for (b = 0; b < nb; b++) {
        const uint64_t len = n - b * bs < bs ? n - b * bs : bs;
        s = (s + (len % 65521u) * a + blocks[3 * b + 2]) % 65521u;
        a = (a + blocks[3 * b + 1]) % 65521u;
    }
    return (uint32_t) ((s << 16) | a);
}

/* zstrm.h: the declared combine (the reference defines it under the name
 * crc32_ncombine, zstrm.c:1428, so the declared symbol does not link there;
 * SURVEY.md §8f).  crc1 advanced over size2 bytes, xor crc2. */
JDEFLATE_API uint32 zstrm_crc32combine(uint32 crc1, uint32 crc2, uintxx size2)
{
    return jdcrc_shift(crc1, (uint64_t) size2) ^ crc2;
}
