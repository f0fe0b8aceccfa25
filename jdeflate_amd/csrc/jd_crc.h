/*
 * jd_crc.h -- host checksum algebra shared by the engine and zstrm.c
 * (internal; not installed).
 */
#ifndef JD_CRC_H
#define JD_CRC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 64 matrices of 32 columns: advancing the CRC register over 2^i zero bytes */
const uint32_t* jdcrc_zero_matrices(void);
/* the CRC register advanced over len zero bytes */
uint32_t jdcrc_shift(uint32_t crc, uint64_t len);
/* running values updated with the per-block triples of k_checksum
 * (crc, A, B per block of bs bytes over n bytes) */
uint32_t jdcrc_join(uint32_t crc, const uint32_t* blocks, uint64_t n, uint32_t bs);
uint32_t jdadler_join(uint32_t adler, const uint32_t* blocks, uint64_t n, uint32_t bs);
/* the same updates scanned on the host (short inputs) */
uint32_t jdcrc_bytes(uint32_t crc, const uint8_t* p, uint64_t n);
uint32_t jdadler_bytes(uint32_t adler, const uint8_t* p, uint64_t n);

/* jd_check.hip */
int jdk_checksum_launch(const uint8_t* in, uint64_t n, uint32_t bs,
                        const uint32_t* shiftm, uint32_t* out, void* stream);

/* jd_check.hip: offsets past each 00 00 FF FF (<= region), per 64 KiB chunk */
#define JD_MK_CH  65536u
#define JD_MK_MAX 64u
int jdk_markers_launch(const uint8_t* in, uint64_t region, uint32_t* cnt, uint32_t* off,
                       void* stream);

#ifdef __cplusplus
}
#endif
#endif
