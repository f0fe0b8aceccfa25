/*
 * jd_internal.h -- hooks between the drop-in layers of libjdeflate_amd (not
 * exported): zstrm.c drives deflator.c / inflator.c and needs the CRC-32 /
 * Adler-32 of the bytes they move, which the engine scans on the device copy
 * it already holds (jdgpu_deflate_cs, jdgpu_inflate_resume).
 */
#ifndef JD_INTERNAL_H
#define JD_INTERNAL_H

#include <jdeflate/deflator.h>
#include <jdeflate/inflator.h>

/* *crc / *adler (either NULL) are updated over every byte the instance
 * compresses / delivers from now on (zstrm_crc32update semantics) */
void jd_deflator_checksums(TDeflator*, uint32* crc, uint32* adler);
void jd_inflator_checksums(TInflator*, uint32* crc, uint32* adler);

#endif
