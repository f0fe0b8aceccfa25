/*
 * jdeflate/zstrm.h -- drop-in replacement for the reference's stream
 * container API (Jpn666/jdeflate jdeflate/zstrm.h): raw deflate, zlib
 * (RFC 1950) and gzip (RFC 1952) framing over the MI355X engine, with the
 * CRC-32 / Adler-32 scans on the GPU.  Same enums, same public struct
 * (zstrm.h:104-130), same exported functions.  SURVEY.md §8f row f1.
 *
 * Differences from the reference, all deliberate (DESIGN.md "zstrm"):
 *  - deflate output: 64 KiB independent blocks (the drop-in deflator, which
 *    zstrm drives as the reference's zstrm drives its deflator);
 *  - the zlib header's FCHECK is valid (the reference writes 78 1F,
 *    zstrm.c:1038, which zlib rejects; here 78 01 / 78 20 with FDICT);
 *  - zstrm_crc32combine links (the reference defines crc32_ncombine);
 *  - preset dictionaries (zstrm_setdctnr): inflate uses them as the
 *    reference does; deflate writes FDICT/DICTID but its independent blocks
 *    do not reference the dictionary (valid, not byte-identical);
 *  - usedinput counts the bytes of the container actually consumed;
 *  - an empty stream finalised with zstrm_flush is a complete container.
 */
#ifndef JDEFLATE_ZSTRM_H
#define JDEFLATE_ZSTRM_H

#include <jdeflate/config/config.h>
#include <jdeflate/deflator.h>
#include <jdeflate/inflator.h>

#ifdef __cplusplus
extern "C" {
#endif

/* zstrm.h:37-41 */
typedef enum {
	ZSTRM_INFLATE = 0x00010000,
	ZSTRM_DEFLATE = 0x00020000
} eZSTRMMode;

/* zstrm.h:45-50 */
typedef enum {
	ZSTRM_DFLT = 0x00100000,
	ZSTRM_ZLIB = 0x00200000,
	ZSTRM_GZIP = 0x00400000
} eZSTRMType;

/* zstrm.h:54-62 */
typedef enum {
	ZSTRM_DOCRC   = 0x01000000,
	ZSTRM_DOADLER = 0x02000000,
	ZSTRM_NOCRC   = 0x04000000,
	ZSTRM_NOADLER = 0x08000000
} eZSTRMFlags;

/* zstrm.h:66-80 */
typedef enum {
	ZSTRM_OK            =  0,
	ZSTRM_EIOERROR      =  1,
	ZSTRM_EOOM          =  2,
	ZSTRM_EBADDATA      =  3,
	ZSTRM_ECHECKSUM     =  4,
	ZSTRM_EFORMAT       =  5,
	ZSTRM_EMISSINGDICT  =  6,
	ZSTRM_ESRCEXHSTD    =  7,
	ZSTRM_ETGTEXHSTD    =  8,
	ZSTRM_EDEFLATE      =  9,
	ZSTRM_EBADDICT      = 10,
	ZSTRM_ELIMIT        = 11,
	ZSTRM_EINCORRECTUSE = 12
} eZSTRMError;

/* zstrm.h:84-90 */
typedef enum {
	ZSTRM_NOTSET   = 0,
	ZSTRM_READY    = 1,
	ZSTRM_NEEDDICT = 2,
	ZSTRM_NORMAL   = 3,
	ZSTRM_END      = 4
} eZSTRMState;

/* zstrm.h:96-100 */
typedef intxx (*TZStrmIFn)(      uint8* buffer, uintxx size, void* user);
typedef intxx (*TZStrmOFn)(const uint8* buffer, uintxx size, void* user);

/* zstrm.h:104-130 */
struct TZStrm {
	uint32 state;
	uint32 error;
	uint32 flags;
	uint32 smode;
	uint32 stype;
	 int32 level;
	uintxx total;
	uint32 dictid;
	uint32 dict;
	uint32 crc;
	uint32 adler;
	uintxx usedinput;
};

typedef struct TZStrm TZStrm;

JDEFLATE_API const TZStrm* zstrm_create(uintxx flags, intxx level, const TAllocator*);
JDEFLATE_API void zstrm_destroy(const TZStrm*);
JDEFLATE_API void zstrm_setsource(const TZStrm*, const uint8* source, uintxx size);
JDEFLATE_API void zstrm_setsourcefn(const TZStrm*, TZStrmIFn fn, void* user);
JDEFLATE_API void zstrm_settargetfn(const TZStrm*, TZStrmOFn fn, void* user);
JDEFLATE_API void zstrm_setdctnr(const TZStrm*, const uint8* dict, uintxx size);
JDEFLATE_API uintxx zstrm_inflate(const TZStrm*, void* target, uintxx n);
JDEFLATE_API uintxx zstrm_deflate(const TZStrm*, const void* source, uintxx n);
JDEFLATE_API void zstrm_flush(const TZStrm*, uint32 final);
JDEFLATE_API void zstrm_reset(const TZStrm*);

/* zstrm.h:205-224.  The CRC-32 value is the reflected register without
 * pre/post inversion (a gzip CRC is zstrm_crc32update(0xFFFFFFFF, ...) ^
 * 0xFFFFFFFF); Adler-32 starts at 1.  Inputs of 64 KiB or more are scanned
 * on the GPU (k_checksum), shorter ones (and any input when no gfx950 device
 * is usable: these calls have no error channel) on the host. */
JDEFLATE_API uint32 zstrm_crc32combine(uint32 crc1, uint32 crc2, uintxx size2);
JDEFLATE_API uint32 zstrm_crc32update(uint32 chcksm, const uint8* source, uintxx size);
JDEFLATE_API uint32 zstrm_adler32update(uint32 chcksm, const uint8* source, uintxx size);

#ifdef __cplusplus
}
#endif
#endif
