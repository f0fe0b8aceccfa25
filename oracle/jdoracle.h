/*
 * jdoracle.h -- CPU restatement of the jdeflate reference codec.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the
 * checker / the timed CPU baseline.  The product (libjdeflate_amd.so) never
 * links or calls it.
 *
 * Parity status: PARTIALLY PINNED.  The reference (Jpn666/jdeflate) cannot be
 * built in this image (it needs the un-vendored ctoolbox library and a
 * meson-generated config.h), so this restatement is pinned by the known
 * answers SURVEY.md recorded from the reference, by RFC 1951 conformance
 * (Python zlib inflates every output; zlib-produced streams inflate to their
 * source) and by internal consistency -- not by reference outputs.
 * See DESIGN.md "Oracle".
 */
#ifndef JDORACLE_H
#define JDORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* result codes mirror jdeflate/deflator.h:48-53 and inflator.h:48-53 */
enum { JDO_OK = 0, JDO_SRCEXHSTD = 1, JDO_TGTEXHSTD = 2, JDO_ERROR = 3 };
/* flush modes mirror deflator.h:57-61 */
enum { JDO_NOFLUSH = 0, JDO_END = 1, JDO_FLUSH = 2 };
/* flags mirror deflator.h:74-76 */
enum { JDO_FIXEDCODES = 1 };

/*
 * One-shot deflate with a fresh deflator (deflator_create + deflator_reset),
 * the whole input given at once, flush = JDO_END or JDO_FLUSH.  Equivalent to
 *   deflator_setsrc(src, n); do { settgt; deflator_deflate(flush) } while TGTEXHSTD
 * in the reference (output is independent of target chunking).
 * Returns the number of bytes written, or (size_t)-1 if cap is too small or
 * the arguments are invalid.  The input may be of any length (the window
 * slides exactly as deflator.c:1818-1897 does).
 */
size_t jdo_deflate(const uint8_t* src, size_t n, int level, unsigned flags,
                   int flush, uint8_t* dst, size_t cap);

/* deflator_setdctnr(dict, dsize) on a fresh deflator, then as jdo_deflate */
size_t jdo_deflate_dict(const uint8_t* dict, size_t dsize, const uint8_t* src, size_t n,
                        int level, unsigned flags, int flush, uint8_t* dst, size_t cap);

/*
 * A sequence of deflator_deflate calls on one deflator (single-window mode,
 * after an optional deflator_setdctnr): call k hands src[ends[k-1], ends[k])
 * (ends[-1] = 0) with flush mode flushes[k] (JDO_NOFLUSH, JDO_FLUSH or
 * JDO_END).  The window, chains and parser state carry across calls; every
 * JDO_FLUSH ends with the byte-aligned empty stored block and keeps the
 * window (deflator.c:763-768).  Returns the total of all outputs, or
 * (size_t)-1.
 */
size_t jdo_deflate_calls(const uint8_t* dict, size_t dsize, const uint8_t* src,
                         const size_t* ends, const int* flushes, size_t ncalls,
                         int level, unsigned flags, uint8_t* dst, size_t cap);

/*
 * Independent-block deflate: input cut into blocks of `blocksize` bytes, each
 * compressed by a fresh deflator with JDO_FLUSH (JDO_END for the last block).
 * The concatenation is one RFC 1951 stream.  sizes[i] receives the compressed
 * size of block i.  Returns the total, or (size_t)-1.
 */
size_t jdo_deflate_blocks(const uint8_t* src, size_t n, size_t blocksize,
                          int level, unsigned flags, uint8_t* dst, size_t cap,
                          uint32_t* sizes);

/* worst-case compressed size of an n-byte block (any level) */
size_t jdo_bound(size_t n);

/*
 * Token trace of the level 6-9 / 1-5 parser for a single fresh block of input
 * (END).  Each token is written as uint32: literal = byte value,
 * match = 0x80000000 | (length << 16) | distance, block end = 0x40000000 |
 * blocktype(1 static, 2 dynamic).  Returns the number of entries written
 * (truncated to cap).
 */
size_t jdo_trace(const uint8_t* src, size_t n, int level, unsigned flags,
                 uint32_t* out, size_t cap);

/*
 * One-shot inflate of a raw RFC 1951 stream (inflator_inflate with final=1
 * and a target of `cap` bytes).  Returns JDO_OK, JDO_TGTEXHSTD (cap too
 * small) or JDO_ERROR with *error set to the inflator.h:57-66 code.
 * *produced = output bytes, *consumed = input bytes up to the byte holding
 * the last bit of the final block.
 */
int jdo_inflate(const uint8_t* src, size_t n, uint8_t* dst, size_t cap,
                size_t* consumed, size_t* produced, int* error);

/*
 * Independent-block inflate: nblocks compressed blocks laid end to end with
 * their compressed sizes in csizes[]; block i decodes into
 * dst + i*blocksize.  Each block is decoded by a fresh inflator until its
 * last byte; the block-end terminator (empty stored block) is consumed like
 * any block.  usizes[i] receives the output size, errors[i] the error code
 * (0 = ok; 9 = the block inflates past blocksize, as in jdgpu.h).
 * Returns the number of failing blocks.
 */
int jdo_inflate_blocks(const uint8_t* src, const uint32_t* csizes,
                       size_t nblocks, size_t blocksize, uint8_t* dst,
                       uint32_t* usizes, int32_t* errors);

/* multithreaded independent-block helpers for the CPU baseline (pthreads) */
size_t jdo_deflate_blocks_mt(const uint8_t* src, size_t n, size_t blocksize,
                             int level, uint8_t* dst, size_t slotcap,
                             uint32_t* sizes, int threads);
int jdo_inflate_blocks_mt(const uint8_t* src, const uint64_t* coffsets,
                          const uint32_t* csizes, size_t nblocks,
                          size_t blocksize, uint8_t* dst, int threads);

#ifdef __cplusplus
}
#endif
#endif
