/*
 * jdeflate/jdgpu.h -- additive independent-block batch API of the MI355X
 * engine (no counterpart in the reference; SURVEY.md §8b "an additive batch
 * API for independent blocks").
 *
 * A stream is cut into blocks of `blocksize` bytes (<= 65536, multiple of
 * 16).  Block i is encoded exactly as the reference encodes it with a fresh
 * deflator (deflator_reset, deflator.c:455) and DEFLT_FLUSH, except the
 * last block of a stream, which uses `lastflush` (DEFLT_END for a complete
 * stream).  The per-block outputs concatenate into one RFC 1951 stream; every
 * block ends byte-aligned with 00 00 FF FF (endstream, deflator.c:610-654),
 * so the block size index (csizes) lets the blocks be inflated in parallel.
 *
 * Return values: 0 (or a byte count) on success, negative JDGPU_E* on error.
 *
 * Devices: every call runs on the HIP device current on the calling thread
 * (hipSetDevice), with that device's own streams and scratch; device
 * buffers passed in must belong to it.
 */
#ifndef JDEFLATE_JDGPU_H
#define JDEFLATE_JDGPU_H

#include <jdeflate/config/config.h>

#ifdef __cplusplus
extern "C" {
#endif

#define JDGPU_EINVAL  (-1)   /* bad argument                              */
#define JDGPU_ENODEV  (-2)   /* no gfx950 device or HIP runtime failure   */
#define JDGPU_EOOM    (-3)   /* device or host allocation failed          */
#define JDGPU_ECAP    (-4)   /* output capacity too small                 */
#define JDGPU_EDATA   (-5)   /* at least one block failed to inflate      */

/* per-block inflate error codes: inflator.h:57-66, plus */
#define JDGPU_EBLOCKOVERFLOW 9   /* a block inflates past `blocksize`    */

/* 1 when a gfx950 device is present and the kernels are loaded */
JDEFLATE_API int jdgpu_available(void);

/* worst-case size of the concatenated output for n input bytes */
JDEFLATE_API uint64 jdgpu_bound(uint64 n, uint32 blocksize);

/*
 * Device-resident deflate.  d_in: n bytes in device memory (16-byte
 * aligned).  d_out: outcap bytes.  d_csizes / d_coffsets: ceil(n/blocksize)
 * (at least 1) entries in device memory, receive each block's compressed
 * size and offset in d_out.  d_total: one uint64 in device memory.
 * `stream` is a hipStream_t (NULL = the engine's stream).  Asynchronous:
 * nothing is synchronised; the caller synchronises the stream.
 */
JDEFLATE_API int jdgpu_deflate_device(const void* d_in, uint64 n, uint32 blocksize,
                                      int level, uint32 flags, int lastflush,
                                      void* d_out, uint64 outcap,
                                      uint32* d_csizes, uint64* d_coffsets,
                                      uint64* d_total, void* stream);

/*
 * Device-resident inflate of nblocks independent blocks (as produced by
 * jdgpu_deflate*): block i is d_in[d_coffsets[i] .. + d_csizes[i]) and
 * decodes into d_out + i*blocksize.  d_usizes / d_errors (device, nblocks)
 * receive the decoded size and error code of each block.  Asynchronous.
 */
JDEFLATE_API int jdgpu_inflate_device(const void* d_in, uint64 inlen,
                                      const uint64* d_coffsets,
                                      const uint32* d_csizes, uint32 nblocks,
                                      uint32 blocksize, void* d_out,
                                      uint32* d_usizes, int32* d_errors,
                                      void* stream);

/*
 * Single-window stream deflate: the output the
 * reference deflator produces when it is given the whole input with one
 * deflator_setsrc and driven with `flush` (DEFLT_END or DEFLT_FLUSH) from a
 * fresh state -- one stream whose LZ77 window slides across the input
 * (deflator.c:1818-1911), not independent blocks.  Levels 0-9.
 * n < 4 GiB - 64 KiB.  d_in 16-byte aligned; outcap >= jdgpu_stream_bound(n).
 * *d_total (device) receives the output size.  Synchronises the stream.
 */
JDEFLATE_API uint64 jdgpu_stream_bound(uint64 n);
/* d_in: dictsize bytes of preset dictionary (deflator_setdctnr, <= 32768;
 * 0 for none) followed by the n input bytes */
JDEFLATE_API int jdgpu_deflate_stream_device(const void* d_in, uint32 dictsize, uint64 n,
                                             int level, uint32 flags, int flush,
                                             void* d_out, uint64 outcap, uint64* d_total,
                                             void* stream);
/* Host-buffer forms: return the compressed size or a negative error.  The
 * _dict form is deflator_setdctnr(dict) on a fresh deflator first (only the
 * last 32 KiB of the dictionary count). */
JDEFLATE_API int64 jdgpu_deflate_stream(const uint8* src, uint64 n, int level,
                                        uint32 flags, int flush, uint8* dst,
                                        uint64 cap);
JDEFLATE_API int64 jdgpu_deflate_stream_dict(const uint8* dict, uint64 dictsize,
                                             const uint8* src, uint64 n, int level,
                                             uint32 flags, int flush, uint8* dst,
                                             uint64 cap);

/*
 * A single-window deflate stream fed in pieces (the drop-in deflator with
 * DEFLT_SINGLEWINDOW; deflator.c:691-786 driven call by call).  Each
 * jdgpu_stream_deflate hands the input since the previous flush: the
 * reference received it in ncalls deflator_deflate calls ending at callends[]
 * (offsets in src, nondecreasing, the last = n; NULL: one call), the last
 * with `flush` (DEFLT_FLUSH or DEFLT_END), the others without a flush.  The
 * output is exactly what those calls write: after a DEFLT_FLUSH the window,
 * hash chains and parser state carry into the next piece (:763-768), the
 * window slides where the reference's does, and the positions whose hashes
 * read past the flush point keep the stale buckets the reference filed them
 * under.  Returns the piece's compressed size or a negative error; after
 * DEFLT_END the stream is closed.  jdgpu_stream_create: level 0-9, flags
 * DEFLT_FIXEDCODES, optional preset dictionary (deflator_setdctnr, last 32 KiB
 * count).
 */
typedef struct JDGPUStream JDGPUStream;
JDEFLATE_API JDGPUStream* jdgpu_stream_create(int level, uint32 flags, const uint8* dict,
                                              uint64 dictsize);
JDEFLATE_API int64 jdgpu_stream_deflate(JDGPUStream* s, const uint8* src, uint64 n,
                                        const uint64* callends, uint32 ncalls, int flush,
                                        uint8* dst, uint64 cap);
JDEFLATE_API void jdgpu_stream_destroy(JDGPUStream* s);

/* Host-buffer deflate: returns the compressed size or a negative error.
 * csizes (host, optional) receives the per-block sizes. */
JDEFLATE_API int64 jdgpu_deflate(const uint8* src, uint64 n, uint32 blocksize,
                                 int level, uint32 flags, int lastflush,
                                 uint8* dst, uint64 cap, uint32* csizes);

/*
 * Several devices from one process (no torch, no launcher).
 * The blocks are cut into contiguous ranges, range k deflated on devs[k]
 * (ndev <= 0 or devs NULL: every visible device); every range but the last
 * ends with FLUSH, the last with `lastflush`, so the result is the
 * single-device stream byte for byte.  The per-device stream lengths are
 * all-gathered over RCCL and the bitstreams gathered to devs[0] by one
 * grouped ncclSend/ncclRecv, into d_out0 (device memory of devs[0], outcap
 * bytes; *total receives the length) or, for jdgpu_deflate_multi, then
 * copied into the host buffer dst (cap bytes; returns the length).  csizes
 * (host, optional) receives the size index.  Synchronous.  RCCL is loaded at
 * the first call (JDGPU_ENODEV without it).
 */
JDEFLATE_API int64 jdgpu_deflate_multi(const uint8* src, uint64 n, uint32 blocksize, int level,
                                       uint32 flags, int lastflush, uint8* dst, uint64 cap,
                                       uint32* csizes, int ndev, const int* devs);
JDEFLATE_API int jdgpu_deflate_multi_device(const uint8* src, uint64 n, uint32 blocksize, int level,
                                            uint32 flags, int lastflush, void* d_out0, uint64 outcap,
                                            uint64* total, uint32* csizes, int ndev, const int* devs);
/* Host-buffer inflate of independent blocks over several devices: block
 * ranges as above, each decoded on its device from the size index (no
 * collective: inflate has no exchange step).  As jdgpu_inflate. */
JDEFLATE_API int jdgpu_inflate_multi(const uint8* src, uint64 srclen, const uint32* csizes,
                                     uint32 nblocks, uint32 blocksize, uint8* dst, uint32* usizes,
                                     int32* errors, int ndev, const int* devs);

/* Host-buffer inflate of independent blocks; returns 0, JDGPU_EDATA when a
 * block failed (see errors[]), or a negative error. */
JDEFLATE_API int jdgpu_inflate(const uint8* src, uint64 srclen,
                               const uint32* csizes, uint32 nblocks,
                               uint32 blocksize, uint8* dst, uint32* usizes,
                               int32* errors);

/* Host-buffer inflate of one arbitrary RFC 1951 stream (no block index):
 * decoded by a single wave; requires a BFINAL block like inflator_inflate.
 * Returns 0 / negative; *error = inflator.h error code (0 = ok),
 * *produced, *consumed = bytes up to the end of the final block. */
JDEFLATE_API int jdgpu_inflate_stream(const uint8* src, uint64 srclen,
                                      uint8* dst, uint64 cap, uint64* produced,
                                      uint64* consumed, int32* error);

/* jdgpu_inflate_stream after inflator_setdctnr(dict) (inflator.c:905-925):
 * back-references may reach into the dictionary's last 32 KiB.  produced
 * counts the stream's own bytes. */
JDEFLATE_API int jdgpu_inflate_stream_dict(const uint8* dict, uint64 dictsize,
                                           const uint8* src, uint64 srclen, uint8* dst,
                                           uint64 cap, uint64* produced, uint64* consumed,
                                           int32* error);

/*
 * Resumable decoder of one RFC 1951 stream (the drop-in inflator's engine,
 * inflator_inflate :765-903).  Between calls the decoder state -- block mode,
 * the current Huffman block's tables, a pending back-reference copy, the
 * stored-block remainder -- and the 32 KiB window stay on the device
 * (decodeblock :1330-1518, copybytes :1214-1290, updatewindow :617-675), and
 * the host keeps only the input bits of an incomplete token or block header.
 * Each call decodes the new input once: src[0, n) continues the stream, the
 * output goes to dst[0, cap) and stops exactly at cap (a back-reference is
 * split, the rest pending).  While the state stands on a byte-aligned block
 * header with >= 128 KiB of input ahead, the input is cut at its 00 00 FF FF
 * sync markers and the verified FLUSH-joined segments are decoded in
 * parallel; everything else is decoded by one wave.  *crc / *adler (NULL:
 * skipped) are updated over the bytes delivered.
 *   status ENDED:     the final block ended; consumed = bytes of src up to
 *                     its last bit (later bytes are not the stream's)
 *   status NEEDINPUT: all of src was taken; more input is needed
 *   status FULL:      dst is full; consumed bytes of src were taken, the
 *                     caller passes the rest (src + consumed) again
 *   status ERROR:     corrupt data, error = inflator.h:57-66 code
 */
typedef struct JDGPUInflateStream JDGPUInflateStream;
enum { JDGPU_IS_ENDED = 0, JDGPU_IS_NEEDINPUT = 1, JDGPU_IS_FULL = 2, JDGPU_IS_ERROR = 3 };
typedef struct {
    uint64 produced;   /* bytes written to dst                              */
    uint64 consumed;   /* bytes of src taken                                */
    int32 status;      /* JDGPU_IS_*                                        */
    int32 error;       /* status ERROR: inflator.h code                     */
    uint32 parallel;   /* segments decoded in parallel by this call         */
    uint32 pad;
} JDGPUInflateStep;
JDEFLATE_API JDGPUInflateStream* jdgpu_istream_create(void);
/* back to a fresh stream; dict (NULL/0: none) = inflator_setdctnr's (the
 * last 32 KiB count) */
JDEFLATE_API int jdgpu_istream_reset(JDGPUInflateStream* s, const uint8* dict, uint64 dictsize);
JDEFLATE_API int jdgpu_istream_inflate(JDGPUInflateStream* s, const uint8* src, uint64 n,
                                       uint8* dst, uint64 cap, JDGPUInflateStep* res,
                                       uint32* crc, uint32* adler);
/* diagnostics: serial launches, segments decoded in parallel, and the input
 * bytes the host carried between calls (each a partial token or header,
 * decoded once the rest arrived) */
JDEFLATE_API int jdgpu_istream_stats(const JDGPUInflateStream* s, uint64* launches,
                                     uint64* parallel, uint64* carried);
/* parallel decode of input without sync markers (on by default): enable
 * 1/0 (-1: unchanged); rounds run and chunks accepted so far */
JDEFLATE_API int jdgpu_istream_fsp(JDGPUInflateStream* s, int enable, uint64* rounds,
                                   uint64* chunks);
/* the span at hand decoded by 64 lanes (k_inflate_rpar; on by default):
 * enable 1/0 (-1: unchanged); its launches so far */
JDEFLATE_API int jdgpu_istream_rpar(JDGPUInflateStream* s, int enable, uint64* launches);
/* 1: the instance launches on a hardware queue of its own (the first 16 live
 * instances of a process), 0: it shares the process's GPU_MAX_HW_QUEUES
 * queues with the other instances past the 16th (their calls then take
 * turns on those queues); negative: invalid instance */
JDEFLATE_API int jdgpu_istream_queue(const JDGPUInflateStream* s);
JDEFLATE_API void jdgpu_istream_destroy(JDGPUInflateStream* s);

/*
 * One-shot decode that starts mid-stream: src continues a stream whose last
 * wlen (<= 32768) decoded bytes are `window`; the first bit0 (< 8) bits of
 * src were consumed earlier (a point the caller got from its own block index
 * or an earlier ENDED result).  Decodes until the final block ends, an
 * error, or the input ends (error INFLT_EINPUTEND), into dst (cap bytes;
 * JDGPU_EBLOCKOVERFLOW when it is too small).  region limits the marker
 * search.  csfrom must be 0.  An input that runs out leaves NO resume point
 * (resumebit = resumeout = 0): the decoder state dies with the call.
 * Resumable decoding across calls is jdgpu_istream_* (above).
 */
typedef struct {
    uint64 produced;   /* bytes written to dst                              */
    uint64 consumed;   /* error 0: bytes of src up to the final block's end */
    uint64 resumebit;  /* error 0: bits of src taken (the stream's end);
                          0 otherwise                                       */
    uint64 resumeout;  /* error 0: = produced; 0 otherwise                  */
    int32 error;       /* 0: final block ended; inflator.h:57-66 code (6 =
                          input ended); JDGPU_EBLOCKOVERFLOW: cap too small */
    uint32 parallel;   /* segments decoded in parallel                      */
} JDGPUInflateResult;

JDEFLATE_API int jdgpu_inflate_resume(const uint8* window, uint32 wlen, const uint8* src,
                                      uint64 srclen, uint64 region, uint32 bit0, uint8* dst,
                                      uint64 cap, JDGPUInflateResult* res, uint64 csfrom,
                                      uint32* crc, uint32* adler);

/* ---- checksums (zstrm semantics) ----------------- */
/*
 * Per-block checksums of n device bytes (d_in 16-byte aligned), blocks of
 * `blocksize` bytes: d_out[3*i] = CRC-32 register of block i from 0 (the
 * reflected register of zstrm_crc32update, no pre/post inversion),
 * d_out[3*i+1] / d_out[3*i+2] = the Adler-32 sums of block i from (0, 0):
 * sum(x) and sum((len - k) * x_k), both mod 65521.  Asynchronous.
 */
JDEFLATE_API int jdgpu_checksum_device(const void* d_in, uint64 n, uint32 blocksize,
                                       uint32* d_out, void* stream);
/* Host buffer: *crc (CRC-32 register) and *adler updated over src[0..n)
 * exactly as zstrm_crc32update / zstrm_adler32update; either may be NULL. */
JDEFLATE_API int jdgpu_checksum(const uint8* src, uint64 n, uint32* crc, uint32* adler);
/* jdgpu_deflate that also updates *crc / *adler (NULL: skipped) over the
 * input, scanned on the device copy. */
JDEFLATE_API int64 jdgpu_deflate_cs(const uint8* src, uint64 n, uint32 blocksize,
                                    int level, uint32 flags, int lastflush,
                                    uint8* dst, uint64 cap, uint32* csizes,
                                    uint32* crc, uint32* adler);
/* jdgpu_inflate_stream that also updates *crc / *adler over the bytes it
 * delivers, scanned where they were decoded. */
JDEFLATE_API int jdgpu_inflate_stream_cs(const uint8* src, uint64 srclen, uint8* dst,
                                         uint64 cap, uint64* produced, uint64* consumed,
                                         int32* error, uint32* crc, uint32* adler);

/*
 * Inflate of one stream that may be FLUSH-joined independent blocks (what
 * jdgpu_deflate and the drop-in deflator write), without an index: src[0 ..
 * region) is searched for the blocks' 00 00 FF FF sync markers and the
 * blocks are decoded in parallel; if the stream is not such a stream (a
 * reference reaches across a marker, a block exceeds 64 KiB, the final
 * block is not last ...) it is decoded serially as by jdgpu_inflate_stream.
 * Either way the result is jdgpu_inflate_stream_cs's.  region = srclen less
 * any container trailer (index-free form).
 */
JDEFLATE_API int jdgpu_inflate_flushed(const uint8* src, uint64 srclen, uint64 region,
                                       uint8* dst, uint64 cap, uint64* produced,
                                       uint64* consumed, int32* error, uint32* crc,
                                       uint32* adler);

/* ---- diagnostics (tests and the benchmark) ---------------------------- */

/* Per-kernel timing with HIP events recorded on each kernel's stream.
 * enable(1) resets the totals; read() fills ms[] / counts[] in kernel-id
 * order: chains4, chains3, match, parse, emit, stored, scan, compact,
 * inflate.  Returns the number of kernel ids. */
JDEFLATE_API int jdgpu_prof_enable(int on);
JDEFLATE_API int jdgpu_prof_read(double* ms, uint64* counts, int n);

/* Run the deflate pipeline on host data (level 1-9, one chunk) and return
 * the parser's tokens (uint32 per position), the deflate-block table
 * (1 + 2*32 uint32 per block) and the match records (uint64 per position). */
JDEFLATE_API int jdgpu_debug_deflate(const uint8* src, uint64 n, uint32 blocksize, int level,
                                     uint32* tokens, uint32* dbinfo, uint64* records);

#ifdef __cplusplus
}
#endif

#endif
