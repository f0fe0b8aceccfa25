/*
 * jd_kernels.h -- C ABI between the host engine (jd_engine.cpp) and the
 * gfx950 kernels (jd_deflate.hip, jd_inflate.hip).  Plain pointers only.
 */
#ifndef JD_KERNELS_H
#define JD_KERNELS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    const uint8_t* in;      /* device: n bytes, 16-byte aligned          */
    uint64_t n;
    uint32_t bs;            /* block size, multiple of 16, <= 65536      */
    uint32_t nblocks;       /* ceil(n / bs), >= 1                        */
    int level;              /* 0..9                                      */
    uint32_t flags;         /* DEFLT_FIXEDCODES                          */
    uint32_t lastfinal;     /* 1: last block ends with BFINAL=1          */
    uint16_t* chains;       /* device: 5 * nslots + 128 uint16: links,
                               then the slices (jdk_deflate_launch)      */
    uint32_t* tokens;       /* device: nslots uint32                     */
    uint64_t nslots;        /* >= nblocks * bs                           */
    uint64_t* rec;          /* device: nslots records                    */
    uint32_t* dbinfo;       /* device: nblocks * (1 + 2*32)              */
    uint8_t* stage;         /* device: nblocks * slotcap                 */
    uint32_t slotcap;
    uint32_t* csize;        /* device: nblocks                           */
    uint64_t* coff;         /* device: nblocks                           */
    uint64_t* total;        /* device: 1                                 */
    const uint64_t* base;   /* device: offset of this chunk (NULL = 0)   */
    uint8_t* out;           /* device: compacted output (may be NULL)    */
    uint64_t outcap;
    /* split lazy parse (levels 6-9; all NULL: the one-lane-per-block parse) */
    uint64_t* plist;        /* device: nblocks * JD_PSEG * pcap entries   */
    uint32_t* pcount;       /* device: nblocks * JD_PSEG                  */
    uint32_t* psync;        /* device: nblocks * JD_PSEG * 2              */
    uint32_t pcap;          /* entries per segment list                   */
    uint32_t* dsg;          /* device: nblocks doshort guesses (split)    */
    uint32_t* pord;         /* device: 2 * nblocks: k_pspec's block weights
                               and order (split; NULL: launch order)      */
    void* stream;           /* hipStream_t                               */
} JdDeflateLaunch;

/* split lazy parse: segments per block and the positions a segment's
 * speculative walk runs past its end (to meet the next segment's path) */
#ifndef JD_PSEG
#define JD_PSEG    4u
#endif
#define JD_PMARGIN 512u
static inline uint32_t jdk_pcap(uint32_t bs) { return bs / JD_PSEG + JD_PMARGIN + 272u; }

int jdk_deflate_launch(const JdDeflateLaunch* L);
/* bytes of `chains` per slot at a level: 4 (links), 10 (slices) */
uint32_t jdk_chains_bytes(int level);

/* The reference's window buffer (deflator.c:1818-1897) at a parse start or
 * end, in offsets of the launch's buffer: window[0] is at sbase, inputend at
 * inend.  Bytes past inputend are those of earlier generations (before a
 * slide) that no later one overwrote: gb[g] + o for window offset o < gh[g],
 * newest first (each older one filled further), else zero. */
#define JD_NGEN 8
typedef struct {
    uint64_t sbase, inend;
    uint64_t gb[JD_NGEN];
    uint32_t gh[JD_NGEN];
    uint32_t ngen;
    uint32_t ds;            /* doshort (aux6)                              */
    uint32_t err;           /* out: 1 = more than JD_NGEN generations      */
    uint32_t nt, nslide, tailed;    /* out: tokens, slides, tail redone   */
} JdWinState;

/* a position filed under given buckets instead of its own hash (the stale
 * hashes at a mid-stream flush, deflator.c:2646-2648 past inputend); h = ~0:
 * not filed */
typedef struct {
    uint64_t pos;
    uint32_t h4, h3;
} JdOverride;
#define JD_DSZ_NONE 0xffffffffu   /* dsize: no stream-start / dictionary rule */

/* Single-window stream deflate: levels 0-9.  Launch buffer = history, then
 * the segment (the reference fed it in calls ending at cend[], the last with
 * DEFLT_END or DEFLT_FLUSH); the parse starts at pstart.  All device
 * pointers. */
typedef struct {
    const uint8_t* in;      /* n bytes, 16-byte aligned: the dictionary
                               (dsize bytes) then the input              */
    uint64_t n;
    uint32_t dsize;         /* deflator_setdctnr bytes (<= 32768), or
                               JD_DSZ_NONE past the stream start          */
    uint32_t pstart;        /* parse start (dsize in a one-shot stream)    */
    const JdOverride* ov;   /* sorted by pos, nov entries (device)        */
    uint32_t nov;
    const uint32_t* inc3;   /* hash-3 heads before position 0, or NULL     */
    const uint64_t* cend;   /* ncall call ends (device); NULL: one call    */
    uint32_t ncall;
    JdWinState w0;          /* the window at pstart                        */
    JdWinState* wout;       /* device: the window at the end               */
    int level;
    uint32_t flags;         /* DEFLT_FIXEDCODES                           */
    uint32_t final;         /* 1: END (BFINAL on the terminator), 0: FLUSH */
    uint16_t* chains;       /* 2 n                                        */
    uint64_t* rec;          /* n                                          */
    uint32_t* tokens;       /* n                                          */
    uint32_t* last3;        /* units * 16384                              */
    uint64_t* plist;        /* 2 * nblocks * JD_PSEG * pcap               */
    uint32_t* pcount;       /* 2 * nblocks * JD_PSEG                      */
    uint32_t* psync;        /* 2 * nblocks * JD_PSEG * 2                  */
    uint32_t* dsg;          /* nblocks                                    */
    uint32_t pcap;
    uint32_t* dbinfo;       /* unused scratch of DBSTRIDE words           */
    uint32_t* sdb;          /* 1 + 2 * maxdb                              */
    uint8_t* stage;         /* 8 n + 1024 maxdb + 64                      */
    uint32_t* bl;           /* maxdb + 1                                  */
    uint64_t* bo;           /* maxdb + 1                                  */
    uint32_t* tslot;        /* 4                                          */
    uint8_t* out;
    uint64_t outcap;
    uint64_t* total;        /* output bytes                               */
    void* stream;
} JdStreamLaunch;

/* deflate blocks a stream of n bytes can have: every block but the last
 * closes at a check (>= 512 tokens) or on a full token list */
static inline uint64_t jdk_stream_maxdb(uint64_t n) { return n / 512 + 2; }

int jdk_deflate_stream_launch(const JdStreamLaunch* L);

typedef struct {
    const uint8_t* in;      /* device: compressed blocks end to end      */
    uint64_t inlen;         /* bytes readable at `in`                    */
    const uint64_t* coff;   /* device: block start offsets               */
    const uint32_t* csize;  /* device: block compressed sizes            */
    uint32_t nblocks;
    uint32_t bs;            /* output slot per block                     */
    uint8_t* out;           /* device: nblocks * bs                      */
    uint32_t* usize;        /* device: output bytes per block            */
    int32_t* err;           /* device: inflator.h error code per block   */
    uint32_t* used;         /* device: bytes consumed per block (or NULL) */
    uint32_t* fin;          /* device: bit 0 = the block ended on BFINAL, bit 1 =
                               it stopped off a byte boundary (or NULL)  */
    int require_final;      /* 1: a BFINAL block is required (one stream) */
    /* two-phase block-mode scratch (all NULL/0: wave-per-block decoder)   */
    uint64_t* recs;         /* device: chunk * reccap records            */
    uint32_t reccap;        /* records per block                         */
    uint32_t* nrec;         /* device: chunk                             */
    uint8_t* fb;            /* device: chunk fallback flags              */
    uint32_t chunk;         /* blocks per launch chunk                   */
    void* stream;
    /* wave-per-block decoder: output starts at pos0 of the slot, whose first
     * pos0 bytes (a preset dictionary, inflator_setdctnr) back-references
     * may reach; usize counts them too */
    uint32_t pos0;
    /* wave-per-block decoder, resumed streams (inflator_inflate with final=0):
     * the first bit0 (< 8) bits of each block are skipped, and hdr (NULL: not
     * wanted) receives per block the bit position of the last deflate block
     * begun and the output position (pos0 included) at its start */
    uint32_t bit0;
    uint64_t* hdr;
} JdInflateLaunch;

int jdk_inflate_launch(const JdInflateLaunch* L);

/* Resumable single-stream decoder state, kept in device memory between calls
 * of the drop-in inflator: the counterpart of the reference's TInflator
 * private state (inflator.c:39-54: the block mode and final flag, the decode
 * tables of the current Huffman block, the pending copy of decodeblock
 * :1330-1518 / copybytes :1214-1290 and the stored-block remainder of
 * decodestrd :931-1019).  The bit position and the 32 KiB window are the
 * host's (a resume bit offset into the next launch's input; window bytes in
 * front of the output). */
#define JD_RS_LT 1344
#define JD_RS_DT 416
enum { JD_RS_HEADER = 0, JD_RS_HUFF = 1, JD_RS_STORED = 2, JD_RS_ENDED = 3 };
enum { JD_RST_ENDED = 0, JD_RST_NEEDINPUT = 1, JD_RST_FULL = 2, JD_RST_MARKER = 3,
       JD_RST_ERROR = 4 };
typedef struct {
    uint32_t mode;          /* JD_RS_*                                       */
    uint32_t fin;           /* BFINAL of the current block                   */
    uint32_t plen, poff;    /* back-reference bytes still to copy, distance  */
    uint32_t srem;          /* stored bytes still to copy                    */
    uint32_t status;        /* out: JD_RST_*                                 */
    int32_t err;            /* out: inflator.h code when status is ERROR     */
    uint32_t pad;
    uint64_t bit;           /* out: resume bit offset from the input base    */
    uint64_t produced;      /* out: bytes written after the window           */
    uint16_t lt[JD_RS_LT];  /* lit/len table of the current Huffman block    */
    uint16_t dt[JD_RS_DT];  /* distance table                                */
} JdInfState;

typedef struct {
    const uint8_t* in;      /* device: input base, 4-byte aligned            */
    uint64_t bitpos;        /* the bit of `in` to start at                   */
    uint32_t inlen;         /* bytes readable from `in` (< 4 GiB)            */
    uint8_t* out;           /* device: output; out[-pos0, 0) is the window   */
    uint32_t pos0;          /* window bytes in front of out (<= 32768)       */
    uint32_t cap;           /* output bytes this launch may write            */
    uint32_t markmin;       /* > 0: stop at a block header that follows an
                               empty stored block (a 00 00 FF FF sync marker)
                               when at least markmin input bytes remain      */
    uint64_t stopat;        /* also stop (MARKER) at the first block header at
                               or past this bit after bitpos (~0: never)     */
    JdInfState* st;         /* device: state in/out                          */
    void* stream;
    uint32_t stopcopy;      /* 1: stop (FULL) once a pending copy is done, so
                               the parallel resume takes the rest            */
    JdInfState* hhead;      /* host-pinned (or NULL): the state's head
                               (mode .. produced) written there as well, so
                               the host needs no copy back after the launch  */
} JdResumeLaunch;

int jdk_inflate_resume_launch(const JdResumeLaunch* L);

/* Parallel resume (k_inflate_rpar): the resumable decoder's work for the span
 * at hand done by 64 lanes (self-synchronising walks, as k_inflate_par), from
 * a state with no pending copy and not inside a stored block.  Output goes to
 * out[0, produced) (at most min(cap, JD_RP_OUT) bytes); the state is left at
 * a point the serial decoder (k_inflate_resume) can continue from:
 *   ENDED      the final block ended;
 *   NEEDINPUT  the span's end: a token, header or stored block it cut;
 *   FULL       the output room (at a token boundary, < 258 bytes short of it
 *              at most, or at a span start when the record scratch is full);
 *   SERIAL     no way on in parallel from the state (a flat literal code, an
 *              error on the true path, ...): the serial decoder takes the next
 *              block.  Earlier blocks of the launch are kept. */
#ifndef JD_RP_OUT
#define JD_RP_OUT    65536u
#endif
#define JD_RP_MAXREC 32768u
enum { JD_RST_SERIAL = 5 };
typedef struct {
    const uint8_t* in;      /* device: span input, 16-byte aligned           */
    uint32_t bitpos;        /* the bit of `in` to start at                   */
    uint32_t inlen;         /* bytes of input (< 512 MiB)                    */
    const uint8_t* win;     /* device: the 32 KiB in front of out            */
    uint8_t* out;           /* device: output, 16-byte aligned (+16 slack)   */
    uint32_t pos0;          /* valid window bytes (<= 32768)                 */
    uint32_t cap;           /* output room                                   */
    uint64_t* recs;         /* device: JD_RP_MAXREC records of scratch       */
    JdInfState* st;         /* device: state in/out                          */
    /* stop (MARKER) at a block header after the first one reached, when
     * the input from there -- inlen plus `extra` bytes beyond -- is at
     * least markmin (headers after an empty stored block: the block-parallel
     * prefix) or hdrmin (any header: the chunk-parallel rounds); 0 = never */
    uint32_t markmin, hdrmin;
    uint64_t extra;
    void* stream;
    JdInfState* hhead;      /* host-pinned (or NULL): as JdResumeLaunch      */
} JdRparLaunch;

int jdk_inflate_rpar_launch(const JdRparLaunch* L);

/* Parallel decode of a stream without sync markers (zlib's default output,
 * Z_SYNC_FLUSH at arbitrary points).  The input from bit0 is cut into search
 * regions of `span` bytes; in each region but the first, k_fsp_find looks
 * for the first bit at which a dynamic-Huffman block header passes every
 * check the decoder applies (decodednmc :1104-1190, readlengths :1030-1101,
 * buildtable :424-474).  k_fsp_decode then decodes every chunk -- from its
 * start to the next chunk's start -- on one wave, independently: output
 * entries are u16, a byte or a marker 0x100 + w for the byte at distance
 * 32768 - w before the chunk's start.  Chunk c is exact when chunk c-1
 * (exact by induction from bit0) ended a block exactly at chunk c's start;
 * the host accepts chunks in that order, then k_fsp_window carries the 32 KiB
 * window across the accepted chunks and k_fsp_resolve replaces the markers. */
enum { JD_FSP_REACHED = 0,  /* a block ended exactly at the next start      */
       JD_FSP_PASSED = 1,   /* a block ended past it (lb): the start was false */
       JD_FSP_ENDED = 2,    /* the BFINAL block ended at lb                 */
       JD_FSP_STOPPED = 3,  /* error, input end or output cap: lb = the last
                               block start reached                           */
       JD_FSP_NONE = 4 };   /* no start found in this region                */
typedef struct {
    const uint8_t* in;      /* device: input base, 16-byte aligned           */
    uint64_t inlen;         /* bytes the decoders may read (<= 4 GiB)        */
    uint64_t bit0;          /* chunk 0 starts here: a block header           */
    uint64_t endbit;        /* searches stop here                            */
    uint32_t nchunk;
    uint32_t span;          /* bytes per search region                       */
    uint64_t* starts;       /* device: nchunk; [c] = chunk c's start or ~0   */
    uint16_t* o16;          /* device: nchunk * ocap entries                 */
    uint32_t ocap;          /* entries per chunk, multiple of 4096           */
    uint32_t wlen;          /* window bytes valid before chunk 0             */
    uint64_t* res;          /* device: nchunk * 4: status, lb, lo (entries
                               at lb), entries written                       */
    void* stream;
} JdFspLaunch;

typedef struct {
    const uint16_t* o16;    /* device: JdFspLaunch.o16                       */
    uint32_t ocap;
    uint32_t npiece;        /* accepted chunks                               */
    const uint64_t* piece;  /* device: npiece * 4: chunk, bytes, output
                               offset, window bytes valid before it          */
    uint32_t maxlen;        /* largest piece                                 */
    uint8_t* win;           /* device: (npiece + 1) * 32768; [0] = the window
                               before chunk 0 (set by the caller)           */
    uint8_t* out;
    uint32_t* flag;         /* device: 1 + npiece words; [0] set to 1 if a
                               marker reaches before the stream's first byte
                               (E_FAROFFSET), the rest scratch               */
    void* stream;
} JdFspResolve;

int jdk_fsp_decode_launch(const JdFspLaunch* L);
int jdk_fsp_resolve_launch(const JdFspResolve* R);

#ifdef __cplusplus
}
#endif
#endif
