/*
 * jd_engine.cpp -- host side of the MI355X engine: device context, stream,
 * workspace, chunking, and the C ABI of jdeflate/jdgpu.h.
 *
 * One process-wide engine (lazy, thread-safe).  Workspace for a deflate
 * chunk of B blocks of `bs` bytes:
 *   chains 10 B/position  hash-4 + hash-3 links, slices S (2 B) + W (4 B)
 *   tokens  4 B/position  parser output
 *   rec     8 B/position  match records
 *   stage   slotcap/block per-block bitstreams before concatenation
 * A chunk is at most JD_CHUNK_BLOCKS blocks (1 GiB of input at 64 KiB),
 * i.e. ~18.5 GiB of HBM; larger inputs run chunk after chunk on the stream,
 * with the output offset carried on the device (no host synchronisation).
 */
#include <hip/hip_runtime.h>

#include <jdeflate/jdgpu.h>

#include <atomic>
#include <cstddef>
#include <mutex>
#include <new>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "jd_crc.h"
#include "jd_kernels.h"
#include "jd_prof.h"

#include <vector>

/* ---- per-kernel event timing (jd_prof.h) ---- */
namespace {
/* Event-pair slots with a free list: a slot is open from jdprof_begin to
 * jdprof_end, then ended until a drain adds its time and frees it, so a
 * drain never waits for (or skips) launches other threads have in flight
 * between their begin and end. */
struct Prof {
    std::mutex mu;
    int on = 0;
    std::vector<hipEvent_t> pool;       /* 2 events per slot                 */
    std::vector<int> kid;
    std::vector<char> st;               /* 0 free, 1 open, 2 ended          */
    std::vector<int> freel;
    double ms[JDK_COUNT] = {0};
    uint64_t cnt[JDK_COUNT] = {0};
};
Prof& prof() { static Prof p; return p; }

/* caller holds p.mu: add up and free every ended slot */
void prof_drain(Prof& p)
{
    for (size_t i = 0; i < p.st.size(); i++) {
        if (p.st[i] != 2) continue;
        float ms = 0;
        if (hipEventSynchronize(p.pool[2 * i + 1]) == hipSuccess &&
            hipEventElapsedTime(&ms, p.pool[2 * i], p.pool[2 * i + 1]) == hipSuccess) {
            p.ms[p.kid[i]] += ms;
            p.cnt[p.kid[i]] += 1;
        }
        p.st[i] = 0;
        p.freel.push_back((int) i);
    }
}
}  // namespace

extern "C" int jdprof_on(void) { return prof().on; }

extern "C" int jdprof_begin(int k, hipStream_t st, int* slot)
{
    Prof& p = prof();
    std::lock_guard<std::mutex> g(p.mu);
    if (p.freel.empty()) prof_drain(p);
    if (p.freel.empty()) return 0;      /* every slot open: not timed */
    const int i = p.freel.back();
    if (hipEventRecord(p.pool[2 * (size_t) i], st) != hipSuccess) return 0;
    p.freel.pop_back();
    p.kid[i] = k;
    p.st[i] = 1;
    *slot = i;
    return 1;
}

extern "C" void jdprof_end(int slot, hipStream_t st)
{
    Prof& p = prof();
    std::lock_guard<std::mutex> g(p.mu);
    /* a failed end record frees the slot untimed */
    if (hipEventRecord(p.pool[2 * (size_t) slot + 1], st) == hipSuccess) {
        p.st[slot] = 2;
    } else {
        p.st[slot] = 0;
        p.freel.push_back(slot);
    }
}

/* enable (1) / disable (0) kernel timing; resets the totals (launches still
 * open at the reset are counted after it) */
extern "C" JDEFLATE_API int jdgpu_prof_enable(int on)
{
    Prof& p = prof();
    std::lock_guard<std::mutex> g(p.mu);
    if (on && p.pool.empty()) {
        const size_t ns = 1024;
        p.pool.resize(2 * ns);
        for (auto& ev : p.pool)
            if (hipEventCreate(&ev) != hipSuccess) {
                p.pool.clear();
                return -1;
            }
        p.kid.assign(ns, 0);
        p.st.assign(ns, 0);
        for (size_t i = ns; i-- > 0;) p.freel.push_back((int) i);
    }
    prof_drain(p);
    for (int i = 0; i < JDK_COUNT; i++) { p.ms[i] = 0; p.cnt[i] = 0; }
    p.on = on;
    return 0;
}

/* total milliseconds and launch count per kernel id (jd_prof.h order) */
extern "C" JDEFLATE_API int jdgpu_prof_read(double* ms, uint64* counts, int n)
{
    Prof& p = prof();
    std::lock_guard<std::mutex> g(p.mu);
    prof_drain(p);
    for (int i = 0; i < n && i < JDK_COUNT; i++) { ms[i] = p.ms[i]; counts[i] = p.cnt[i]; }
    return JDK_COUNT;
}

#define JD_CHUNK_BLOCKS 16384u
#define JD_DBSTRIDE (1 + 2 * 32)

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    bool ensure(size_t n)
    {
        if (n <= cap) return true;
        if (p) (void) hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, n) != hipSuccess) { p = nullptr; return false; }
        cap = n;
        return true;
    }
    void release()
    {
        if (p) (void) hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T* as() const { return (T*) p; }
};

/* deflate workspace for one launch chunk */
struct DScratch {
    DevBuf chains, tokens, rec, stage, dbinfo;
    DevBuf plist, pcount, psync, dsg, pord;           /* split lazy parse */
};

/* two-phase inflate workspace for one launch chunk */
struct IScratch {
    DevBuf irec, inrec, ifb;
};

/* single-window stream workspace */
struct SScratch {
    DevBuf chains, rec, tokens, last3, plist, pcount, psync, dsg, dbinfo;
    DevBuf sdb, stage, bl, bo, tslot, total;
    DevBuf win, ov, cend;                             /* carried stream state */
};

struct Engine {
    std::mutex mu;
    SScratch ss;
    int state = 0;          /* 0 untried, 1 ready, -1 unavailable */
    hipStream_t stream = nullptr;
    DScratch ds;
    IScratch is;
    DevBuf csize, coff, total, zero;
    DevBuf hin, hout, hsz, hoff, hus, herr, hused;   /* host-API staging */
    DevBuf shiftm, ck;                                /* checksums         */
    DevBuf mk, fin, hhdr;                             /* one-stream decode */
    DevBuf fo16, fres, fstart, fwin, fpiece, fflag;   /* marker-free streams */
    std::vector<uint32_t> hck;
    /* the workspace is engine-global, so work enqueued on one stream waits
     * for the last work enqueued on another (see order / mark) */
    hipEvent_t evlast = nullptr;
    hipStream_t lastst = nullptr;
    bool haslast = false;
};

/* one engine (streams, scratch) per device: calls go to the engine of the
 * device current on the calling thread, as HIP's own calls do */
#define JD_MAXDEV 64
Engine& eng()
{
    static Engine e[JD_MAXDEV];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= JD_MAXDEV) dev = 0;
    return e[dev];
}

/* caller holds the lock */
bool ready(Engine& e)
{
    if (e.state) return e.state > 0;
    e.state = -1;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return false;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    hipDeviceProp_t pr;
    if (hipGetDeviceProperties(&pr, dev) != hipSuccess) return false;
    if (strncmp(pr.gcnArchName, "gfx950", 6) != 0) return false;
    if (hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&e.evlast, hipEventDisableTiming) != hipSuccess) return false;
    if (!e.zero.ensure(64)) return false;
    if (hipMemset(e.zero.p, 0, 64) != hipSuccess) return false;
    /* k_checksum's zero-byte operators for 2^0 .. 2^16 bytes */
    if (!e.shiftm.ensure(17 * 32 * 4)) return false;
    if (hipMemcpy(e.shiftm.p, jdcrc_zero_matrices(), 17 * 32 * 4, hipMemcpyHostToDevice) != hipSuccess)
        return false;
    e.state = 1;
    return true;
}

/* Callers may pass any stream to the asynchronous entry points, but the
 * scratch buffers are shared: before enqueueing on `st`, wait for the last
 * work the engine enqueued on another stream; afterwards record it.  (The
 * caller holds the lock.) */
void order(Engine& e, hipStream_t st)
{
    if (e.haslast && e.lastst != st) (void) hipStreamWaitEvent(st, e.evlast, 0);
}

void mark(Engine& e, hipStream_t st)
{
    if (hipEventRecord(e.evlast, st) == hipSuccess) {
        e.haslast = true;
        e.lastst = st;
    }
}

/* the synchronous host paths: mark the stream when the entry point returns,
 * after everything it enqueued on every exit path */
struct Fence {
    Engine& e;
    hipStream_t st;
    Fence(Engine& e_, hipStream_t s_) : e(e_), st(s_) {}
    ~Fence() { mark(e, st); }
};

uint32_t slotcap_for(uint32_t bs)
{
    /* worst case is ~1.34x plus trees; 2x + 1 KiB never overflows */
    return ((2u * bs + 1024u) + 255u) & ~255u;
}

bool valid_bs(uint32_t bs) { return bs >= 16 && bs <= 65536 && (bs & 15) == 0; }

/* Scratch for the two-phase block-mode inflate (k_inflate_par /
 * k_inflate_resolve): per block up to bs/4 + 64 records (8 B each); a block
 * that needs more is decoded by the wave-per-block kernel instead.  Blocks
 * are processed in chunks of JD_CHUNK_BLOCKS.  Leaves L untouched (the
 * wave-per-block path) when the slots are not 16-byte blocks. */
void inflate_scratch(Engine& e, JdInflateLaunch& L)
{
    if (L.require_final || L.bs > 65536 || (L.bs & 15) || ((uintptr_t) L.out & 15)) return;
    const uint32_t ch = L.nblocks < JD_CHUNK_BLOCKS ? L.nblocks : JD_CHUNK_BLOCKS;
    uint32_t rc = L.bs / 4 + 64;
    const char* rcenv = getenv("JD_INFLATE_RECCAP");   /* tests: force the fallback path */
    if (rcenv && atoi(rcenv) > 0) rc = (uint32_t) atoi(rcenv);
    IScratch& x = e.is;
    if (!x.irec.ensure((uint64_t) ch * rc * 8 + 64) || !x.inrec.ensure((uint64_t) ch * 4 + 64) ||
        !x.ifb.ensure((uint64_t) ch + 64))
        return;
    L.recs = x.irec.as<uint64_t>();
    L.reccap = rc;
    L.nrec = x.inrec.as<uint32_t>();
    L.fb = x.ifb.as<uint8_t>();
    L.chunk = ch;
}

/* deflate workspace for chunks of up to cb blocks */
int dscratch(DScratch& x, uint32_t cb, uint32_t bs, int level, bool split)
{
    const uint64_t slots = (uint64_t) cb * bs;
    if (level) {
        /* prev4 + prev3 links, then the slices S (+16 entries of padding)
         * and W (jdk_deflate_launch) */
        if (!x.chains.ensure(slots * jdk_chains_bytes(level) + 256)) return JDGPU_EOOM;
        if (!x.tokens.ensure(slots * 4 + 64)) return JDGPU_EOOM;
        if (!x.rec.ensure(slots * 8 + 64)) return JDGPU_EOOM;
    }
    const uint32_t pcap = jdk_pcap(bs);
    if (split) {
        if (!x.plist.ensure((uint64_t) cb * 2 * JD_PSEG * pcap * 8 + 64) ||
            !x.pcount.ensure((uint64_t) cb * 2 * JD_PSEG * 4 + 64) ||
            !x.psync.ensure((uint64_t) cb * 2 * JD_PSEG * 8 + 64) ||
            !x.dsg.ensure((uint64_t) cb * 4 + 64) || !x.pord.ensure((uint64_t) cb * 8 + 64))
            return JDGPU_EOOM;
    }
    if (!x.stage.ensure((uint64_t) cb * slotcap_for(bs) + 256)) return JDGPU_EOOM;
    if (!x.dbinfo.ensure((uint64_t) cb * JD_DBSTRIDE * 4)) return JDGPU_EOOM;
    return 0;
}

/* deflate a device-resident input in launch chunks of up to
 * JD_CHUNK_BLOCKS blocks; caller holds the lock */
int deflate_dev(Engine& e, const uint8_t* d_in, uint64_t n, uint32_t bs, int level,
                uint32_t flags, int lastflush, uint8_t* d_out, uint64_t outcap,
                uint32_t* d_csizes, uint64_t* d_coffs, uint64_t* d_total, hipStream_t st)
{
    if (!valid_bs(bs) || level < 0 || level > 9) return JDGPU_EINVAL;
    if (lastflush != 1 && lastflush != 2) return JDGPU_EINVAL;
    if (((uintptr_t) d_in & 15) != 0 && n) return JDGPU_EINVAL;
    const uint64_t nb = n ? (n + bs - 1) / bs : 1;
    const uint32_t cb = (uint32_t) (nb < JD_CHUNK_BLOCKS ? nb : JD_CHUNK_BLOCKS);
    const uint32_t slot = slotcap_for(bs);
    const uint64_t slots = (uint64_t) cb * bs;
    /* levels 6-9: the segment-split parse (k_pspec/k_psync/k_pjoin); levels
     * 1-5: the one-lane-per-block greedy k_parse */
    const bool split = level >= 6;
    const uint32_t pcap = jdk_pcap(bs);
    const int r = dscratch(e.ds, cb, bs, level, split);
    if (r) return r;
    if (!d_csizes && !e.csize.ensure(nb * 4)) return JDGPU_EOOM;
    if (!d_coffs && !e.coff.ensure(nb * 8)) return JDGPU_EOOM;
    if (!d_total && !e.total.ensure(64)) return JDGPU_EOOM;
    uint32_t* csz = d_csizes ? d_csizes : e.csize.as<uint32_t>();
    uint64_t* cof = d_coffs ? d_coffs : e.coff.as<uint64_t>();
    uint64_t* tot = d_total ? d_total : e.total.as<uint64_t>();
    DScratch& x = e.ds;
    for (uint64_t b0 = 0; b0 < nb; b0 += cb) {
        const uint32_t k = (uint32_t) (nb - b0 < cb ? nb - b0 : cb);
        const uint64_t off = b0 * bs;
        JdDeflateLaunch L;
        memset(&L, 0, sizeof(L));
        L.in = d_in + off;
        L.n = n - off;
        if (L.n > (uint64_t) k * bs) L.n = (uint64_t) k * bs;
        L.bs = bs;
        L.nblocks = k;
        L.level = level;
        L.flags = flags;
        L.lastfinal = (b0 + k == nb && lastflush == 1) ? 1 : 0;
        L.chains = x.chains.as<uint16_t>();
        L.tokens = x.tokens.as<uint32_t>();
        L.nslots = slots;
        L.rec = x.rec.as<uint64_t>();
        L.dbinfo = x.dbinfo.as<uint32_t>();
        L.stage = x.stage.as<uint8_t>();
        L.slotcap = slot;
        L.csize = csz + b0;
        L.coff = cof + b0;
        L.total = tot;
        L.base = b0 ? tot : nullptr;
        L.out = d_out;
        L.outcap = outcap;
        if (split) {
            L.plist = x.plist.as<uint64_t>();
            L.pcount = x.pcount.as<uint32_t>();
            L.psync = x.psync.as<uint32_t>();
            L.pcap = pcap;
            L.dsg = x.dsg.as<uint32_t>();
            L.pord = x.pord.as<uint32_t>();
        }
        L.stream = st;
        if (jdk_deflate_launch(&L)) return JDGPU_ENODEV;
    }
    return 0;
}

uint64_t stream_bound(uint64_t n)
{
    const uint64_t stored = (n + 65534) / 65535 * 5 + n + 5;
    const uint64_t coded = n + n / 8 + jdk_stream_maxdb(n) * 640 + 64;
    return stored > coded ? stored : coded;
}

/* one launch of the single-window pipeline (jd_kernels.h JdStreamLaunch):
 * the launch buffer is the history, then the piece; the reference's calls,
 * the window at the parse start, the stale-bucket overrides and the hash-3
 * heads before the buffer come from the stream's carried state */
struct StreamParams {
    uint32_t dsz = 0;                 /* dictionary rule, JD_DSZ_NONE past the start */
    uint32_t pstart = 0;
    std::vector<JdOverride> ov;
    const uint32_t* inc3 = nullptr;   /* device */
    std::vector<uint64_t> cend;       /* launch offsets; empty: one call to n */
    JdWinState w0;
    JdWinState* wout = nullptr;       /* host: the window at the end (synchronises) */
    StreamParams() { memset(&w0, 0, sizeof(w0)); }
};

/* caller holds the lock.  *d_total gets the output size. */
int stream_launch(Engine& e, const uint8_t* d_in, uint64_t n, int level, uint32_t flags, int flush,
                  uint8_t* d_out, uint64_t outcap, uint64_t* d_total, hipStream_t st,
                  const StreamParams& P)
{
    if (level < 0 || level > 9) return JDGPU_EINVAL;
    if (flush != 1 && flush != 2) return JDGPU_EINVAL;
    if ((((uintptr_t) d_in & 15) && n) || n >= (1ull << 32) - 65536 || P.pstart > n) return JDGPU_EINVAL;
    if (outcap < stream_bound(n - P.pstart)) return JDGPU_ECAP;
    SScratch& x = e.ss;
    const uint64_t nb = (n + 65535) / 65536, nunits = (n + 32767) / 32768;
    const uint64_t maxdb = jdk_stream_maxdb(n);
    const uint32_t pcap = jdk_pcap(65536);
    if (level) {
        if (!x.chains.ensure(n * 4 + 64) || !x.rec.ensure(n * 8 + 64) || !x.tokens.ensure(n * 4 + 64) ||
            !x.last3.ensure(nunits * 16384 * 4 + 64) ||
            !x.plist.ensure(nb * 2 * JD_PSEG * pcap * 8 + 64) ||
            !x.pcount.ensure(nb * 2 * JD_PSEG * 4 + 64) || !x.psync.ensure(nb * 2 * JD_PSEG * 8 + 64) ||
            !x.dsg.ensure(nb * 4 + 64) || !x.dbinfo.ensure(JD_DBSTRIDE * 4 + 64) ||
            !x.stage.ensure(n * 8 + maxdb * 1024 + 256))
            return JDGPU_EOOM;
    }
    const uint64_t ncall = P.cend.empty() ? 1 : P.cend.size();
    if (!x.sdb.ensure((1 + 2 * maxdb) * 4 + 64) || !x.win.ensure(sizeof(JdWinState) + 64) ||
        !x.bl.ensure((maxdb + 1) * 4 + 64) || !x.bo.ensure((maxdb + 1) * 8 + 64) ||
        !x.tslot.ensure(64) || !x.dbinfo.ensure(JD_DBSTRIDE * 4 + 64) ||
        !x.ov.ensure((P.ov.size() + 1) * sizeof(JdOverride)) || !x.cend.ensure(ncall * 8 + 64))
        return JDGPU_EOOM;
    if (!x.stage.ensure(256)) return JDGPU_EOOM;
    if (!P.ov.empty() && hipMemcpyAsync(x.ov.p, P.ov.data(), P.ov.size() * sizeof(JdOverride),
                                        hipMemcpyHostToDevice, st) != hipSuccess)
        return JDGPU_ENODEV;
    if (P.cend.empty()) {
        if (hipMemcpyAsync(x.cend.p, &n, 8, hipMemcpyHostToDevice, st) != hipSuccess) return JDGPU_ENODEV;
    } else if (hipMemcpyAsync(x.cend.p, P.cend.data(), ncall * 8, hipMemcpyHostToDevice, st) != hipSuccess) {
        return JDGPU_ENODEV;
    }
    /* the uploads read host memory that ends with this call */
    if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
    JdStreamLaunch L;
    memset(&L, 0, sizeof(L));
    L.in = d_in;
    L.n = n;
    L.dsize = P.dsz;
    L.pstart = P.pstart;
    L.ov = P.ov.empty() ? nullptr : x.ov.as<JdOverride>();
    L.nov = (uint32_t) P.ov.size();
    L.inc3 = P.inc3;
    L.cend = x.cend.as<uint64_t>();
    L.ncall = (uint32_t) ncall;
    L.w0 = P.w0;
    L.wout = x.win.as<JdWinState>();
    L.level = level;
    L.flags = flags;
    L.final = flush == 1 ? 1 : 0;
    L.chains = x.chains.as<uint16_t>();
    L.rec = x.rec.as<uint64_t>();
    L.tokens = x.tokens.as<uint32_t>();
    L.last3 = x.last3.as<uint32_t>();
    L.plist = x.plist.as<uint64_t>();
    L.pcount = x.pcount.as<uint32_t>();
    L.psync = x.psync.as<uint32_t>();
    L.dsg = x.dsg.as<uint32_t>();
    L.pcap = pcap;
    L.dbinfo = x.dbinfo.as<uint32_t>();
    L.sdb = x.sdb.as<uint32_t>();
    L.stage = x.stage.as<uint8_t>();
    L.bl = x.bl.as<uint32_t>();
    L.bo = x.bo.as<uint64_t>();
    L.tslot = x.tslot.as<uint32_t>();
    L.out = d_out;
    L.outcap = outcap;
    L.total = d_total;
    L.stream = st;
    if (jdk_deflate_stream_launch(&L)) return JDGPU_ENODEV;
    if (P.wout) {
        if (hipMemcpyAsync(P.wout, x.win.p, sizeof(JdWinState), hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
            return JDGPU_ENODEV;
    }
    return 0;
}

/* single-window stream deflate of device-resident data (the reference fed
 * the whole input in one call, then `flush`); caller holds the lock */
int deflate_stream_dev(Engine& e, const uint8_t* d_in, uint32_t dsize, uint64_t nd, int level,
                       uint32_t flags, int flush, uint8_t* d_out, uint64_t outcap,
                       uint64_t* d_total, hipStream_t st)
{
    if (dsize > 32768) return JDGPU_EINVAL;
    StreamParams P;
    P.dsz = level ? dsize : 0;
    P.pstart = level ? dsize : 0;
    P.w0.inend = P.pstart;
    if (level == 0) {
        /* deflator_setdctnr has no effect at level 0 (:2112) */
        d_in += dsize;
    }
    return stream_launch(e, d_in, nd + (level ? dsize : 0), level, flags, flush, d_out, outcap,
                         d_total, st, P);
}

}  // namespace

extern "C" {

JDEFLATE_API uint64 jdgpu_stream_bound(uint64 n)
{
    return stream_bound(n);
}

JDEFLATE_API int jdgpu_deflate_stream_device(const void* d_in, uint32 dictsize, uint64 n,
                                             int level, uint32 flags, int flush, void* d_out,
                                             uint64 outcap, uint64* d_total, void* stream)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    hipStream_t st = stream ? (hipStream_t) stream : e.stream;
    order(e, st);
    const int r = deflate_stream_dev(e, (const uint8_t*) d_in, dictsize, n, level, flags, flush,
                                     (uint8_t*) d_out, outcap, (uint64_t*) d_total, st);
    mark(e, st);
    return r;
}

/* ---- single-window stream fed in pieces (jdgpu.h JDGPUStream) ---------- */

}  // extern "C"

struct JDGPUStream {
    int level = 6;
    uint32_t flags = 0;
    uint64_t F = 0;                   /* stream offset: input so far          */
    uint64_t H = 0;                   /* stream offset of hist[0] (64 KiB-aligned) */
    uint32_t dsize = 0;               /* dictionary bytes at the stream start */
    std::vector<uint8_t> hist;        /* stream bytes [H, F)                  */
    JdWinState win;                   /* the window at F (stream offsets)     */
    std::vector<JdOverride> ov;       /* stale buckets (stream offsets)       */
    DevBuf inc3;                      /* hash-3 heads before H                */
    bool has3 = false, ended = false;
    JDGPUStream() { memset(&win, 0, sizeof(win)); }
    ~JDGPUStream() { if (inc3.p) (void) hipFree(inc3.p); }
};

namespace {

/* history kept before the flush point: the 32 KiB window and the hash-3
 * ring are within it, and so is every byte an older window generation can
 * still show past inputend (each generation reaches one window size further
 * back) */
uint64_t jd_hist()
{
    static const uint64_t h = [] {
        const char* v = getenv("JDAMD_HIST_KIB");      /* tests: a longer history */
        const uint64_t k = v ? strtoull(v, nullptr, 10) : 0;
        return k >= 512 ? (k << 10) : (uint64_t) (512u << 10);
    }();
    return h;
}

uint32_t hash4(uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3)
{
    return (((b0 << 24) | (b1 << 16) | (b2 << 8) | b3) * 0x1e35a7bdu) >> 16;
}
uint32_t hash3(uint32_t b0, uint32_t b1, uint32_t b2)
{
    return (((b0 << 16) | (b1 << 8) | b2) * 0x1e35a7bdu) >> 18;
}

}  // namespace

extern "C" {

JDEFLATE_API JDGPUStream* jdgpu_stream_create(int level, uint32 flags, const uint8* dict,
                                              uint64 dictsize)
{
    if (level < 0 || level > 9 || (!dict && dictsize)) return nullptr;
    JDGPUStream* s = new (std::nothrow) JDGPUStream;
    if (!s) return nullptr;
    s->level = level;
    s->flags = flags;
    if (level && dictsize) {
        /* deflator_setdctnr :2124-2127: the last 32 KiB only */
        if (dictsize > 32768) {
            dict += dictsize - 32768;
            dictsize = 32768;
        }
        s->hist.assign(dict, dict + dictsize);
        s->dsize = (uint32_t) dictsize;
        s->F = dictsize;
        s->win.inend = dictsize;      /* window[0, dictsize) = the dictionary */
    }
    return s;
}

JDEFLATE_API void jdgpu_stream_destroy(JDGPUStream* s)
{
    if (!s) return;
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    delete s;
}

JDEFLATE_API int64 jdgpu_stream_deflate(JDGPUStream* s, const uint8* src, uint64 n,
                                        const uint64* callends, uint32 ncalls, int flush,
                                        uint8* dst, uint64 cap)
{
    if (!s || (!src && n) || !dst || (flush != 1 && flush != 2) || s->ended) return JDGPU_EINVAL;
    if (callends) {
        if (ncalls == 0 || callends[ncalls - 1] != n) return JDGPU_EINVAL;
        for (uint32_t k = 1; k < ncalls; k++)
            if (callends[k] < callends[k - 1]) return JDGPU_EINVAL;
    }
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    hipStream_t st = e.stream;
    order(e, st);
    Fence fence(e, st);
    if (n == 0) {
        /* nothing since the last flush: endstream :610-654 alone (the output
         * is byte-aligned after a flush or at the start) */
        if (cap < 5) return JDGPU_ECAP;
        const uint8_t t[5] = {(uint8_t) (flush == 1 ? 1 : 0), 0x00, 0x00, 0xff, 0xff};
        memcpy(dst, t, 5);
        if (flush == 1) s->ended = true;
        return 5;
    }
    const bool lazy = s->level >= 6;
    const uint64_t hn = s->level ? s->hist.size() : 0;    /* level 0: pieces are independent */
    const uint64_t ntot = hn + n;
    if (ntot >= (1ull << 32) - 65536) return JDGPU_EINVAL;
    const uint64_t bound = stream_bound(n);
    if (!e.hin.ensure(ntot + 64) || !e.hout.ensure(bound + 64) || !e.ss.total.ensure(64))
        return JDGPU_EOOM;
    if (hn && hipMemcpyAsync(e.hin.p, s->hist.data(), hn, hipMemcpyHostToDevice, st) != hipSuccess)
        return JDGPU_ENODEV;
    if (hipMemcpyAsync(e.hin.as<uint8_t>() + hn, src, n, hipMemcpyHostToDevice, st) != hipSuccess)
        return JDGPU_ENODEV;

    StreamParams P;
    JdWinState wout;
    memset(&wout, 0, sizeof(wout));
    const uint64_t H = s->H;
    if (s->level) {
        P.dsz = H == 0 ? s->dsize : JD_DSZ_NONE;
        P.pstart = (uint32_t) (s->F - H);
        for (const JdOverride& o : s->ov) {
            if (o.pos < H) continue;
            JdOverride r = o;
            r.pos -= H;
            P.ov.push_back(r);
        }
        P.inc3 = s->has3 ? s->inc3.as<uint32_t>() : nullptr;
        if (callends)
            for (uint32_t k = 0; k < ncalls; k++) P.cend.push_back(P.pstart + callends[k]);
        P.w0 = s->win;
        P.w0.sbase -= H;
        P.w0.inend -= H;
        for (uint32_t g = 0; g < s->win.ngen; g++) {
            /* every byte a generation can show lies in the history */
            if (s->win.gb[g] < H) return JDGPU_EINVAL;
            P.w0.gb[g] -= H;
        }
        P.wout = &wout;
    }
    int r = stream_launch(e, e.hin.as<uint8_t>(), ntot, s->level, s->flags & 1u, flush,
                          e.hout.as<uint8_t>(), bound, e.ss.total.as<uint64_t>(), st, P);
    if (r) return r;
    if (s->level && (wout.err || wout.inend != ntot)) return JDGPU_EINVAL;

    uint64_t total = 0;
    if (hipMemcpyAsync(&total, e.ss.total.p, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    if (total > cap) return JDGPU_ECAP;
    if (hipMemcpyAsync(dst, e.hout.p, total, hipMemcpyDeviceToHost, st) != hipSuccess)
        return JDGPU_ENODEV;

    const uint64_t F1 = s->F + n;
    if (flush == 2 && s->level) {
        /* the buffer as the host holds it: history, then the piece */
        std::vector<uint8_t> buf;
        buf.reserve(ntot);
        buf.insert(buf.end(), s->hist.begin(), s->hist.end());
        buf.insert(buf.end(), src, src + n);
        /* bytes past the flush point as the window shows them (SView) */
        auto view = [&](uint64_t x) -> uint32_t {   /* x: launch offset */
            if (x < ntot) return buf[x];
            const uint64_t o = x - wout.sbase;
            for (uint32_t gg = 0; gg < wout.ngen; gg++)
                if (o < wout.gh[gg]) {
                    const uint64_t y = wout.gb[gg] + o;
                    return y < ntot ? buf[y] : 0u;
                }
            return 0u;
        };
        /* compress2 filed position p under the hash computed at p - 1
         * (gethead(cursor + 1), :2646-2648): for p - 1 inside this piece
         * and p + 3 past the flush point that read the window's stale bytes
         * (aux3/aux4 carry the hash of F1 itself into the next piece) */
        std::vector<JdOverride> nov;
        for (uint64_t p = F1 >= 3 ? F1 - 3 : 0; p <= F1; p++) {
            if (p < s->F + 1) continue;
            const uint64_t q = p - H;
            JdOverride o;
            o.pos = p;
            o.h4 = hash4(view(q), view(q + 1), view(q + 2), view(q + 3));
            o.h3 = lazy ? hash3(view(q), view(q + 1), view(q + 2)) : 0xffffffffu;
            nov.push_back(o);
        }
        /* the window at F1 in stream offsets */
        JdWinState w = wout;
        w.sbase += H;
        w.inend += H;
        for (uint32_t gg = 0; gg < w.ngen; gg++) w.gb[gg] += H;
        /* the history for the next piece, and the hash-3 heads before it */
        const uint64_t F1a = F1 & ~0xffffull;
        const uint64_t H1 = F1a > jd_hist() ? F1a - jd_hist() : 0;
        if (lazy && H1 > H) {
            const uint64_t u = (H1 - H) / 32768;
            if (!s->inc3.ensure(16384 * 4) ||
                hipMemcpyAsync(s->inc3.p, e.ss.last3.as<uint32_t>() + u * 16384, 16384 * 4,
                               hipMemcpyDeviceToDevice, st) != hipSuccess)
                return JDGPU_ENODEV;
            s->has3 = true;
        }
        if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
        std::vector<JdOverride> keep;
        for (const JdOverride& o : s->ov)
            if (o.pos >= H1 && o.pos < nov.front().pos) keep.push_back(o);
        for (const JdOverride& o : nov) keep.push_back(o);
        s->ov.swap(keep);
        s->hist.assign(buf.begin() + (H1 - H), buf.end());
        s->H = H1;
        s->win = w;
    } else if (hipStreamSynchronize(st) != hipSuccess) {
        return JDGPU_ENODEV;
    }
    s->F = F1;
    if (flush == 1) s->ended = true;
    return (int64) total;
}

JDEFLATE_API int64 jdgpu_deflate_stream_dict(const uint8* dict, uint64 dictsize, const uint8* src,
                                             uint64 n, int level, uint32 flags, int flush,
                                             uint8* dst, uint64 cap)
{
    if ((!src && n) || !dst || (!dict && dictsize)) return JDGPU_EINVAL;
    JDGPUStream* s = jdgpu_stream_create(level, flags, dict, dictsize);
    if (!s) return JDGPU_EINVAL;
    const int64 r = jdgpu_stream_deflate(s, src, n, nullptr, 0, flush, dst, cap);
    jdgpu_stream_destroy(s);
    return r;
}


JDEFLATE_API int jdgpu_available(void)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    return ready(e) ? 1 : 0;
}

JDEFLATE_API uint64 jdgpu_bound(uint64 n, uint32 blocksize)
{
    if (!valid_bs(blocksize)) return 0;
    const uint64_t nb = n ? (n + blocksize - 1) / blocksize : 1;
    return nb * slotcap_for(blocksize);
}

JDEFLATE_API int64 jdgpu_deflate_stream(const uint8* src, uint64 n, int level, uint32 flags,
                                        int flush, uint8* dst, uint64 cap)
{
    static const uint8 none = 0;
    return jdgpu_deflate_stream_dict(&none, 0, src, n, level, flags, flush, dst, cap);
}

JDEFLATE_API int jdgpu_deflate_device(const void* d_in, uint64 n, uint32 blocksize,
                                      int level, uint32 flags, int lastflush,
                                      void* d_out, uint64 outcap, uint32* d_csizes,
                                      uint64* d_coffsets, uint64* d_total, void* stream)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    hipStream_t st = stream ? (hipStream_t) stream : e.stream;
    order(e, st);
    const int r = deflate_dev(e, (const uint8_t*) d_in, n, blocksize, level, flags, lastflush,
                              (uint8_t*) d_out, outcap, d_csizes, (uint64_t*) d_coffsets,
                              (uint64_t*) d_total, st);
    mark(e, st);
    return r;
}

JDEFLATE_API int jdgpu_inflate_device(const void* d_in, uint64 inlen,
                                      const uint64* d_coffsets, const uint32* d_csizes,
                                      uint32 nblocks, uint32 blocksize, void* d_out,
                                      uint32* d_usizes, int32* d_errors, void* stream)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    if (!blocksize || (blocksize & 3)) return JDGPU_EINVAL;
    JdInflateLaunch L;
    memset(&L, 0, sizeof(L));
    L.in = (const uint8_t*) d_in;
    L.inlen = inlen;
    L.coff = (const uint64_t*) d_coffsets;
    L.csize = d_csizes;
    L.nblocks = nblocks;
    L.bs = blocksize;
    L.out = (uint8_t*) d_out;
    L.usize = d_usizes;
    L.err = (int32_t*) d_errors;
    L.stream = stream ? stream : (void*) e.stream;
    order(e, (hipStream_t) L.stream);
    inflate_scratch(e, L);
    const int r = jdk_inflate_launch(&L) ? JDGPU_ENODEV : 0;
    mark(e, (hipStream_t) L.stream);
    return r;
}

/* CRC register and Adler-32 of n device bytes at d (16-byte aligned),
 * updated in place (NULL: not wanted), with the per-block results in the
 * caller's scratch (ck device, hck host); synchronises the stream.  The
 * engine's zero-byte operators (shiftm) are read-only after ready(). */
static int checksum_scan(Engine& e, DevBuf& ck, std::vector<uint32_t>& hck, const uint8_t* d, uint64_t n,
                         uint32_t* crc, uint32_t* adler, hipStream_t st)
{
    if ((!crc && !adler) || !n) return 0;
    const uint32_t bs = 65536;
    const uint64_t nb = (n + bs - 1) / bs;
    if (!ck.ensure(nb * 12 + 64)) return JDGPU_EOOM;
    hck.resize(nb * 3);
    if (jdk_checksum_launch(d, n, bs, e.shiftm.as<uint32_t>(), ck.as<uint32_t>(), st) ||
        hipMemcpyAsync(hck.data(), ck.p, nb * 12, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    if (crc) *crc = jdcrc_join(*crc, hck.data(), n, bs);
    if (adler) *adler = jdadler_join(*adler, hck.data(), n, bs);
    return 0;
}

/* the same with the engine's scratch (caller holds the lock) */
static int checksum_dev(Engine& e, const uint8_t* d, uint64_t n, uint32_t* crc, uint32_t* adler,
                        hipStream_t st)
{
    return checksum_scan(e, e.ck, e.hck, d, n, crc, adler, st);
}

static int64 deflate_host(Engine& e, const uint8* src, uint64 n, uint32 blocksize, int level,
                          uint32 flags, int lastflush, uint8* dst, uint64 cap,
                          uint32* csizes, uint32* crc, uint32* adler)
{
    if (!ready(e)) return JDGPU_ENODEV;
    if (!valid_bs(blocksize) || (!src && n) || !dst) return JDGPU_EINVAL;
    const uint64_t nb = n ? (n + blocksize - 1) / blocksize : 1;
    const uint64_t bound = nb * slotcap_for(blocksize);
    if (!e.hin.ensure(n + 64) || !e.hout.ensure(bound + 64) || !e.hsz.ensure(nb * 4 + 64))
        return JDGPU_EOOM;
    hipStream_t st = e.stream;
    order(e, st);
    Fence fence(e, st);
    if (n && hipMemcpyAsync(e.hin.p, src, n, hipMemcpyHostToDevice, st) != hipSuccess)
        return JDGPU_ENODEV;
    int r = deflate_dev(e, e.hin.as<uint8_t>(), n, blocksize, level, flags, lastflush,
                        e.hout.as<uint8_t>(), bound, e.hsz.as<uint32_t>(), nullptr,
                        nullptr, st);
    if (r) return r;
    uint64_t total = 0;
    if (hipMemcpyAsync(&total, e.total.p, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    if (total > cap) return JDGPU_ECAP;
    if (hipMemcpyAsync(dst, e.hout.p, total, hipMemcpyDeviceToHost, st) != hipSuccess)
        return JDGPU_ENODEV;
    if (csizes && hipMemcpyAsync(csizes, e.hsz.p, nb * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return JDGPU_ENODEV;
    if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
    if ((r = checksum_dev(e, e.hin.as<uint8_t>(), n, crc, adler, st))) return r;
    return (int64) total;
}

JDEFLATE_API int64 jdgpu_deflate(const uint8* src, uint64 n, uint32 blocksize, int level,
                                 uint32 flags, int lastflush, uint8* dst, uint64 cap,
                                 uint32* csizes)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    return deflate_host(e, src, n, blocksize, level, flags, lastflush, dst, cap, csizes,
                        nullptr, nullptr);
}

JDEFLATE_API int64 jdgpu_deflate_cs(const uint8* src, uint64 n, uint32 blocksize, int level,
                                    uint32 flags, int lastflush, uint8* dst, uint64 cap,
                                    uint32* csizes, uint32* crc, uint32* adler)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    return deflate_host(e, src, n, blocksize, level, flags, lastflush, dst, cap, csizes,
                        crc, adler);
}

JDEFLATE_API int jdgpu_checksum_device(const void* d_in, uint64 n, uint32 blocksize,
                                       uint32* d_out, void* stream)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    if (!valid_bs(blocksize) || (n && (!d_in || !d_out)) || ((uintptr_t) d_in & 15))
        return JDGPU_EINVAL;
    hipStream_t st = stream ? (hipStream_t) stream : e.stream;
    order(e, st);
    const int r = jdk_checksum_launch((const uint8_t*) d_in, n, blocksize, e.shiftm.as<uint32_t>(),
                                      d_out, st) ? JDGPU_ENODEV : 0;
    mark(e, st);
    return r;
}

JDEFLATE_API int jdgpu_checksum(const uint8* src, uint64 n, uint32* crc, uint32* adler)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    if (n && !src) return JDGPU_EINVAL;
    hipStream_t st = e.stream;
    order(e, st);
    Fence fence(e, st);
    const uint64_t chunk = 256ull << 20;
    for (uint64_t o = 0; o < n; o += chunk) {
        const uint64_t m = n - o < chunk ? n - o : chunk;
        if (!e.hin.ensure(m + 64)) return JDGPU_EOOM;
        if (hipMemcpyAsync(e.hin.p, src + o, m, hipMemcpyHostToDevice, st) != hipSuccess)
            return JDGPU_ENODEV;
        int r = checksum_dev(e, e.hin.as<uint8_t>(), m, crc, adler, st);
        if (r) return r;
    }
    return 0;
}

static int inflate_host(Engine& e, const uint8_t* src, uint64_t srclen, const uint32_t* csizes,
                        uint32_t nblocks, uint32_t bs, uint8_t* dst, uint64_t dstcap,
                        uint32_t* usizes, int32_t* errors, uint32_t* used, int require_final)
{
    if (!ready(e)) return JDGPU_ENODEV;
    if (!nblocks || !bs || (bs & 3)) return JDGPU_EINVAL;
    uint64_t* offs = (uint64_t*) malloc((size_t) nblocks * 8);
    if (!offs) return JDGPU_EOOM;
    uint64_t acc = 0;
    for (uint32_t i = 0; i < nblocks; i++) { offs[i] = acc; acc += csizes[i]; }
    const uint64_t outn = (uint64_t) nblocks * bs;
    int r = 0;
    if (acc > srclen) r = JDGPU_EINVAL;
    else if (!e.hin.ensure(srclen + 64) || !e.hout.ensure(outn + 64) ||
             !e.hsz.ensure((uint64_t) nblocks * 4 + 64) || !e.hoff.ensure((uint64_t) nblocks * 8 + 64) ||
             !e.hus.ensure((uint64_t) nblocks * 4 + 64) || !e.herr.ensure((uint64_t) nblocks * 4 + 64) ||
             !e.hused.ensure((uint64_t) nblocks * 4 + 64))
        r = JDGPU_EOOM;
    hipStream_t st = e.stream;
    order(e, st);
    Fence fence(e, st);
    if (!r) {
        if ((srclen && hipMemcpyAsync(e.hin.p, src, srclen, hipMemcpyHostToDevice, st) != hipSuccess) ||
            hipMemcpyAsync(e.hsz.p, csizes, (size_t) nblocks * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
            hipMemcpyAsync(e.hoff.p, offs, (size_t) nblocks * 8, hipMemcpyHostToDevice, st) != hipSuccess)
            r = JDGPU_ENODEV;
    }
    if (!r) {
        JdInflateLaunch L;
        memset(&L, 0, sizeof(L));
        L.in = e.hin.as<uint8_t>();
        L.inlen = srclen;
        L.coff = e.hoff.as<uint64_t>();
        L.csize = e.hsz.as<uint32_t>();
        L.nblocks = nblocks;
        L.bs = bs;
        L.out = e.hout.as<uint8_t>();
        L.usize = e.hus.as<uint32_t>();
        L.err = e.herr.as<int32_t>();
        L.used = e.hused.as<uint32_t>();
        L.require_final = require_final;
        L.stream = st;
        inflate_scratch(e, L);
        if (jdk_inflate_launch(&L)) r = JDGPU_ENODEV;
    }
    uint32_t* us = usizes ? usizes : (uint32_t*) malloc((size_t) nblocks * 4);
    int32_t* er = errors ? errors : (int32_t*) malloc((size_t) nblocks * 4);
    if (!r && (!us || !er)) r = JDGPU_EOOM;
    if (!r) {
        if (hipMemcpyAsync(us, e.hus.p, (size_t) nblocks * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipMemcpyAsync(er, e.herr.p, (size_t) nblocks * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
            (used && hipMemcpyAsync(used, e.hused.p, (size_t) nblocks * 4, hipMemcpyDeviceToHost, st) != hipSuccess) ||
            hipStreamSynchronize(st) != hipSuccess)
            r = JDGPU_ENODEV;
    }
    bool full = !r;
    for (uint32_t i = 0; full && i + 1 < nblocks; i++) full = us[i] == bs;
    if (full) {
        /* every block but the last filled its slot: the device layout is the
         * destination layout, one copy moves it all */
        uint64_t m = (uint64_t) (nblocks - 1) * bs + us[nblocks - 1];
        if (m > dstcap) m = dstcap;
        if (m && hipMemcpyAsync(dst, e.hout.p, m, hipMemcpyDeviceToHost, st) != hipSuccess)
            r = JDGPU_ENODEV;
        if (!r && hipStreamSynchronize(st) != hipSuccess) r = JDGPU_ENODEV;
        for (uint32_t i = 0; i < nblocks && !r; i++)
            if (er[i]) r = JDGPU_EDATA;
    } else if (!r) {
        /* copy each block's decoded bytes */
        for (uint32_t i = 0; i < nblocks && !r; i++) {
            const uint64_t o = (uint64_t) i * bs;
            if (o >= dstcap) break;
            uint64_t m = us[i];
            if (o + m > dstcap) m = dstcap - o;
            if (m && hipMemcpyAsync(dst + o, e.hout.as<uint8_t>() + o, m, hipMemcpyDeviceToHost, st) != hipSuccess)
                r = JDGPU_ENODEV;
        }
        if (!r && hipStreamSynchronize(st) != hipSuccess) r = JDGPU_ENODEV;
        for (uint32_t i = 0; i < nblocks && !r; i++)
            if (er[i]) r = JDGPU_EDATA;
    }
    if (!usizes) free(us);
    if (!errors) free(er);
    free(offs);
    return r;
}

JDEFLATE_API int jdgpu_inflate(const uint8* src, uint64 srclen, const uint32* csizes,
                               uint32 nblocks, uint32 blocksize, uint8* dst, uint32* usizes,
                               int32* errors)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    return inflate_host(e, src, srclen, csizes, nblocks, blocksize, dst,
                        (uint64_t) nblocks * blocksize, usizes, errors, nullptr, 0);
}

/* ---- one RFC 1951 stream: the resumable decoder ------------------------
 *
 * JDGPUInflateStream is the device side of one drop-in inflator (and of the
 * one-shot stream entry points).  Between calls it keeps, in device memory,
 * the decoder state (JdInfState: block mode, the current block's tables, a
 * pending copy, the stored remainder) and the window -- the last <= 32 KiB
 * of output, or the preset dictionary -- in front of the output area:
 *
 *     out: [ window (JD_WIN bytes, the last wlen of them valid) | output ]
 *
 * and on the host only the input bytes from the resume byte on that the
 * decoder could not use yet (a partial token or block header, a few hundred
 * bytes at most).  A call decodes the carried bytes followed by its new
 * input, so every bit is decoded once (inflator.c decodeblock :1330-1518,
 * copybytes :1214-1290, updatewindow :617-675 keep the same state).
 *
 * Decode, per launch slab (<= JD_OSLAB output bytes, <= JD_ISLAB input):
 *  1. Parallel prefix: while the state stands at a block header on a byte
 *     boundary with >= JD_PAR_MIN input bytes ahead, the input is cut at its
 *     00 00 FF FF sync markers (k_markers) and the segments are decoded as
 *     independent blocks (k_inflate_par / k_inflate_resolve) into
 *     consecutive 64 KiB slots.  Segments are accepted in order while each
 *     decodes without error to exactly its last bit, references nothing
 *     before its own start, and filled its slot (all but the last
 *     accepted); a segment with BFINAL ends the stream.  The accepted prefix
 *     is exactly what a serial decode yields; nothing is inferred from a
 *     marker that was not verified.
 *  2. Serial (k_inflate_resume, one wave) from the state, until the input
 *     ends, the output slab is full, the final block ends, an error, or a
 *     sync marker with enough input behind it for step 1 again.
 * The result goes to the caller's buffer (D2H) and the window moves on.
 */
#define JD_WIN 32768u
#define JD_PAR_MIN (128u << 10)
#define JD_OSLAB (1ull << 30)
#define JD_ISLAB (1ull << 30)
#define JD_AHEAD (64ull << 20)    /* parallel output decoded ahead of a small target */
#define JD_FSP_SPAN (128u << 10)  /* input bytes per search region (a chunk)          */
#define JD_FSP_MAXC 512u          /* chunks per parallel round                        */
#define JD_FSP_MIN (1u << 20)     /* input bytes ahead for a parallel round           */
#define JD_FSP_OCAP (16u * JD_FSP_SPAN)   /* output entries per chunk                */
#define JD_FSP_OCAPMAX (64u << 20)        /* ... at most (a 128 MiB u16 chunk)       */
#define JD_FSP_SCRATCH (2ull << 30)      /* u16 chunk output per round               */
#define JD_RP_MIN 2048u                   /* input bytes for a parallel resume        */
#define JD_HBOUNCE (1u << 20)             /* pinned bounce buffers of a stream decoder */

/* The engine-wide lock, taken by a stream decoder call only where it uses
 * the engine's shared workspace (the marker and chunk-parallel rounds, the
 * checksum scan): everything else -- its kernels, its own buffers, its own
 * HIP stream -- is per instance, so instances on different threads overlap
 * (the reference permits one instance per thread, inflator.h).  The first
 * use orders the instance's stream after the last shared-workspace work of
 * any stream (order), and the release marks it (mark). */
struct IsLock {
    Engine& e;
    hipStream_t st;
    std::unique_lock<std::mutex> lk;
    bool caller_holds;
    IsLock(Engine& e_, hipStream_t st_, bool held) : e(e_), st(st_), lk(e_.mu, std::defer_lock), caller_holds(held) {}
    void need()
    {
        if (caller_holds || lk.owns_lock()) return;
        lk.lock();
        order(e, st);
    }
    ~IsLock()
    {
        if (lk.owns_lock()) mark(e, st);
    }
};

struct JDGPUInflateStream {
    int dev = 0;
    hipStream_t hs = nullptr;    /* this instance's HIP stream            */
    bool own_hs = false;
    bool own_q = false;          /* hs has a hardware queue of its own        */
    hipEvent_t give_ev = nullptr; /* recorded after a copy of output to the host */
    bool gave = false;           /* give_ev follows the last such copy        */
    IsLock* lk = nullptr;        /* the current call's shared-workspace lock */
    DevBuf st, in, out, tmp;
    DevBuf ck;                   /* checksums of delivered output: own scratch, */
    std::vector<uint32_t> hck;   /* so a gzip/zlib decode needs no engine lock */
    uint64_t outcap = 0;         /* output bytes `out` holds after the window */
    uint32_t wlen = 0;
    uint32_t bit0 = 0;           /* bits of the first carried/new byte consumed */
    uint32_t mode = JD_RS_HEADER;
    uint32_t plen = 0;           /* a back-reference copy is pending          */
    /* decoded ahead of a small target: out[JD_WIN + pend_off, + pend_len)
     * is still to be delivered, of pend_total bytes decoded at out + JD_WIN
     * (the window moves on once all of them went) */
    uint64_t pend_off = 0, pend_len = 0, pend_total = 0;
    uint32_t last = JD_RST_NEEDINPUT;
    int32_t err = 0;
    std::vector<uint8_t> carry;
    /* the caller's input still staged on the device after a full target:
     * its next call continues at cache_src (the rest of the same buffer) */
    const uint8_t* cache_src = nullptr;
    uint64_t cache_len = 0, cache_dev = 0;
    uint64_t cache_hash = 0;                  /* span_hash of those bytes    */
    uint64_t stat_launches = 0, stat_parallel = 0, stat_carried = 0;
    /* parallel decode of marker-free input (stream_fsp) */
    bool fsp = true;
    uint32_t fsp_ocap = JD_FSP_OCAP;
    uint64_t stat_frounds = 0, stat_fchunks = 0;
    /* pinned bounce buffers for small calls (a pageable copy costs a staged
     * round trip each way; a 32 KiB read and a 64 KiB target are the
     * reference's callback-mode pattern, zstrm.c:900-930) */
    void* hhead = nullptr;        /* pinned: the state head read back after a launch */
    bool pinned_tried = false;    /* the pinned buffers below were set up     */
    uint8_t* hb_in = nullptr;
    uint8_t* hb_out = nullptr;
    /* the span at hand decoded by 64 lanes (k_inflate_rpar) */
    DevBuf rrec;
    bool rpar = true;
    double rp_bpb = 4.0;          /* input bits per output byte, as last seen */
    uint64_t stat_rpar = 0;
};

namespace {

/* parallel prefix over d[0, len) (len <= JD_ISLAB): accepted segments decode
 * into dout (at most cap bytes); returns the number accepted (0 = none) */
int stream_prefix(Engine& e, const uint8_t* base, uint64_t x0, uint64_t len, uint8_t* dout,
                  uint64_t cap, uint64_t* outp, uint64_t* inpos, bool* ended, hipStream_t st)
{
    const uint8_t* d = base + x0;        /* the block decoders read from the aligned base */
    const uint32_t bs = 65536;
    const uint64_t nc = (len + JD_MK_CH - 1) / JD_MK_CH;
    if (!e.mk.ensure(nc * (JD_MK_MAX + 1) * 4 + 64)) return JDGPU_EOOM;
    uint32_t* dcnt = e.mk.as<uint32_t>();
    uint32_t* doff = dcnt + nc;
    std::vector<uint32_t> cnt(nc), off(nc * JD_MK_MAX);
    if (jdk_markers_launch(d, len, dcnt, doff, st) ||
        hipMemcpyAsync(cnt.data(), dcnt, nc * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(off.data(), doff, nc * JD_MK_MAX * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    /* segment ends: the markers, up to the first chunk with too many to list
     * (those segments are short; the serial decoder takes over there) */
    std::vector<uint32_t> ends;
    for (uint64_t c = 0; c < nc; c++) {
        if (cnt[c] == 0xffffffffu) break;
        for (uint32_t k = 0; k < cnt[c]; k++) ends.push_back(off[c * JD_MK_MAX + k]);
    }
    /* whole slots only: nb full slots never exceed cap */
    const uint64_t maxseg = cap / bs;
    if (ends.size() > maxseg) ends.resize(maxseg);
    const uint32_t nb = (uint32_t) ends.size();
    if (nb < 1) return 0;
    std::vector<uint32_t> csz(nb);
    std::vector<uint64_t> cof(nb);
    for (uint32_t i = 0; i < nb; i++) {
        const uint64_t a0 = i ? ends[i - 1] : 0;
        cof[i] = x0 + a0;
        csz[i] = (uint32_t) (ends[i] - a0);
    }
    if (!e.hsz.ensure((uint64_t) nb * 4 + 64) || !e.hoff.ensure((uint64_t) nb * 8 + 64) ||
        !e.hus.ensure((uint64_t) nb * 4 + 64) || !e.herr.ensure((uint64_t) nb * 4 + 64) ||
        !e.hused.ensure((uint64_t) nb * 4 + 64) || !e.fin.ensure((uint64_t) nb * 4 + 64))
        return JDGPU_EOOM;
    if (hipMemcpyAsync(e.hsz.p, csz.data(), (size_t) nb * 4, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(e.hoff.p, cof.data(), (size_t) nb * 8, hipMemcpyHostToDevice, st) != hipSuccess)
        return JDGPU_ENODEV;
    JdInflateLaunch L;
    memset(&L, 0, sizeof(L));
    L.in = base;
    L.inlen = x0 + len;
    L.coff = e.hoff.as<uint64_t>();
    L.csize = e.hsz.as<uint32_t>();
    L.nblocks = nb;
    L.bs = bs;
    L.out = dout;
    L.usize = e.hus.as<uint32_t>();
    L.err = e.herr.as<int32_t>();
    L.used = e.hused.as<uint32_t>();
    L.fin = e.fin.as<uint32_t>();
    L.stream = st;
    inflate_scratch(e, L);
    if (jdk_inflate_launch(&L)) return JDGPU_ENODEV;
    std::vector<uint32_t> us(nb), used(nb), fin(nb);
    std::vector<int32_t> er(nb);
    if (hipMemcpyAsync(us.data(), e.hus.p, (size_t) nb * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(er.data(), e.herr.p, (size_t) nb * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(used.data(), e.hused.p, (size_t) nb * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(fin.data(), e.fin.p, (size_t) nb * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    uint32_t acc = 0;
    *ended = false;
    for (uint32_t i = 0; i < nb; i++) {
        /* exactly to the segment's last bit, byte-aligned, no error */
        if (er[i] || used[i] != csz[i] || (fin[i] & 2)) break;
        acc = i + 1;
        if (fin[i] & 1) { *ended = true; break; }
        if (us[i] != bs) break;       /* the next slot would not follow on */
    }
    if (acc < 1) return 0;
    *outp = (uint64_t) (acc - 1) * bs + us[acc - 1];
    *inpos = ends[acc - 1];
    return (int) acc;
}

/* parallel round over a stream without sync markers (JdFspLaunch): the
 * state stands at a block header at bit b0 of din; chunks are searched for
 * up to byte eb and decoded from din[0, inlen); the accepted ones decode into
 * dout (at most cap bytes).  win: the 32 KiB window in front of the output
 * (its last wlen bytes valid).  Returns 1 with the output size, the end bit
 * (from din) and whether the final block ended, 0 if no chunk was accepted
 * or a reference reaches before the stream (the serial decoder then reports
 * it), or an error code. */
int stream_fsp(Engine& e, const uint8_t* din, uint64_t inlen, uint64_t b0, uint64_t eb,
               const uint8_t* win, uint32_t wlen, uint8_t* dout, uint64_t cap,
               uint64_t* outp, uint64_t* endbit, bool* ended, uint32_t* npiece, uint32_t* ocapp,
               hipStream_t st)
{
    const uint64_t rem = eb * 8 > b0 ? eb * 8 - b0 : 0;
    const uint64_t sb = (uint64_t) JD_FSP_SPAN * 8;
    const uint32_t ocap = *ocapp;
    uint64_t nc = (rem + sb - 1) / sb;
    /* about the chunks whose output the target can take (ratio >= 2) */
    const uint64_t byout = cap / (2ull * JD_FSP_SPAN) + 1;
    if (nc > byout) nc = byout;
    if (nc > JD_FSP_MAXC) nc = JD_FSP_MAXC;
    if (nc > JD_FSP_SCRATCH / (2ull * ocap)) nc = JD_FSP_SCRATCH / (2ull * ocap);
    if (nc < 2) return 0;
    if (!e.fo16.ensure(nc * ocap * 2 + 64) || !e.fres.ensure(nc * 32 + 64) ||
        !e.fstart.ensure(nc * 8 + 64) || !e.fwin.ensure((nc + 1) * 32768ull + 64) ||
        !e.fpiece.ensure(nc * 32 + 64) || !e.fflag.ensure(nc * 4 + 64))
        return JDGPU_EOOM;
    JdFspLaunch L;
    memset(&L, 0, sizeof(L));
    L.in = din;
    L.inlen = inlen;
    L.bit0 = b0;
    L.endbit = b0 + nc * sb < eb * 8 ? b0 + nc * sb : eb * 8;
    L.nchunk = (uint32_t) nc;
    L.span = JD_FSP_SPAN;
    L.starts = e.fstart.as<uint64_t>();
    L.o16 = e.fo16.as<uint16_t>();
    L.ocap = ocap;
    L.wlen = wlen;
    L.res = e.fres.as<uint64_t>();
    L.stream = st;
    std::vector<uint64_t> res(nc * 4), starts(nc);
    if (jdk_fsp_decode_launch(&L) ||
        hipMemcpyAsync(res.data(), L.res, nc * 32, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipMemcpyAsync(starts.data(), L.starts, nc * 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    /* the output room per chunk follows the data's ratio: a chunk that ran
     * out of entries (a deflate block can expand to megabytes) makes the
     * next rounds' room 4x larger (and their chunk count smaller) */
    uint64_t most = 0;
    for (uint64_t c = 0; c < nc; c++)
        if (res[4 * c] != JD_FSP_NONE && res[4 * c + 3] > most) most = res[4 * c + 3];
    if (most + 258 > ocap && ocap < JD_FSP_OCAPMAX) *ocapp = ocap * 4;
    /* accept in order: chunk c is exact if the chunk before it reached its
     * start exactly (chunk 0 starts at the decoder's own state) */
    std::vector<uint64_t> pc;
    uint64_t tot = 0, bit = b0, vw = wlen, maxlen = 0;
    bool fin = false;
    for (uint64_t c = 0; c < nc; c++) {
        if (c && starts[c] == ~0ull) continue;
        const uint64_t stt = res[4 * c], lb = res[4 * c + 1], lo = res[4 * c + 2];
        if (stt == JD_FSP_NONE || tot + lo > cap) break;
        pc.insert(pc.end(), {c, lo, tot, vw});
        tot += lo;
        bit = lb;
        vw = vw + lo < 32768 ? vw + lo : 32768;
        if (lo > maxlen) maxlen = lo;
        if (stt == JD_FSP_REACHED) continue;
        fin = stt == JD_FSP_ENDED;
        break;
    }
    const uint32_t np = (uint32_t) (pc.size() / 4);
    if (bit == b0 && !fin) return 0;
    uint32_t flag = 0;
    JdFspResolve R;
    R.o16 = L.o16;
    R.ocap = L.ocap;
    R.npiece = np;
    R.piece = e.fpiece.as<uint64_t>();
    R.maxlen = (uint32_t) maxlen;
    R.win = e.fwin.as<uint8_t>();
    R.out = dout;
    R.flag = e.fflag.as<uint32_t>();
    R.stream = st;
    if (hipMemcpyAsync(e.fpiece.p, pc.data(), pc.size() * 8, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipMemcpyAsync(R.win, win, 32768, hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemsetAsync(R.flag, 0, 4, st) != hipSuccess || jdk_fsp_resolve_launch(&R) ||
        hipMemcpyAsync(&flag, R.flag, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    if (flag) return 0;
    *outp = tot;
    *endbit = bit;
    *ended = fin;
    *npiece = np;
    return 1;
}

/* room for `n` output bytes behind the window (the window is kept) */
bool is_reserve(JDGPUInflateStream* s, uint64_t n, hipStream_t st)
{
    if (n <= s->outcap) return true;
    DevBuf nb;
    if (!nb.ensure(JD_WIN + n + 64)) return false;
    if (s->out.p && (hipMemcpyAsync(nb.p, s->out.p, JD_WIN, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                     hipStreamSynchronize(st) != hipSuccess))
        return false;
    std::swap(s->out.p, nb.p);
    std::swap(s->out.cap, nb.cap);
    if (nb.p) (void) hipFree(nb.p);
    s->outcap = n;
    return true;
}

/* `p` new bytes were decoded at out + JD_WIN: deliver them to dst, update
 * the checksums, and move the window on (the last JD_WIN bytes of window ||
 * output end at JD_WIN again) */
int is_give(Engine& e, JDGPUInflateStream* s, uint64_t from, uint64_t m, uint8_t* dst,
            uint32_t* crc, uint32_t* adler, hipStream_t st)
{
    if (!m) return 0;
    uint8_t* o = s->out.as<uint8_t>() + JD_WIN + from;
    if (hipMemcpyAsync(dst, o, m, hipMemcpyDeviceToHost, st) != hipSuccess) return JDGPU_ENODEV;
    if (!crc && !adler) {
        /* the call's end waits for this copy (an event), not for the stream */
        s->gave = s->give_ev && hipEventRecord(s->give_ev, st) == hipSuccess;
        return 0;
    }
    s->gave = false;
    if (!(from & 15)) return checksum_scan(e, s->ck, s->hck, o, m, crc, adler, st);
    /* k_checksum wants 16-byte aligned input: scan the delivered host copy */
    if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
    if (crc) *crc = jdcrc_bytes(*crc, dst, m);
    if (adler) *adler = jdadler_bytes(*adler, dst, m);
    return 0;
}

int is_slide(JDGPUInflateStream* s, uint64_t p, hipStream_t st)
{
    if (!p) return 0;
    uint8_t* o = s->out.as<uint8_t>();
    if (p >= JD_WIN) {
        if (hipMemcpyAsync(o, o + p, JD_WIN, hipMemcpyDeviceToDevice, st) != hipSuccess) return JDGPU_ENODEV;
        s->wlen = JD_WIN;
    } else {
        const uint32_t keep = s->wlen + p > JD_WIN ? JD_WIN - (uint32_t) p : s->wlen;
        const uint64_t n = keep + p;
        if (!s->tmp.ensure(JD_WIN + 64) ||
            hipMemcpyAsync(s->tmp.p, o + JD_WIN - keep, n, hipMemcpyDeviceToDevice, st) != hipSuccess ||
            hipMemcpyAsync(o + JD_WIN - n, s->tmp.p, n, hipMemcpyDeviceToDevice, st) != hipSuccess)
            return JDGPU_ENODEV;
        s->wlen = (uint32_t) n;
    }
    return 0;
}

int is_take(Engine& e, JDGPUInflateStream* s, uint64_t p, uint8_t* dst, uint32_t* crc,
            uint32_t* adler, hipStream_t st)
{
    int r = is_give(e, s, 0, p, dst, crc, adler, st);
    return r ? r : is_slide(s, p, st);
}

/* a 64-bit hash of n host bytes (four multiply-rotate lanes over 8-byte
 * words, then the tail bytes and the length): tells a rewritten input span
 * from the one still staged on the device */
#define JD_CACHE_MIN (1ull << 20)
#define JD_CACHE_MAX (64ull << 20)
static uint64_t span_hash(const uint8_t* p, uint64_t n)
{
    const uint64_t K = 0x9e3779b97f4a7c15ull;
    uint64_t a[4] = {K, K ^ 1, K ^ 2, K ^ 3};
    uint64_t i = 0;
    for (; i + 32 <= n; i += 32)
        for (int j = 0; j < 4; j++) {
            uint64_t w;
            memcpy(&w, p + i + 8 * j, 8);
            a[j] = ((a[j] ^ w) * K);
            a[j] = (a[j] << 31) | (a[j] >> 33);
        }
    uint64_t h = n * K;
    for (int j = 0; j < 4; j++) h = ((h ^ a[j]) * K) ^ (h >> 29);
    for (; i < n; i++) h = ((h ^ p[i]) * K) ^ (h >> 29);
    return h ^ (h >> 32);
}

/* head of JdInfState read back after a launch */
struct RsHead {
    uint32_t mode, fin, plen, poff, srem, status;
    int32_t err;
    uint32_t pad;
    uint64_t bit, produced;
};

/* one call: decode carry || src[0, n) into dst[0, cap) */
int is_inflate_core(Engine& e, JDGPUInflateStream* s, const uint8_t* src, uint64_t n, uint64_t region,
                    uint8_t* dst, uint64_t cap, JDGPUInflateStep* res, uint32_t* crc, uint32_t* adler)
{
    memset(res, 0, sizeof(*res));
    hipStream_t st = s->hs;
    uint64_t produced = 0;
    if (s->pend_len) {
        /* output decoded ahead of an earlier, smaller target */
        const uint64_t m = s->pend_len < cap ? s->pend_len : cap;
        int r = is_give(e, s, s->pend_off, m, dst, crc, adler, st);
        if (r) return r;
        produced = m;
        s->pend_off += m;
        s->pend_len -= m;
        if (s->pend_len) {
            if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
            res->produced = produced;
            res->status = JDGPU_IS_FULL;
            return 0;
        }
        if ((r = is_slide(s, s->pend_total, st))) return r;
        s->pend_total = 0;
    }
    if (s->mode == JD_RS_ENDED || s->err || (n == 0 && s->last == JD_RST_NEEDINPUT)) {
        if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
        res->produced = produced;
        res->status = s->mode == JD_RS_ENDED ? JDGPU_IS_ENDED : s->err ? JDGPU_IS_ERROR
                                                                     : JDGPU_IS_NEEDINPUT;
        res->error = s->err;
        return 0;
    }
    const uint64_t C = s->carry.size();
    const uint64_t total = C + n;
    if (region > n) region = n;
    const uint64_t vreg = C + region;         /* the marker search stops here */
    /* the same buffer, at least the cached span of it, and the same bytes (a
     * 64-bit hash of the span, read at ~10x the rate of the copy it saves):
     * a caller that rewrote, shortened or reallocated its buffer in between
     * gets it staged again.  The span is a bounded window (JD_CACHE_MIN ..
     * JD_CACHE_MAX, 4x what the last call consumed), so a large source read
     * through small targets costs each call a bounded hash, not one of the
     * whole rest; input past the window is staged from the host. */
    const bool cached = C == 0 && n && src == s->cache_src && s->cache_len && n >= s->cache_len &&
                        span_hash(src, s->cache_len) == s->cache_hash;
    const uint64_t cache_len = s->cache_len;
    uint64_t vb = 0;                           /* byte of V = carry || src           */
    uint32_t bit0 = s->bit0;
    bool prefix_ok = true, fsp_ok = true, done = false;
    uint64_t stopat = ~0ull;                   /* serial stop for another parallel round */
    uint32_t status = JD_RST_NEEDINPUT;
    int32_t err = 0;
    s->cache_src = nullptr;
    s->cache_len = 0;
    uint64_t v0 = 0, doff = 0, vend = 0;       /* the staged slab: V[v0, vend) at in + doff */
    while (!done) {
        /* stage V[vb, vb + slab) at s->in + doff */
        uint64_t slab = total - vb < JD_ISLAB ? total - vb : JD_ISLAB;
        if (cached && vb == 0) slab = cache_len;      /* the verified window */
        /* no input left: only a pending copy can still produce bytes */
        if (slab == 0 && !s->plen) { status = JD_RST_NEEDINPUT; break; }
        v0 = vb;
        doff = 0;
        if (cached && vb == 0) {
            doff = s->cache_dev;
        } else {
            if (!s->in.ensure(slab + 64)) return JDGPU_EOOM;
            uint64_t k = 0;
            if (slab <= JD_HBOUNCE && s->hb_in) {
                /* one pinned copy of carry || src */
                const uint64_t kc = vb < C ? (C - vb < slab ? C - vb : slab) : 0;
                if (kc) memcpy(s->hb_in, s->carry.data() + vb, kc);
                if (slab > kc) memcpy(s->hb_in + kc, src + (vb + kc - C), slab - kc);
                if (hipMemcpyAsync(s->in.p, s->hb_in, slab, hipMemcpyHostToDevice, st) != hipSuccess)
                    return JDGPU_ENODEV;
                k = slab;
            } else if (vb < C) {
                k = C - vb < slab ? C - vb : slab;
                if (hipMemcpyAsync(s->in.p, s->carry.data() + vb, k, hipMemcpyHostToDevice, st) != hipSuccess)
                    return JDGPU_ENODEV;
            }
            if (slab > k && hipMemcpyAsync(s->in.as<uint8_t>() + k, src + (vb + k - C), slab - k,
                                           hipMemcpyHostToDevice, st) != hipSuccess)
                return JDGPU_ENODEV;
        }
        vend = vb + slab;
        /* V byte x is at din + xo + (x - v0); din stays 16-byte aligned */
        const uint8_t* din = s->in.as<uint8_t>() + (doff & ~15ull);
        const uint64_t xo = doff & 15;
        bool serial_next = false;                /* the serial decoder's turn */
        for (;;) {
            const uint64_t left = cap - produced;
            const uint64_t oslab = left < JD_OSLAB ? left : JD_OSLAB;
            if (!is_reserve(s, oslab ? oslab : 1, st)) return JDGPU_EOOM;
            uint8_t* dout = s->out.as<uint8_t>() + JD_WIN;
            /* 1. parallel prefix at a byte-aligned block header; it may
             * decode ahead of a small target (JD_AHEAD), the rest of its
             * output then waits on the device for the next calls */
            const uint64_t pcap = oslab > JD_AHEAD ? oslab : JD_AHEAD;
            const uint64_t vfe = vreg < vend ? vreg : vend;     /* parallel rounds stop here */
            uint64_t p = 0;
            bool ended = false;
            int k = 0;
            if (s->mode == JD_RS_HEADER && bit0 == 0 && prefix_ok && vb < vfe &&
                vfe - vb >= JD_PAR_MIN && is_reserve(s, pcap, st)) {
                dout = s->out.as<uint8_t>() + JD_WIN;
                uint64_t ip = 0;
                s->lk->need();
                k = stream_prefix(e, din, xo + (vb - v0), vfe - vb, dout, pcap, &p, &ip, &ended, st);
                if (k < 0) return k;
                if (k > 0) {
                    s->stat_parallel += (uint64_t) k;
                    vb += ip;
                } else {
                    prefix_ok = false;
                }
            }
            /* 1b. no usable markers: chunks found by their block headers */
            if (k == 0 && s->mode == JD_RS_HEADER && !s->plen && fsp_ok && s->fsp && vb < vfe &&
                vfe - vb >= JD_FSP_MIN && is_reserve(s, pcap, st)) {
                dout = s->out.as<uint8_t>() + JD_WIN;
                const uint64_t b0 = (xo + (vb - v0)) * 8 + bit0;
                uint64_t eb = 0;
                uint32_t np = 0;
                const uint32_t oc0 = s->fsp_ocap;
                s->lk->need();
                k = stream_fsp(e, din, xo + (vend - v0), b0, xo + (vfe - v0), s->out.as<uint8_t>(),
                               s->wlen, dout, pcap, &p, &eb, &ended, &np, &s->fsp_ocap, st);
                if (k < 0) return k;
                if (k == 0 && s->fsp_ocap != oc0) continue;      /* again with more room */
                if (k > 0) {
                    s->stat_frounds++;
                    s->stat_fchunks += np;
                    k = (int) np;
                    vb = v0 + (eb >> 3) - xo;
                    bit0 = (uint32_t) (eb & 7);
                } else {
                    /* decode a few regions serially, then try again */
                    fsp_ok = false;
                    stopat = b0 + 4ull * JD_FSP_SPAN * 8;
                }
            }
            {
                if (k > 0) {
                    res->parallel += (uint32_t) k;
                    if (ended) s->mode = JD_RS_ENDED;
                    if (p > left) {
                        int r = is_give(e, s, 0, left, dst + produced, crc, adler, st);
                        if (r) return r;
                        produced += left;
                        s->pend_off = left;
                        s->pend_len = p - left;
                        s->pend_total = p;
                        status = JD_RST_FULL;
                        done = true;
                        break;
                    }
                    int r = is_take(e, s, p, dst + produced, crc, adler, st);
                    if (r) return r;
                    produced += p;
                    if (ended) {
                        status = JD_RST_ENDED;
                        done = true;
                        break;
                    }
                    continue;
                }
            }
            /* 2. the span at hand, by 64 lanes (k_inflate_rpar) while it
             * makes progress; the serial decoder takes what it leaves (a
             * pending copy, a stored remainder, the last token before a full
             * target, a block it cannot take) */
            const uint64_t il = vend - vb;
            if (il == 0 && !s->plen) { status = JD_RST_NEEDINPUT; break; }
            if (s->rpar && !serial_next && stopat == ~0ull &&
                (s->mode == JD_RS_HUFF || (s->mode == JD_RS_HEADER && !s->plen)) &&
                il >= JD_RP_MIN && oslab >= 1024) {
                const uint64_t xb = xo + (vb - v0);
                const uint64_t a0 = xb & ~15ull;
                const uint32_t room = (uint32_t) (oslab < JD_RP_OUT ? oslab : JD_RP_OUT);
                /* input for about the room's output at the last ratio seen */
                uint64_t want = (uint64_t) ((double) room * s->rp_bpb / 8.0 * 1.25) + 2048;
                if (want < 16384) want = 16384;
                const uint64_t inl = xo + (vend - v0) - a0;
                uint64_t use = inl < (xb - a0) + want ? inl : (xb - a0) + want;
                if (!s->rrec.ensure((uint64_t) JD_RP_MAXREC * 8 + 64)) return JDGPU_EOOM;
                JdRparLaunch P;
                P.in = din + a0;
                P.bitpos = (uint32_t) ((xb - a0) * 8 + bit0);
                P.inlen = (uint32_t) use;
                P.win = s->out.as<uint8_t>();
                P.out = dout;
                P.pos0 = s->wlen;
                P.cap = room;
                P.recs = s->rrec.as<uint64_t>();
                P.st = s->st.as<JdInfState>();
                /* headers where the block-parallel prefix or the chunk-
                 * parallel rounds could take over: within the region */
                P.markmin = prefix_ok ? JD_PAR_MIN : 0;
                P.hdrmin = (s->fsp && fsp_ok) ? JD_FSP_MIN : 0;
                {
                    const uint64_t fe = xo + (vfe - v0), le = a0 + use;
                    P.extra = fe > le ? fe - le : 0;
                }
                P.stream = st;
                RsHead hl, *hp = s->hhead ? (RsHead*) s->hhead : &hl;
                P.hhead = (JdInfState*) s->hhead;      /* written by the kernel (or NULL) */
                if (jdk_inflate_rpar_launch(&P) ||
                    (!P.hhead && hipMemcpyAsync(hp, s->st.p, sizeof(RsHead), hipMemcpyDeviceToHost, st) != hipSuccess) ||
                    hipStreamSynchronize(st) != hipSuccess)
                    return JDGPU_ENODEV;
                const RsHead h = *hp;
                s->stat_rpar++;
                const uint64_t nb = a0 * 8 + h.bit;            /* bit of din */
                const uint64_t used = nb - (xb * 8 + bit0);
                if (h.produced) {
                    int r = is_take(e, s, h.produced, dst + produced, crc, adler, st);
                    if (r) return r;
                    produced += h.produced;
                    if (used > 64) s->rp_bpb = 0.5 * s->rp_bpb + 0.5 * ((double) used / (double) h.produced);
                }
                vb = v0 + (nb >> 3) - xo;
                bit0 = (uint32_t) (nb & 7);
                s->mode = h.mode;
                s->plen = h.plen;
                status = h.status;
                if (status == JD_RST_ENDED) { done = true; break; }
                if (status == JD_RST_MARKER) continue;             /* the parallel rounds */
                if (status == JD_RST_NEEDINPUT && a0 + use < xo + (vend - v0)) continue;  /* the soft end */
                if (status == JD_RST_NEEDINPUT && h.pad) {
                    /* a valid token, header or stored block cut by the
                     * input's end: nothing more until more input */
                    if (vend < total) break;                             /* restage from vb */
                    done = true;
                    break;
                }
                if (status == JD_RST_FULL && room < oslab && produced < cap) continue;   /* its own limit */
                /* full where the serial decoder stops too (before a literal, or
                 * a match split with the rest pending) */
                if (status == JD_RST_FULL && produced >= cap && h.pad) { done = true; break; }
                /* otherwise the serial decoder takes the next step: the rest
                 * of this block (SERIAL: it stops at the next header), the
                 * token that splits at the target's end (FULL; with the target
                 * exactly full it runs with no room, so that a match or an
                 * end of block there is taken as the serial decoder takes it,
                 * copybytes :1214-1290), or the input's last bits (NEEDINPUT:
                 * a token, header or stored block cut by the input's end,
                 * reported as it reports them) */
                serial_next = true;
                if (status == JD_RST_SERIAL) stopat = nb + 1;
                continue;
            }
            const bool handed = serial_next;         /* rpar handed this step over */
            serial_next = false;
            JdResumeLaunch L;
            L.in = din;
            L.bitpos = (xo + (vb - v0)) * 8 + bit0;
            L.inlen = (uint32_t) (xo + (vend - v0));
            L.out = dout;
            L.pos0 = s->wlen;
            L.cap = (uint32_t) oslab;
            L.markmin = prefix_ok ? JD_PAR_MIN : 0;
            L.stopat = stopat;
            stopat = ~0ull;
            L.st = s->st.as<JdInfState>();
            L.stream = st;
            /* with the parallel resume on, the serial decoder only finishes
             * a pending copy (with room to spare) or a stored block, and
             * hands the rest back */
            L.stopcopy = 0;
            if (s->rpar && !handed && s->plen && s->plen < oslab) L.stopcopy = 1;
            if (s->rpar && !handed && s->mode == JD_RS_STORED && L.stopat == ~0ull) L.stopat = L.bitpos + 1;
            RsHead hl, *hp = s->hhead ? (RsHead*) s->hhead : &hl;
            L.hhead = (JdInfState*) s->hhead;
            if (jdk_inflate_resume_launch(&L) ||
                (!L.hhead && hipMemcpyAsync(hp, s->st.p, sizeof(RsHead), hipMemcpyDeviceToHost, st) != hipSuccess) ||
                hipStreamSynchronize(st) != hipSuccess)
                return JDGPU_ENODEV;
            const RsHead h = *hp;
            s->stat_launches++;
            int r = is_take(e, s, h.produced, dst + produced, crc, adler, st);
            if (r) return r;
            produced += h.produced;
            vb = v0 + (h.bit >> 3) - xo;
            bit0 = (uint32_t) (h.bit & 7);
            s->mode = h.mode;
            s->plen = h.plen;
            status = h.status;
            err = h.err;
            if (status == JD_RST_MARKER) {
                fsp_ok = true;
                continue;
            }
            if (status == JD_RST_FULL && produced < cap) continue;
            if (status == JD_RST_NEEDINPUT && vend < total) break;   /* restage from vb */
            done = true;
            break;
        }
        if (!done && status == JD_RST_NEEDINPUT && vend >= total) break;
    }
    /* dst complete: the last copy to the host, not the window slide queued
     * behind it (later work on this stream follows the slide in order) */
    if (s->give_ev && s->gave) {
        if (hipEventSynchronize(s->give_ev) != hipSuccess) return JDGPU_ENODEV;
    } else if (hipStreamSynchronize(st) != hipSuccess) {
        return JDGPU_ENODEV;
    }
    s->gave = false;
    s->last = status;
    res->produced = produced;
    switch (status) {
    case JD_RST_ENDED: {
        const uint64_t vendb = vb + (bit0 ? 1 : 0);       /* the final byte is taken */
        res->consumed = vendb > C ? vendb - C : 0;
        res->status = JDGPU_IS_ENDED;
        s->carry.clear();
        s->bit0 = 0;
        break;
    }
    case JD_RST_FULL:
        /* the final block ended in output still pending: its last byte is taken */
        if (s->mode == JD_RS_ENDED && bit0) {
            vb++;
            bit0 = 0;
        }
        res->consumed = vb > C ? vb - C : 0;
        res->status = JDGPU_IS_FULL;
        if (vb < C) {
            s->carry.erase(s->carry.begin(), s->carry.begin() + (ptrdiff_t) vb);
        } else {
            s->carry.clear();
            /* the rest of the slab is on the device already: a window of it
             * (4x this call's input, JD_CACHE_MIN .. JD_CACHE_MAX) is kept
             * for the caller's next call, which passes the rest of src */
            if (vb < vend) {
                uint64_t w = 4 * vb;
                w = w < JD_CACHE_MIN ? JD_CACHE_MIN : w > JD_CACHE_MAX ? JD_CACHE_MAX : w;
                s->cache_src = src + (vb - C);
                s->cache_len = vend - vb < w ? vend - vb : w;
                s->cache_dev = doff + (vb - v0);
                s->cache_hash = span_hash(s->cache_src, s->cache_len);
            }
        }
        s->bit0 = bit0;
        break;
    case JD_RST_ERROR:
        res->consumed = n;
        res->status = JDGPU_IS_ERROR;
        res->error = err;
        s->err = err ? err : 1;
        break;
    default: {                                   /* input exhausted */
        std::vector<uint8_t> nc;
        nc.reserve(total - vb);
        for (uint64_t x = vb; x < total; x++) nc.push_back(x < C ? s->carry[x] : src[x - C]);
        s->carry.swap(nc);
        s->stat_carried += s->carry.size();
        s->bit0 = bit0;
        res->consumed = n;
        res->status = JDGPU_IS_NEEDINPUT;
        s->last = JD_RST_NEEDINPUT;
    }
    }
    return 0;
}

/* is_inflate_core through the pinned bounce buffers when the call is small:
 * every exit with a result has synchronised the stream, so the bounce holds
 * the output */
int is_inflate(Engine& e, JDGPUInflateStream* s, const uint8_t* src, uint64_t n, uint64_t region,
               uint8_t* dst, uint64_t cap, JDGPUInflateStep* res, uint32_t* crc, uint32_t* adler)
{
    if (!s->pinned_tried && s->own_hs) {
        /* once per instance: each buffer is optional (a failed one leaves
         * its pointer NULL and the path that would use it falls back), and
         * nothing is allocated again on later calls */
        s->pinned_tried = true;
        if (hipHostMalloc((void**) &s->hb_in, JD_HBOUNCE, hipHostMallocDefault) != hipSuccess) s->hb_in = nullptr;
        if (hipHostMalloc((void**) &s->hb_out, JD_HBOUNCE, hipHostMallocDefault) != hipSuccess) s->hb_out = nullptr;
        if (hipHostMalloc(&s->hhead, 256, hipHostMallocDefault) != hipSuccess) s->hhead = nullptr;
        if (hipEventCreateWithFlags(&s->give_ev, hipEventDisableTiming) != hipSuccess) s->give_ev = nullptr;
    }
    if (!s->hb_out || cap > JD_HBOUNCE || !cap)
        return is_inflate_core(e, s, src, n, region, dst, cap, res, crc, adler);
    const int r = is_inflate_core(e, s, src, n, region, s->hb_out, cap, res, crc, adler);
    if (!r && res->produced) memcpy(dst, s->hb_out, res->produced);
    return r;
}

/* a fresh state: header next, window = the dictionary's last 32 KiB */
int is_reset(JDGPUInflateStream* s, const uint8_t* dict, uint64_t dsize, hipStream_t st)
{
    /* a reset gives back the slabs a large stream grew (up to 1 GiB each):
     * an idle instance keeps about 100 KB of device memory */
    if (hipStreamSynchronize(st) != hipSuccess) return JDGPU_ENODEV;
    if (s->in.cap > (4u << 20)) s->in.release();
    if (s->outcap > (4u << 20)) {
        s->out.release();
        s->outcap = 0;
    }
    s->pend_off = s->pend_len = s->pend_total = 0;
    if (!s->st.ensure(sizeof(JdInfState) + 64) || !is_reserve(s, 65536, st)) return JDGPU_EOOM;
    if (dsize > JD_WIN) {
        dict += dsize - JD_WIN;
        dsize = JD_WIN;
    }
    JdInfState h;
    memset(&h, 0, offsetof(JdInfState, lt));
    h.mode = JD_RS_HEADER;
    if (hipMemcpyAsync(s->st.p, &h, offsetof(JdInfState, lt), hipMemcpyHostToDevice, st) != hipSuccess ||
        (dsize && hipMemcpyAsync(s->out.as<uint8_t>() + JD_WIN - dsize, dict, dsize,
                                 hipMemcpyHostToDevice, st) != hipSuccess) ||
        hipStreamSynchronize(st) != hipSuccess)
        return JDGPU_ENODEV;
    s->wlen = (uint32_t) dsize;
    s->bit0 = 0;
    s->mode = JD_RS_HEADER;
    s->plen = 0;
    s->last = JD_RST_NEEDINPUT;
    s->err = 0;
    s->carry.clear();
    s->cache_src = nullptr;
    return 0;
}

/* Instances on hardware queues of their own.  Plain streams share the
 * process's GPU_MAX_HW_QUEUES hardware queues (4 by default) round-robin, so
 * eight instances on eight threads ran two to a queue, one after the other
 * (8 x 8: 4.0x one instance with 4 queues, 6.1x with 16; gpurun_out/s32).  A
 * stream created with a CU mask -- here every CU -- is given a queue of its
 * own; up to IS_OWNQ_MAX live instances take one, the rest a plain stream
 * (jdgpu_istream_queue tells which). */
#define IS_OWNQ_MAX 16
static std::atomic<int> is_ownq_live{0};

static bool is_stream_create(JDGPUInflateStream* s)
{
    if (is_ownq_live.fetch_add(1) < IS_OWNQ_MAX) {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s->dev) == hipSuccess &&
            ncu > 0) {
            std::vector<uint32_t> m((size_t) (ncu + 31) / 32, 0xffffffffu);
            if (ncu % 32) m.back() = (1u << (ncu % 32)) - 1;
            if (hipExtStreamCreateWithCUMask(&s->hs, (uint32_t) m.size(), m.data()) == hipSuccess) {
                s->own_q = true;
                return true;
            }
        }
    }
    is_ownq_live.fetch_sub(1);
    return hipStreamCreateWithFlags(&s->hs, hipStreamNonBlocking) == hipSuccess;
}

void is_free(JDGPUInflateStream* s)
{
    for (DevBuf* b : {&s->st, &s->in, &s->out, &s->tmp, &s->rrec, &s->ck})
        if (b->p) (void) hipFree(b->p);
    if (s->hb_in) (void) hipHostFree(s->hb_in);
    if (s->hb_out) (void) hipHostFree(s->hb_out);
    if (s->hhead) (void) hipHostFree(s->hhead);
    if (s->give_ev) (void) hipEventDestroy(s->give_ev);
    s->give_ev = nullptr;
    if (s->own_hs && s->hs) (void) hipStreamDestroy(s->hs);
    if (s->own_q) is_ownq_live.fetch_sub(1);
    s->own_q = false;
}

}  // namespace

JDEFLATE_API JDGPUInflateStream* jdgpu_istream_create(void)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return nullptr;
    JDGPUInflateStream* s = new (std::nothrow) JDGPUInflateStream();
    if (!s) return nullptr;
    (void) hipGetDevice(&s->dev);
    const char* rp = getenv("JD_RPAR");            /* tests: 0 = serial only */
    s->rpar = !(rp && *rp == '0');
    if (!is_stream_create(s)) {
        delete s;
        return nullptr;
    }
    s->own_hs = true;
    if (is_reset(s, nullptr, 0, s->hs)) {
        is_free(s);
        delete s;
        return nullptr;
    }
    return s;
}

JDEFLATE_API int jdgpu_istream_reset(JDGPUInflateStream* s, const uint8* dict, uint64 dictsize)
{
    if (!s || (!dict && dictsize)) return JDGPU_EINVAL;
    Engine& e = eng();
    {
        std::lock_guard<std::mutex> g(e.mu);
        if (!ready(e)) return JDGPU_ENODEV;
    }
    return is_reset(s, dict, dictsize, s->hs);
}

JDEFLATE_API void jdgpu_istream_destroy(JDGPUInflateStream* s)
{
    if (!s) return;
    if (s->hs) (void) hipStreamSynchronize(s->hs);
    is_free(s);
    delete s;
}

JDEFLATE_API int jdgpu_istream_inflate(JDGPUInflateStream* s, const uint8* src, uint64 n,
                                       uint8* dst, uint64 cap, JDGPUInflateStep* res,
                                       uint32* crc, uint32* adler)
{
    if (!s || !res || (!src && n) || (!dst && cap)) return JDGPU_EINVAL;
    Engine& e = eng();
    {
        std::lock_guard<std::mutex> g(e.mu);
        if (!ready(e)) return JDGPU_ENODEV;
    }
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev != s->dev) return JDGPU_EINVAL;
    /* the engine lock only around the shared workspace (IsLock) */
    IsLock lk(e, s->hs, false);
    s->lk = &lk;
    const int r = is_inflate(e, s, src, n, n, dst, cap, res, crc, adler);
    s->lk = nullptr;
    return r;
}

JDEFLATE_API int jdgpu_istream_fsp(JDGPUInflateStream* s, int enable, uint64* rounds,
                                   uint64* chunks)
{
    if (!s) return JDGPU_EINVAL;
    if (enable >= 0) s->fsp = enable != 0;
    if (rounds) *rounds = s->stat_frounds;
    if (chunks) *chunks = s->stat_fchunks;
    return 0;
}

JDEFLATE_API int jdgpu_istream_rpar(JDGPUInflateStream* s, int enable, uint64* launches)
{
    if (!s) return JDGPU_EINVAL;
    if (enable >= 0) s->rpar = enable != 0;
    if (launches) *launches = s->stat_rpar;
    return 0;
}

JDEFLATE_API int jdgpu_istream_stats(const JDGPUInflateStream* s, uint64* launches,
                                     uint64* parallel, uint64* carried)
{
    if (!s) return JDGPU_EINVAL;
    if (launches) *launches = s->stat_launches;
    if (parallel) *parallel = s->stat_parallel;
    if (carried) *carried = s->stat_carried;
    return 0;
}

JDEFLATE_API int jdgpu_istream_queue(const JDGPUInflateStream* s)
{
    if (!s) return JDGPU_EINVAL;
    return s->own_q ? 1 : 0;
}

/* the one-shot forms: a whole stream, final input (the input ending before
 * the final block is INFLT_EINPUTEND); `window` (the dictionary, or the
 * output before a resume point) and bit0 start the decoder mid-stream */
static int stream_once(const uint8* window, uint64 wlen, uint32 bit0, const uint8* src,
                       uint64 srclen, uint64 region, uint8* dst, uint64 cap,
                       JDGPUInflateStep* res, uint32* crc, uint32* adler)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    if ((!src && srclen) || (!window && wlen) || (!dst && cap) || bit0 > 7 || (bit0 && !srclen))
        return JDGPU_EINVAL;
    hipStream_t st = e.stream;
    order(e, st);
    Fence f(e, st);
    JDGPUInflateStream s;
    (void) hipGetDevice(&s.dev);
    s.hs = st;
    IsLock lk(e, st, true);
    s.lk = &lk;
    int r = is_reset(&s, window, wlen, st);
    s.bit0 = bit0;
    if (!r) r = is_inflate(e, &s, src, srclen, region, dst, cap, res, crc, adler);
    (void) hipStreamSynchronize(st);
    is_free(&s);
    return r;
}

/* JDGPUInflateStep -> (error, produced, consumed) of the one-shot API:
 * ended -> 0; input exhausted -> INFLT_EINPUTEND; output full ->
 * JDGPU_EBLOCKOVERFLOW; else the inflator.h code */
static int32 once_error(const JDGPUInflateStep& s)
{
    switch (s.status) {
    case JDGPU_IS_ENDED: return 0;
    case JDGPU_IS_NEEDINPUT: return 6;
    case JDGPU_IS_FULL: return JDGPU_EBLOCKOVERFLOW;
    default: return s.error;
    }
}

JDEFLATE_API int jdgpu_inflate_resume(const uint8* window, uint32 wlen, const uint8* src,
                                      uint64 srclen, uint64 region, uint32 bit0, uint8* dst,
                                      uint64 cap, JDGPUInflateResult* res, uint64 csfrom,
                                      uint32* crc, uint32* adler)
{
    if (!res || csfrom) return JDGPU_EINVAL;
    JDGPUInflateStep s;
    memset(&s, 0, sizeof(s));
    const int r = stream_once(window, wlen, bit0, src, srclen, region, dst, cap, &s, crc, adler);
    memset(res, 0, sizeof(*res));
    res->produced = s.produced;
    res->error = once_error(s);
    res->consumed = s.consumed;
    res->parallel = s.parallel;
    /* a resume point only where the stream ended (its end); an input that
     * ran out leaves none -- the decoder state (tables, a half-read token)
     * is gone with this call: resumable decoding is jdgpu_istream_* */
    if (s.status == JDGPU_IS_ENDED) {
        res->resumebit = s.consumed * 8;
        res->resumeout = s.produced;
    }
    return r;
}

static int once(const uint8* dict, uint64 dsize, const uint8* src, uint64 srclen, uint64 region,
                uint8* dst, uint64 cap, uint64* produced, uint64* consumed, int32* error,
                uint32* crc, uint32* adler)
{
    JDGPUInflateStep s;
    memset(&s, 0, sizeof(s));
    const int r = stream_once(dict, dsize, 0, src, srclen, region, dst, cap, &s, crc, adler);
    if (produced) *produced = s.produced;
    if (consumed) *consumed = s.status == JDGPU_IS_ENDED ? s.consumed : 0;
    if (error) *error = once_error(s);
    return r;
}

JDEFLATE_API int jdgpu_inflate_flushed(const uint8* src, uint64 srclen, uint64 region, uint8* dst,
                                       uint64 cap, uint64* produced, uint64* consumed, int32* error,
                                       uint32* crc, uint32* adler)
{
    return once(nullptr, 0, src, srclen, region, dst, cap, produced, consumed, error, crc, adler);
}

JDEFLATE_API int jdgpu_inflate_stream(const uint8* src, uint64 srclen, uint8* dst, uint64 cap,
                                      uint64* produced, uint64* consumed, int32* error)
{
    return once(nullptr, 0, src, srclen, 0, dst, cap, produced, consumed, error, nullptr, nullptr);
}

JDEFLATE_API int jdgpu_inflate_stream_dict(const uint8* dict, uint64 dictsize, const uint8* src,
                                           uint64 srclen, uint8* dst, uint64 cap,
                                           uint64* produced, uint64* consumed, int32* error)
{
    return once(dict, dictsize, src, srclen, 0, dst, cap, produced, consumed, error, nullptr,
                nullptr);
}

JDEFLATE_API int jdgpu_inflate_stream_cs(const uint8* src, uint64 srclen, uint8* dst, uint64 cap,
                                         uint64* produced, uint64* consumed, int32* error,
                                         uint32* crc, uint32* adler)
{
    return once(nullptr, 0, src, srclen, 0, dst, cap, produced, consumed, error, crc, adler);
}

JDEFLATE_API struct JDEFLATEVersion jdeflate_getversion(void)
{
    struct JDEFLATEVersion v;
    v.major = JDEFLATE_VERSION_MAJOR;
    v.minor = JDEFLATE_VERSION_MINOR;
    v.patch = JDEFLATE_VERSION_PATCH;
    v.versionstring = JDEFLATE_VERSION_STRING;
    v.builddate = __DATE__;
    return v;
}

}  /* extern "C" */

/* Test hook (not in the public headers): run the deflate pipeline on host
 * data and return the parser's tokens, the per-block deflate-block table and
 * the match records, for diffing against the oracle's trace. */
extern "C" JDEFLATE_API int jdgpu_debug_deflate(const uint8* src, uint64 n, uint32 bs,
                                                int level, uint32* tokens, uint32* dbinfo,
                                                uint64* records)
{
    Engine& e = eng();
    std::lock_guard<std::mutex> g(e.mu);
    if (!ready(e)) return JDGPU_ENODEV;
    if (!valid_bs(bs) || level < 1 || level > 9) return JDGPU_EINVAL;
    const uint64_t nb = n ? (n + bs - 1) / bs : 1;
    if (nb > JD_CHUNK_BLOCKS) return JDGPU_EINVAL;
    const uint64_t bound = nb * slotcap_for(bs);
    if (!e.hin.ensure(n + 64) || !e.hout.ensure(bound + 64) || !e.hsz.ensure(nb * 4 + 64))
        return JDGPU_EOOM;
    hipStream_t st = e.stream;
    order(e, st);
    Fence fence(e, st);
    if (n && hipMemcpyAsync(e.hin.p, src, n, hipMemcpyHostToDevice, st) != hipSuccess)
        return JDGPU_ENODEV;
    int r = deflate_dev(e, e.hin.as<uint8_t>(), n, bs, level, 0, 1, e.hout.as<uint8_t>(), bound,
                        e.hsz.as<uint32_t>(), nullptr, nullptr, st);
    if (r) return r;
    if (tokens && hipMemcpyAsync(tokens, e.ds.tokens.p, nb * bs * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return JDGPU_ENODEV;
    if (dbinfo && hipMemcpyAsync(dbinfo, e.ds.dbinfo.p, nb * JD_DBSTRIDE * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
        return JDGPU_ENODEV;
    if (records && hipMemcpyAsync(records, e.ds.rec.p, nb * bs * 8, hipMemcpyDeviceToHost, st) != hipSuccess)
        return JDGPU_ENODEV;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : JDGPU_ENODEV;
}
