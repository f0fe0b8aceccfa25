/*
 * jd_multi.cpp -- the node-level path of SURVEY.md §8e for C callers: one
 * process drives several MI355X devices, with no torch and no launcher.
 *
 *   deflate: the blocks are cut into contiguous ranges, one per device; every
 *            device deflates its range with the block engine (block k of the
 *            last range alone ends with the caller's flush, every other range
 *            ends with FLUSH, so the concatenation is the single-device
 *            stream byte for byte); the per-device stream lengths are
 *            all-gathered (ncclAllGather) and the bitstreams gathered to the
 *            first device by one grouped ncclSend / ncclRecv into their final
 *            offsets -- the only exchange the path has.
 *   inflate: the size index gives every block's offset, so each device
 *            decodes its contiguous range of blocks on its own (no
 *            collective: there is no exchange step in inflate).
 *
 * RCCL is loaded at the first call (dlopen of librccl.so.1), so the library
 * keeps no link-time dependency on it and a host without it gets
 * JDGPU_ENODEV from these entry points only.  Reference: the caller-side
 * loop this replaces is deflator_deflate / inflator_inflate over a whole
 * buffer (/root/reference/jdeflate/deflator.h:106-153, inflator.h:97-153).
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <jdeflate/jdgpu.h>

#include <dlfcn.h>
#include <mutex>
#include <stdint.h>
#include <string.h>
#include <vector>

namespace {

struct Rccl {
    bool ok = false;
    ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
};

Rccl& rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        r.init_all = (decltype(r.init_all)) dlsym(h, "ncclCommInitAll");
        r.destroy = (decltype(r.destroy)) dlsym(h, "ncclCommDestroy");
        r.all_gather = (decltype(r.all_gather)) dlsym(h, "ncclAllGather");
        r.send = (decltype(r.send)) dlsym(h, "ncclSend");
        r.recv = (decltype(r.recv)) dlsym(h, "ncclRecv");
        r.group_start = (decltype(r.group_start)) dlsym(h, "ncclGroupStart");
        r.group_end = (decltype(r.group_end)) dlsym(h, "ncclGroupEnd");
        r.ok = r.init_all && r.destroy && r.all_gather && r.send && r.recv && r.group_start && r.group_end;
    });
    return r;
}

/* the devices to use: devs[0..ndev), or every visible device when ndev <= 0 */
int pick_devices(int ndev, const int* devs, std::vector<int>& out)
{
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0) return JDGPU_ENODEV;
    out.clear();
    if (ndev <= 0 || !devs) {
        for (int d = 0; d < cnt; d++) out.push_back(d);
    } else {
        for (int k = 0; k < ndev; k++) {
            if (devs[k] < 0 || devs[k] >= cnt) return JDGPU_EINVAL;
            for (int j = 0; j < k; j++)
                if (devs[j] == devs[k]) return JDGPU_EINVAL;      /* one rank per device */
            out.push_back(devs[k]);
        }
    }
    return 0;
}

/* per-device state of one call */
struct Part {
    int dev = 0;
    uint64_t b0 = 0, b1 = 0;            /* blocks [b0, b1)                   */
    uint64_t off = 0, len = 0;          /* input bytes [off, off + len)      */
    hipStream_t st = nullptr;
    void *in = nullptr, *out = nullptr, *csz = nullptr, *coff = nullptr, *tot = nullptr, *tots = nullptr;
    uint64_t outcap = 0;
    bool own_out = true;
};

void release(std::vector<Part>& ps)
{
    for (Part& p : ps) {
        if (hipSetDevice(p.dev) != hipSuccess) continue;
        if (p.st) (void) hipStreamSynchronize(p.st);
        void* bufs[] = {p.in, p.csz, p.coff, p.tot, p.tots};
        for (void* b : bufs)
            if (b) (void) hipFree(b);
        if (p.out && p.own_out) (void) hipFree(p.out);
        if (p.st) (void) hipStreamDestroy(p.st);
        p = Part{};
    }
}

/* contiguous block ranges, nb = max(1, ceil(n / bs)) blocks over the devices */
void split(std::vector<Part>& ps, const std::vector<int>& devs, uint64_t n, uint32_t bs)
{
    const uint64_t nb = n ? (n + bs - 1) / bs : 1;
    const uint64_t k = devs.size();
    ps.assign(k, Part{});
    for (uint64_t i = 0; i < k; i++) {
        Part& p = ps[i];
        p.dev = devs[i];
        p.b0 = nb * i / k;
        p.b1 = nb * (i + 1) / k;
        p.off = p.b0 * bs;
        const uint64_t e = p.b1 * bs < n ? p.b1 * bs : n;
        p.len = e > p.off ? e - p.off : 0;
    }
}

#define CK(x)                                   \
    do {                                        \
        if ((x) != hipSuccess) {                \
            release(ps);                        \
            return JDGPU_ENODEV;                \
        }                                       \
    } while (0)

/* the shared body of jdgpu_deflate_multi[_device]: the gathered stream ends
 * up in d_out0 (device memory on the first device) or, when that is NULL, in
 * the host buffer dst */
int64_t deflate_multi(const uint8_t* src, uint64_t n, uint32_t bs, int level, uint32_t flags,
                      int lastflush, int ndev, const int* devs, void* d_out0, uint64_t outcap,
                      uint8_t* dst, uint32_t* csizes)
{
    if ((!src && n) || bs < 16 || bs > 65536 || (bs & 15) || level < 0 || level > 9 ||
        (lastflush != 1 && lastflush != 2) || (!d_out0 && !dst))
        return JDGPU_EINVAL;
    std::vector<int> dv;
    int r = pick_devices(ndev, devs, dv);
    if (r) return r;
    Rccl& R = rccl();
    if (!R.ok) return JDGPU_ENODEV;
    std::vector<Part> ps;
    split(ps, dv, n, bs);
    const int K = (int) ps.size();
    /* the last device with blocks carries the caller's flush */
    int last = 0;
    for (int i = 0; i < K; i++)
        if (ps[i].b1 > ps[i].b0) last = i;
    for (int i = 0; i < K; i++) {
        Part& p = ps[i];
        CK(hipSetDevice(p.dev));
        CK(hipStreamCreateWithFlags(&p.st, hipStreamNonBlocking));
        CK(hipMalloc(&p.tot, 64));
        CK(hipMalloc(&p.tots, 8 * (size_t) K + 64));
        CK(hipMemsetAsync(p.tot, 0, 8, p.st));
        if (p.b1 == p.b0) continue;
        const uint64_t nbk = p.b1 - p.b0;
        p.outcap = jdgpu_bound(p.len, bs);
        if (i == 0 && d_out0 && outcap >= p.outcap) {
            p.out = d_out0;                     /* first range: in place */
            p.own_out = false;
        } else {
            CK(hipMalloc(&p.out, p.outcap + 64));
        }
        CK(hipMalloc(&p.in, p.len + 64));
        CK(hipMalloc(&p.csz, nbk * 4 + 64));
        CK(hipMalloc(&p.coff, nbk * 8 + 64));
        if (p.len) CK(hipMemcpyAsync(p.in, src + p.off, p.len, hipMemcpyHostToDevice, p.st));
        r = jdgpu_deflate_device(p.in, p.len, bs, level, flags, i == last ? lastflush : 2, p.out, p.outcap,
                                 (uint32*) p.csz, (uint64*) p.coff, (uint64*) p.tot, p.st);
        if (r) {
            release(ps);
            return r;
        }
    }
    /* one communicator per device, all in this process */
    std::vector<ncclComm_t> comm(K);
    if (R.init_all(comm.data(), K, dv.data()) != ncclSuccess) {
        release(ps);
        return JDGPU_ENODEV;
    }
    auto fail = [&](int code) -> int64_t {
        for (auto c : comm) (void) R.destroy(c);
        release(ps);
        return code;
    };
    /* every device learns every range's stream length */
    if (R.group_start() != ncclSuccess) return fail(JDGPU_ENODEV);
    for (int i = 0; i < K; i++)
        if (R.all_gather(ps[i].tot, ps[i].tots, 1, ncclUint64, comm[i], ps[i].st) != ncclSuccess) {
            (void) R.group_end();
            return fail(JDGPU_ENODEV);
        }
    if (R.group_end() != ncclSuccess) return fail(JDGPU_ENODEV);
    std::vector<uint64_t> tl(K);
    if (hipSetDevice(ps[0].dev) != hipSuccess ||
        hipMemcpyAsync(tl.data(), ps[0].tots, 8 * (size_t) K, hipMemcpyDeviceToHost, ps[0].st) != hipSuccess ||
        hipStreamSynchronize(ps[0].st) != hipSuccess)
        return fail(JDGPU_ENODEV);
    std::vector<uint64_t> off(K + 1, 0);
    for (int i = 0; i < K; i++) off[i + 1] = off[i] + tl[i];
    const uint64_t total = off[K];
    if (total > outcap) return fail(JDGPU_ECAP);
    /* the gather: range i's bitstream to the first device at off[i] */
    void* g = d_out0;
    bool own_g = false;
    if (!g) {
        if (hipSetDevice(ps[0].dev) != hipSuccess || hipMalloc(&g, total + 64) != hipSuccess)
            return fail(JDGPU_EOOM);
        own_g = true;
    }
    auto fail_g = [&](int code) -> int64_t {
        if (own_g) {
            (void) hipSetDevice(ps[0].dev);
            (void) hipFree(g);
        }
        return fail(code);
    };
    if (tl[0] && ps[0].out != g) {
        if (hipSetDevice(ps[0].dev) != hipSuccess ||
            hipMemcpyAsync(g, ps[0].out, tl[0], hipMemcpyDeviceToDevice, ps[0].st) != hipSuccess)
            return fail_g(JDGPU_ENODEV);
    }
    if (R.group_start() != ncclSuccess) return fail_g(JDGPU_ENODEV);
    for (int i = 1; i < K; i++) {
        if (!tl[i]) continue;
        if (R.send(ps[i].out, tl[i], ncclUint8, 0, comm[i], ps[i].st) != ncclSuccess ||
            R.recv((uint8_t*) g + off[i], tl[i], ncclUint8, i, comm[0], ps[0].st) != ncclSuccess) {
            (void) R.group_end();
            return fail_g(JDGPU_ENODEV);
        }
    }
    if (R.group_end() != ncclSuccess) return fail_g(JDGPU_ENODEV);
    /* the size index and (host output) the stream */
    for (int i = 0; i < K; i++) {
        Part& p = ps[i];
        if (hipSetDevice(p.dev) != hipSuccess) return fail_g(JDGPU_ENODEV);
        if (csizes && p.b1 > p.b0 &&
            hipMemcpyAsync(csizes + p.b0, p.csz, (p.b1 - p.b0) * 4, hipMemcpyDeviceToHost, p.st) != hipSuccess)
            return fail_g(JDGPU_ENODEV);
        if (hipStreamSynchronize(p.st) != hipSuccess) return fail_g(JDGPU_ENODEV);
    }
    if (!d_out0) {
        if (hipSetDevice(ps[0].dev) != hipSuccess ||
            (total && hipMemcpy(dst, g, total, hipMemcpyDeviceToHost) != hipSuccess))
            return fail_g(JDGPU_ENODEV);
    }
    if (own_g) {
        (void) hipSetDevice(ps[0].dev);
        (void) hipFree(g);
    }
    for (auto c : comm) (void) R.destroy(c);
    release(ps);
    return (int64_t) total;
}

}  // namespace

extern "C" {

JDEFLATE_API int64 jdgpu_deflate_multi(const uint8* src, uint64 n, uint32 blocksize, int level,
                                       uint32 flags, int lastflush, uint8* dst, uint64 cap,
                                       uint32* csizes, int ndev, const int* devs)
{
    int cur = 0;
    (void) hipGetDevice(&cur);
    const int64_t r = deflate_multi(src, n, blocksize, level, flags, lastflush, ndev, devs, nullptr, cap,
                                    dst, csizes);
    (void) hipSetDevice(cur);
    return r;
}

JDEFLATE_API int jdgpu_deflate_multi_device(const uint8* src, uint64 n, uint32 blocksize, int level,
                                            uint32 flags, int lastflush, void* d_out0, uint64 outcap,
                                            uint64* total, uint32* csizes, int ndev, const int* devs)
{
    if (!d_out0 || !total) return JDGPU_EINVAL;
    int cur = 0;
    (void) hipGetDevice(&cur);
    const int64_t r = deflate_multi(src, n, blocksize, level, flags, lastflush, ndev, devs, d_out0, outcap,
                                    nullptr, csizes);
    (void) hipSetDevice(cur);
    if (r < 0) return (int) r;
    *total = (uint64) r;
    return 0;
}

JDEFLATE_API int jdgpu_inflate_multi(const uint8* src, uint64 srclen, const uint32* csizes,
                                     uint32 nblocks, uint32 blocksize, uint8* dst, uint32* usizes,
                                     int32* errors, int ndev, const int* devs)
{
    if (!src || !csizes || !nblocks || !dst || !usizes || !errors || blocksize < 16 || blocksize > 65536 ||
        (blocksize & 15))
        return JDGPU_EINVAL;
    std::vector<int> dv;
    int r = pick_devices(ndev, devs, dv);
    if (r) return r;
    std::vector<uint64_t> coff(nblocks + 1, 0);
    for (uint32_t i = 0; i < nblocks; i++) coff[i + 1] = coff[i] + csizes[i];
    if (coff[nblocks] > srclen) return JDGPU_EINVAL;
    int cur = 0;
    (void) hipGetDevice(&cur);
    std::vector<Part> ps;
    split(ps, dv, (uint64_t) nblocks * blocksize, blocksize);
    std::vector<std::vector<uint64_t>> los(ps.size());   /* live until the copies land */
    for (size_t i = 0; i < ps.size(); i++) {
        Part& p = ps[i];
        if (p.b1 == p.b0) continue;
        const uint64_t nbk = p.b1 - p.b0, c0 = coff[p.b0], clen = coff[p.b1] - c0;
        CK(hipSetDevice(p.dev));
        CK(hipStreamCreateWithFlags(&p.st, hipStreamNonBlocking));
        CK(hipMalloc(&p.in, clen + 64));
        CK(hipMalloc(&p.out, nbk * blocksize + 64));
        CK(hipMalloc(&p.csz, nbk * 4 + 64));
        CK(hipMalloc(&p.coff, nbk * 8 + 64));
        CK(hipMalloc(&p.tot, nbk * 8 + 64));            /* usizes + errors */
        std::vector<uint64_t>& lo = los[i];
        lo.resize(nbk);
        for (uint64_t j = 0; j < nbk; j++) lo[j] = coff[p.b0 + j] - c0;
        if (clen) CK(hipMemcpyAsync(p.in, src + c0, clen, hipMemcpyHostToDevice, p.st));
        CK(hipMemcpyAsync(p.csz, csizes + p.b0, nbk * 4, hipMemcpyHostToDevice, p.st));
        CK(hipMemcpyAsync(p.coff, lo.data(), nbk * 8, hipMemcpyHostToDevice, p.st));
        r = jdgpu_inflate_device(p.in, clen, (const uint64*) p.coff, (const uint32*) p.csz, (uint32) nbk,
                                 blocksize, p.out, (uint32*) p.tot, (int32*) ((uint32_t*) p.tot + nbk), p.st);
        if (r) {
            release(ps);
            (void) hipSetDevice(cur);
            return r;
        }
    }
    int bad = 0;
    for (Part& p : ps) {
        if (p.b1 == p.b0) continue;
        const uint64_t nbk = p.b1 - p.b0;
        CK(hipSetDevice(p.dev));
        CK(hipStreamSynchronize(p.st));
        CK(hipMemcpy(dst + p.b0 * blocksize, p.out, nbk * blocksize, hipMemcpyDeviceToHost));
        CK(hipMemcpy(usizes + p.b0, p.tot, nbk * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(errors + p.b0, (uint32_t*) p.tot + nbk, nbk * 4, hipMemcpyDeviceToHost));
        for (uint64_t j = 0; j < nbk; j++) bad |= errors[p.b0 + j] != 0;
    }
    release(ps);
    (void) hipSetDevice(cur);
    return bad ? JDGPU_EDATA : 0;
}

}  // extern "C"
