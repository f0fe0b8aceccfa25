"""Benchmark: level-6 deflate + inflate of 64 KiB independent blocks on MI355X.

Workload (BASELINE.json configs[1]/[2], SURVEY.md §8d C2+C3): 1 GiB of
synthetic Zipf text per GPU, cut into 16,384 independent 64 KiB blocks,
deflated at level 6 (bit-identical to the reference deflator per block) and
inflated back, inputs resident in HBM.  One step = deflate of the shard +
(N > 1: RCCL gather of the per-block bitstreams to rank 0) + inflate of the
shard.  value = bytes of all shards / (time of the step) in MB/s (1e6 B/s).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--size BYTES] [--level L]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N,
  or bench.py --gpus N alone (it launches the N ranks itself).
  Default size per GPU: 1 GiB at N=1 (configs[1]); 8 GiB at N>1, so that N=8
  is configs[3] (64 GiB over 8 GPUs, 131,072 blocks per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "deflate+inflate MB/s at level 6, 64 KiB blocks; ratio vs reference"


def metric_for(level: int) -> str:
    """BASELINE.json's metric string, with the level the run actually used"""
    return METRIC if level == 6 else METRIC.replace("level 6", f"level {level}")
HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E, MI355X_MICROARCH.md
BS = 65536


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=0,
                    help="input bytes per GPU (default: 1 GiB at N=1, configs[1]; 8 GiB per GPU "
                         "at N>1, so N=8 is configs[3]: 64 GiB over 8 GPUs)")
    ap.add_argument("--level", type=int, default=6)
    ap.add_argument("--corpus", choices=("text", "mixed"), default="text")
    ap.add_argument("--no-gather", action="store_true", help="skip the RCCL bitstream gather")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-host-api", action="store_true",
                    help="skip the PCIe-inclusive host-API rate (profiling passes: keeps every "
                         "launch of a kernel at the bench size)")
    ap.add_argument("--cpu-sample", type=int, default=256 << 20)
    ap.add_argument("--stream-sample", type=int, default=256 << 20,
                    help="bytes for the drop-in inflator's 32 KiB-read rate")
    ap.add_argument("--foreign-sample", type=int, default=128 << 20,
                    help="bytes of the zlib-made stream for the marker-free decode rate")
    return ap.parse_args()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_quota():
    """CPUs the cgroup grants this process (cpu.max), or None"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(data_np, level, sample_bytes):
    """Oracle restatement (port) on the host cores: 1 thread, and one thread
    per CPU this process may actually use: min(online CPUs (sysconf
    _SC_NPROCESSORS_ONLN), the cgroup's CPU quota, the
    affinity mask).  On the GPU box the sysconf count is the whole machine's
    (256) while the quota is 16, so 256 threads would only time-slice 16 CPUs."""
    import ctypes
    import numpy as np
    from oracle import jdoracle as O

    L = O.lib()
    online = max(1, os.sysconf("SC_NPROCESSORS_ONLN"))
    q = cpu_quota()
    threads = min(online, len(os.sched_getaffinity(0)), int(q) if q and q >= 1 else online)
    res = {}
    for nt, nbytes in ((1, min(sample_bytes // 4, 64 << 20)), (threads, sample_bytes)):
        n = min(nbytes, data_np.size) // BS * BS
        src = np.ascontiguousarray(data_np[:n])
        nb = n // BS
        slot = O.lib().jdo_bound(BS) + 64
        dst = np.empty(nb * slot, dtype=np.uint8)
        sizes = (ctypes.c_uint32 * nb)()
        t0 = time.perf_counter()
        tot = L.jdo_deflate_blocks_mt(src.ctypes.data, n, BS, level, dst.ctypes.data, slot,
                                      sizes, nt)
        t1 = time.perf_counter()
        offs = (ctypes.c_uint64 * nb)(*[i * slot for i in range(nb)])
        back = np.empty(n, dtype=np.uint8)
        bad = L.jdo_inflate_blocks_mt(dst.ctypes.data, offs, sizes, nb, BS, back.ctypes.data, nt)
        t2 = time.perf_counter()
        if bad or not np.array_equal(back, src):
            raise RuntimeError("CPU baseline round trip failed")
        res[nt] = dict(n=n, td=t1 - t0, ti=t2 - t1, ratio=tot / n)
    one, allc = res[1], res[threads]
    return {
        "value": round(allc["n"] / (allc["td"] + allc["ti"]) / 1e6, 2),
        "unit": "MB/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{allc['n'] >> 20} MiB of the same corpus, {allc['n'] // BS} blocks, "
                   f"level {level} deflate+inflate, oracle/jdoracle.c restatement, "
                   f"{threads} pthreads = min(online CPUs {online}, cgroup quota {q}, "
                   f"affinity {len(os.sched_getaffinity(0))}) on {cpu_model()}; "
                   f"deflate {allc['n'] / allc['td'] / 1e6:.1f} MB/s, "
                   f"inflate {allc['n'] / allc['ti'] / 1e6:.1f} MB/s; 1 thread on "
                   f"{one['n'] >> 20} MiB: {one['n'] / (one['td'] + one['ti']) / 1e6:.1f} MB/s"),
        "cpu_model": cpu_model(),
        "online_cpus": online,
        "cgroup_cpus": q,
        "effective_cores": threads,
        "value_1thread": round(one["n"] / (one["td"] + one["ti"]) / 1e6, 2),
        "deflate_1thread_MBps": round(one["n"] / one["td"] / 1e6, 2),
        "inflate_1thread_MBps": round(one["n"] / one["ti"] / 1e6, 2),
    }


def host_api_rate(J, host, level, nbytes):
    """PCIe-inclusive rate of the host-buffer entry points (jdgpu_deflate /
    jdgpu_inflate: H2D copy, kernels, D2H copy) on a slice of the same data.
    Reported beside the HBM-resident value, never as it."""
    import ctypes
    import numpy as np
    L = J.load_library()
    n = min(nbytes, host.size) // BS * BS
    nb = n // BS
    src = np.ascontiguousarray(host[:n])
    cap = J.bound(n)
    out = np.empty(cap, dtype=np.uint8)
    sizes = np.empty(nb, dtype=np.uint32)
    back = np.empty(n, dtype=np.uint8)
    us = np.empty(nb, dtype=np.uint32)
    er = np.empty(nb, dtype=np.int32)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    i32p = ctypes.POINTER(ctypes.c_int32)
    best_d = best_i = None
    for _ in range(2):
        t0 = time.perf_counter()
        c = L.jdgpu_deflate(ctypes.c_char_p(src.ctypes.data), n, BS, level, 0, 1,
                            out.ctypes.data, cap, sizes.ctypes.data_as(u32p))
        t1 = time.perf_counter()
        r = L.jdgpu_inflate(ctypes.c_char_p(out.ctypes.data), c, sizes.ctypes.data_as(u32p), nb,
                            BS, back.ctypes.data, us.ctypes.data_as(u32p), er.ctypes.data_as(i32p))
        t2 = time.perf_counter()
        if c < 0 or r != 0 or not np.array_equal(back, src):
            raise RuntimeError("host-API round trip failed")
        best_d = min(best_d or 1e9, t1 - t0)
        best_i = min(best_i or 1e9, t2 - t1)
    return {"bytes": n, "deflate_MBps": round(n / best_d / 1e6, 2),
            "inflate_MBps": round(n / best_i / 1e6, 2),
            "roundtrip_MBps": round(n / (best_d + best_i) / 1e6, 2)}


def checksum_rate(J, d_in, n, host, stream):
    """k_checksum (the zstrm CRC-32 / Adler-32 scan) on
    the HBM-resident input: GB/s of N read, against the HBM roofline.  The
    first and last blocks are checked against zlib."""
    import zlib
    import numpy as np
    import torch
    L = J.load_library()
    nb = -(-n // BS)
    out = torch.zeros(3 * nb, dtype=torch.int32, device=d_in.device)
    for _ in range(2):
        L.jdgpu_checksum_device(d_in.data_ptr(), n, BS, out.data_ptr(), stream)
    torch.cuda.synchronize()
    J.prof_enable(True)
    reps = 5
    for _ in range(reps):
        if L.jdgpu_checksum_device(d_in.data_ptr(), n, BS, out.data_ptr(), stream):
            raise RuntimeError("jdgpu_checksum_device failed")
    torch.cuda.synchronize()
    ms = J.prof_read()["k_checksum"][0] / reps
    J.prof_enable(False)
    got = out.cpu().numpy().astype(np.uint32).reshape(nb, 3)
    ok = True
    for b in (0, nb - 1):
        blk = host[b * BS:(b + 1) * BS].tobytes()
        r0 = zlib.crc32(blk) ^ 0xFFFFFFFF ^ J.crc32_combine(0xFFFFFFFF, 0, len(blk))
        ok &= int(got[b, 0]) == r0 and int(got[b, 1]) == sum(blk) % 65521
    gbps = n / (ms / 1e3) / 1e9
    return {"kernel": "k_checksum", "avg_launch_ms": round(ms, 3), "GBps": round(gbps, 1),
            "roofline_frac": round(gbps / HBM_PEAK_GBPS, 4), "ok": bool(ok)}


def dropin_rate(J, host, level, nbytes):
    """PCIe-inclusive rate of the drop-in C API itself (deflator_* /
    inflator_*, jdeflate/deflator.h and inflator.h, north_star's product
    entry): one deflator_deflate(DEFLT_END) over a host buffer, then one
    inflator_inflate(final=1) of the result, targets large enough for one
    call each; output checked."""
    import ctypes
    import numpy as np
    from jdeflate_amd import engine as E
    L = J.load_library()
    n = min(nbytes, host.size)
    src = np.ascontiguousarray(host[:n])
    cap = J.bound(n)
    comp = np.empty(cap, dtype=np.uint8)
    back = np.empty(n + 64, dtype=np.uint8)
    best_d = best_i = None
    for _ in range(2):
        d = L.deflator_create(0, level, None)
        p = d.contents
        p.source = p.sbgn = src.ctypes.data
        p.send = src.ctypes.data + n
        p.target = p.tbgn = comp.ctypes.data
        p.tend = comp.ctypes.data + cap
        t0 = time.perf_counter()
        r = L.deflator_deflate(d, E.DEFLT_END)
        t1 = time.perf_counter()
        c = p.target - p.tbgn
        L.deflator_destroy(d)
        i = L.inflator_create(0, None)
        q = i.contents
        q.source = q.sbgn = comp.ctypes.data
        q.send = comp.ctypes.data + c
        q.target = q.tbgn = back.ctypes.data
        q.tend = back.ctypes.data + back.size
        t2 = time.perf_counter()
        ri = L.inflator_inflate(i, 1)
        t3 = time.perf_counter()
        m = q.target - q.tbgn
        L.inflator_destroy(i)
        if r != E.DEFLT_OK or ri != E.INFLT_OK or m != n or not np.array_equal(back[:n], src):
            raise RuntimeError(f"drop-in round trip failed ({r}, {ri}, {m})")
        best_d = min(best_d or 1e9, t1 - t0)
        best_i = min(best_i or 1e9, t3 - t2)
    return {"bytes": n, "deflate_MBps": round(n / best_d / 1e6, 2),
            "inflate_MBps": round(n / best_i / 1e6, 2)}


def _dropin_compress(J, host, level, nbytes):
    """the drop-in deflator's stream of the first nbytes (DEFLT_END)"""
    import numpy as np
    from jdeflate_amd import engine as E
    L = J.load_library()
    n = min(nbytes, host.size)
    src = np.ascontiguousarray(host[:n])
    cap = J.bound(n)
    comp = np.empty(cap, dtype=np.uint8)
    d = L.deflator_create(0, level, None)
    p = d.contents
    p.source = p.sbgn = src.ctypes.data
    p.send = src.ctypes.data + n
    p.target = p.tbgn = comp.ctypes.data
    p.tend = comp.ctypes.data + cap
    r = L.deflator_deflate(d, E.DEFLT_END)
    c = p.target - p.tbgn
    L.deflator_destroy(d)
    if r != E.DEFLT_OK:
        raise RuntimeError(f"drop-in deflate failed ({r})")
    return src, comp, c


def _dropin_decode(L, comp, c, back, piece, tgt):
    """one drop-in inflator fed `piece`-byte reads, final = 0 on every call,
    each drained through a `tgt`-byte target; -> (result, bytes, calls)"""
    from jdeflate_amd import engine as E
    i = L.inflator_create(0, None)
    q = i.contents
    got = 0
    calls = 0
    ri = E.INFLT_SRCEXHSTD
    for off in range(0, c, piece):
        m = min(piece, c - off)
        q.source = q.sbgn = comp.ctypes.data + off
        q.send = comp.ctypes.data + off + m
        while True:
            q.target = q.tbgn = back.ctypes.data + got
            q.tend = back.ctypes.data + got + tgt
            ri = L.inflator_inflate(i, 0)
            calls += 1
            got += q.target - q.tbgn
            if ri != E.INFLT_TGTEXHSTD:
                break
        if ri != E.INFLT_SRCEXHSTD:
            break
    L.inflator_destroy(i)
    return ri, got, calls


def dropin_stream_rate(J, host, level, nbytes, piece=32768, tgt=65536):
    """PCIe-inclusive rate of the drop-in inflator fed the way zstrm.c:900-930
    feeds it in callback mode: the compressed stream (this library's
    FLUSH-joined 64 KiB blocks, one deflator_deflate(DEFLT_END)) handed over
    in `piece`-byte reads with final=0 on every call, each drained through a
    `tgt`-byte target.  The resumable decoder keeps its state on the device,
    so each call decodes only its new bytes (64 lanes by self-synchronising
    walks, k_inflate_rpar; block-parallel from a sync marker once >= 128 KiB
    are at hand)."""
    import numpy as np
    from jdeflate_amd import engine as E
    L = J.load_library()
    src, comp, c = _dropin_compress(J, host, level, nbytes)
    n = src.size
    back = np.empty(n + tgt, dtype=np.uint8)
    t0 = time.perf_counter()
    ri, got, calls = _dropin_decode(L, comp, c, back, piece, tgt)
    t1 = time.perf_counter()
    if ri != E.INFLT_OK or got != n or not np.array_equal(back[:n], src):
        raise RuntimeError(f"drop-in chunked inflate failed ({ri}, {got})")
    return {"bytes": n, "compressed": c, "piece": piece, "target": tgt, "calls": calls,
            "inflate_MBps": round(n / (t1 - t0) / 1e6, 2)}


def dropin_stream_mt_rate(J, host, level, nbytes, threads=8, piece=32768, tgt=65536):
    """The same 32 KiB-read pattern on `threads` drop-in inflators at once,
    one per thread (the reference's threading model: independent instances,
    inflator.h): each instance has its own HIP stream and device state, and
    the engine lock is taken only around shared workspace, so the instances'
    kernels overlap.  Whole-job rate of all instances, and the rate of one
    instance alone on the same stream."""
    import threading
    import numpy as np
    from jdeflate_amd import engine as E
    L = J.load_library()
    src, comp, c = _dropin_compress(J, host, level, nbytes)
    n = src.size
    backs = [np.empty(n + tgt, dtype=np.uint8) for _ in range(threads)]
    t0 = time.perf_counter()
    r1 = _dropin_decode(L, comp, c, backs[0], piece, tgt)
    t1 = time.perf_counter()
    res = [None] * threads

    def work(k):
        res[k] = _dropin_decode(L, comp, c, backs[k], piece, tgt)

    ths = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    t2 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    t3 = time.perf_counter()
    ok = r1[0] == E.INFLT_OK and all(r is not None and r[0] == E.INFLT_OK and r[1] == n for r in res)
    ok = ok and all(np.array_equal(b[:n], src) for b in backs)
    if not ok:
        raise RuntimeError("multi-instance drop-in inflate failed")
    one = n / (t1 - t0) / 1e6
    many = threads * n / (t3 - t2) / 1e6
    return {"bytes_per_instance": n, "instances": threads, "threads": threads, "piece": piece,
            "target": tgt, "one_instance_MBps": round(one, 2), "all_instances_MBps": round(many, 2),
            "speedup": round(many / one, 2)}


def foreign_stream_rate(J, host, nbytes):
    """PCIe-inclusive rate of jdgpu_istream_inflate on a stream it did not
    make: zlib's default output (level 6, no sync markers) of `nbytes` of the
    corpus, handed over in one call.  The decoder cuts it at block headers it
    finds itself and decodes the chunks in parallel (k_fsp_*)."""
    import ctypes
    import zlib
    from jdeflate_amd import engine as E
    n = min(nbytes, host.size)
    data = host[:n].tobytes()
    c = zlib.compressobj(6, zlib.DEFLATED, -15)
    comp = c.compress(data) + c.flush()
    src = ctypes.create_string_buffer(comp, len(comp))
    out = ctypes.create_string_buffer(n + 1)
    s = E.IStream()
    s.inflate(len(comp), n + 1, src_addr=ctypes.addressof(src), out=out)     # warm
    s.close()
    s = E.IStream()
    t0 = time.perf_counter()
    st, err, prod, used, _ = s.inflate(len(comp), n + 1, src_addr=ctypes.addressof(src), out=out)
    t1 = time.perf_counter()
    rounds, chunks = s.fsp()
    s.close()
    if st != E.IS_ENDED or prod != n or out.raw[:n] != data:
        raise RuntimeError(f"foreign stream inflate failed ({st}, {err}, {prod})")
    return {"bytes": n, "compressed": len(comp), "maker": "zlib level 6, one stream",
            "rounds": rounds, "chunks": chunks, "inflate_MBps": round(n / (t1 - t0) / 1e6, 1)}


def zstrm_rate(J, host, level, nbytes):
    """PCIe-inclusive rate of the zstrm gzip container:
    zstrm_deflate of the whole buffer + zstrm_flush (the compressed bytes
    leave through the target callback in 32 KiB writes, as the reference's
    do), then zstrm_inflate of the container from a buffer source into one
    target (index-free parallel decode of the FLUSH-joined blocks, f4),
    CRC-32 scanned on the device."""
    import ctypes
    import numpy as np
    from jdeflate_amd import engine as E
    L = J.load_library()
    n = min(nbytes, host.size)
    src = np.ascontiguousarray(host[:n])
    comp = np.empty(J.bound(n) + 64, dtype=np.uint8)
    back = np.empty(n + 64, dtype=np.uint8)
    best_d = best_i = None
    base = comp.ctypes.data

    class Sink(ctypes.Structure):
        _fields_ = [("base", ctypes.c_void_p), ("cap", ctypes.c_size_t), ("pos", ctypes.c_size_t)]
    helper = os.path.join(ROOT, "tools", "libbenchsink.so")
    for _ in range(2):
        pos = [0]

        def ofn(buf, size, user):
            ctypes.memmove(base + pos[0], buf, size)
            pos[0] += size
            return size
        z = L.zstrm_create(E.ZSTRM_DEFLATE | E.ZSTRM_GZIP, level, None)
        sink = Sink(base, comp.size, 0)
        if os.path.exists(helper):
            # a C callback, as a C caller of zstrm would have (tools/benchsink.c)
            cb = ctypes.cast(ctypes.CDLL(helper).bench_sink_write, E.ZSTRM_OFN)
            L.zstrm_settargetfn(z, cb, ctypes.byref(sink))
        else:
            cb = E.ZSTRM_OFN(ofn)
            L.zstrm_settargetfn(z, cb, None)
        t0 = time.perf_counter()
        L.zstrm_deflate(z, src.ctypes.data, n)
        L.zstrm_flush(z, 1)
        t1 = time.perf_counter()
        err = z.contents.error
        L.zstrm_destroy(z)
        c = sink.pos if os.path.exists(helper) else pos[0]
        zi = L.zstrm_create(E.ZSTRM_INFLATE, 0, None)
        t2 = time.perf_counter()
        L.zstrm_setsource(zi, base, c)
        m = L.zstrm_inflate(zi, back.ctypes.data, n + 1)
        t3 = time.perf_counter()
        erri = zi.contents.error
        L.zstrm_destroy(zi)
        if err or erri or m != n or not np.array_equal(back[:n], src):
            raise RuntimeError(f"zstrm gzip round trip failed ({err}, {erri}, {m})")
        best_d = min(best_d or 1e9, t1 - t0)
        best_i = min(best_i or 1e9, t3 - t2)
    return {"bytes": n, "deflate_MBps": round(n / best_d / 1e6, 2),
            "inflate_MBps": round(n / best_i / 1e6, 2)}


def pmc_traffic(kernel, level, size, corpus="text"):
    """HBM bytes per launch from a committed rocprofv3 PMC summary taken on
    this exact workload (profiles/pmc_summary*.json: C2+C3, C5, ...)."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_summary*.json"))):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        text = "Zipf text" in (w.get("workload") or "")
        # a kernel template is named with its arguments (k_match<false>)
        ks = [k for k in d.get("kernels", {}) if k.split("<")[0] == kernel]
        if w.get("level") == level and w.get("bytes") == size and text == (corpus == "text") and ks:
            src = (f"profiles/{os.path.basename(p)} (tag {d.get('tag')}, {ks[0]}, "
                   f"{d.get('command', '?')})")
            return d["kernels"][ks[0]].get("hbm_bytes_per_launch"), src
    return None, None


CLOCK_HZ = 2.4e9          # MI355X peak engine clock (MI355X_MICROARCH.md)
SIMDS = 1024              # 256 CUs x 4 SIMD-32
VALU_PEAK = 0.5           # wave64 VALU instructions per SIMD per cycle (2 cycles each)


def sq_compute(kt, steps, level, size, corpus="text", min_ms=1.0):
    """The compute side of the roofline, per kernel taking >= min_ms per
    step: VALU wave-instructions per SIMD per cycle against the wave64 peak,
    LDS instructions per CU per cycle, lanes active per VALU instruction and
    the share of wave cycles parked in s_waitcnt (SQ_WAIT_ANY), from the
    committed SQ counter summary of this exact workload
    (profiles/sq_summary*.json, tools/prof_counters.sh) over this run's
    per-launch kernel times (the engine's HIP events)."""
    import glob
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "sq_summary*.json"))):
        try:
            with open(p) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        w = d.get("workload", {})
        if (w.get("bytes"), w.get("level"), w.get("corpus")) != (size, level, corpus):
            continue
        out = {"source": f"profiles/{os.path.basename(p)} (tag {d.get('tag')})",
               "clock_hz": CLOCK_HZ, "valu_peak_per_simd_cycle": VALU_PEAK}
        for name, (ms, cnt) in kt.items():
            if not cnt or ms / steps < min_ms:
                continue
            ks = [k for k in d.get("kernels", {}) if k.split("<")[0] == name.split("<")[0] and
                  (("<" not in name) or k.startswith(name.replace(">", "")))]
            if not ks:
                continue
            c = d["kernels"][ks[0]]
            t = ms / cnt / 1e3                                   # seconds per launch
            cyc = t * CLOCK_HZ
            valu = c.get("SQ_INSTS_VALU", 0.0)
            lds = c.get("SQ_INSTS_LDS", 0.0)
            wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
            out[name] = {
                "counters": ks[0],
                "valu_per_simd_cycle": round(valu / (cyc * SIMDS), 4),
                "valu_frac": round(valu / (cyc * SIMDS) / VALU_PEAK, 4),
                "lds_per_cu_cycle": round(lds / (cyc * SIMDS / 4), 4),
                "lanes_per_valu": round(c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (valu or 1.0), 1),
                "wait_any_frac": round(c.get("SQ_WAIT_ANY", 0.0) / wc, 3),
                "active_frac": round(c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, 3),
            }
        return out
    return None


def workload_name(args, n, nb, world):
    what = ("Zipf text" if args.corpus == "text" else "Silesia-like mixed-entropy")
    tag = ("C4" if world > 1 and args.corpus == "text" else
           "C2+C3" if args.corpus == "text" else "C5" if args.level == 9 else "mixed")
    return (f"{tag}: {n >> 20} MiB {what} per GPU x {world} GPU(s), {nb} independent 64 KiB "
            f"blocks per GPU, level {args.level} deflate then inflate, HBM-resident")


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start the N ranks as child
    processes (torch.distributed.run) before this process touches the GPU,
    and exit with their status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if not args.size:
        args.size = (1 << 30) if args.gpus == 1 else (8 << 30)
    import numpy as np
    import torch
    import torch.distributed as dist
    import jdeflate_amd as J
    from jdeflate_amd import dist as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if not J.available():
        raise SystemExit("HIP engine unavailable (no gfx950 device or library not built)")

    n = args.size // BS * BS
    nb = n // BS
    gen = J.corpus_text if args.corpus == "text" else J.corpus_mixed
    host = gen(n, seed=1000 + rank, threads=16)
    dev = torch.device("cuda", local)
    d_in = torch.from_numpy(host).to(dev)
    cap = J.bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
    d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)
    stream = torch.cuda.Stream(dev)          # a real stream handle for the engine
    torch.cuda.set_stream(stream)
    sp = stream.cuda_stream
    gather = world > 1 and not args.no_gather
    lastflush = D.shard_lastflush(rank, world)   # END only on the job's last block
    recv = None
    side = torch.cuda.Stream(dev)            # the gather's stream
    ev_def = torch.cuda.Event()
    ev_gat = torch.cuda.Event()

    def step():
        nonlocal recv
        if gather:
            stream.wait_event(ev_gat)        # the last gather has read d_out / d_csz
        J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(),
                         d_coff.data_ptr(), d_tot.data_ptr(), level=args.level,
                         lastflush=lastflush, stream=sp)
        ev_def.record(stream)
        # the local inflate is queued before the host waits for any count
        J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb,
                         d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), stream=sp)
        if gather:
            # RCCL over xGMI: size index to every rank, then
            # the bitstreams into their final offsets on rank 0, on a side
            # stream that waits only for the deflate: the host's one wait
            # (for the all-gathered totals) overlaps the inflate kernels
            with torch.cuda.stream(side):
                side.wait_event(ev_def)
                D.gather_sizes(d_csz)
                recv, _ = D.gather_streams(d_out, d_tot, recv=recv)
                ev_gat.record(side)
            stream.wait_event(ev_gat)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # deflate / inflate split, measured on the same stream (outside the timed loop)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(stream)
    J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(),
                     d_coff.data_ptr(), d_tot.data_ptr(), level=args.level,
                     lastflush=lastflush, stream=sp)
    ev[1].record(stream)
    J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb,
                     d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), stream=sp)
    ev[2].record(stream)
    torch.cuda.synchronize()
    t_def, t_inf = ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2])

    # timed region: K steps, per-kernel HIP events on the engine's stream
    J.prof_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kt = J.prof_read()
    J.prof_enable(False)
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())

    # correctness of the last step (outside the timed region)
    ok = bool(torch.equal(d_back, d_in)) and int(d_err.abs().sum().item()) == 0
    ctotal = int(d_tot.item())
    if rank == 0:
        from oracle import jdoracle as O
        csz = d_csz.cpu().numpy().astype(np.int64)
        coff = d_coff.cpu().numpy()
        for b in (0, nb // 2, nb - 1):
            gpu_blk = d_out[int(coff[b]):int(coff[b]) + int(csz[b])].cpu().numpy().tobytes()
            ref = O.deflate(host[b * BS:(b + 1) * BS].tobytes(), level=args.level,
                            flush=lastflush if b == nb - 1 else 2)
            ok &= gpu_blk == ref
    if world > 1:
        f = torch.tensor([1 if ok else 0], device=dev)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item())
        tot = torch.tensor([ctotal], dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        call = int(tot.item())
    else:
        call = ctotal

    if rank == 0:
        ms = el / args.steps * 1e3
        total_bytes = n * world
        value = total_bytes * args.steps / el / 1e6
        # dominant kernel and its roofline (algorithmic bytes)
        dom, (dms, dcnt) = max(kt.items(), key=lambda kv: kv[1][0])
        avg_s = dms / dcnt / 1e3
        # a step launches each kernel once per chunk of <= 16,384 blocks
        # (1 GiB); one launch covers its chunk: N read + C written (deflate),
        # C read + N written (inflate), pro rata
        launches = max(1, round(dcnt / args.steps))
        alg = (n + ctotal) / launches
        achieved = alg / avg_s / 1e9
        traffic, traffic_src = pmc_traffic(dom, args.level, n, args.corpus)
        line = {
            "metric": metric_for(args.level),
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": workload_name(args, n, nb, world),
                "block": BS,
                "level": args.level,
                "bytes_per_gpu": n,
                "parallelism": f"shard{world}" + ("+rccl_gather" if gather else ""),
                "ratio": round(call / total_bytes, 6),
                "deflate_MBps_per_gpu": round(n / (t_def / 1e3) / 1e6, 2),
                "inflate_MBps_per_gpu": round(n / (t_inf / 1e3) / 1e6, 2),
                # SURVEY.md §8d per direction: (N + C) / t, and the north
                # star's HBM-read fraction (N / t_def, C / t_inf over 8 TB/s)
                "deflate_NplusC_GBps": round((n + ctotal) / (t_def / 1e3) / 1e9, 2),
                "inflate_NplusC_GBps": round((n + ctotal) / (t_inf / 1e3) / 1e9, 2),
                "deflate_hbm_read_frac": round(n / (t_def / 1e3) / 1e9 / HBM_PEAK_GBPS, 5),
                "inflate_hbm_read_frac": round(ctotal / (t_inf / 1e3) / 1e9 / HBM_PEAK_GBPS, 5),
                "roundtrip_ok": ok,
                "kernel_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in kt.items()},
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5),
                "traffic": traffic,
                # not measured in this run: the rocprofv3 FETCH_SIZE/WRITE_SIZE
                # passes of the same workload, committed under profiles/
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": int(alg),
                "launches_per_step": launches,
                "avg_launch_ms": round(avg_s * 1e3, 3),
                # no kernel here is HBM-bound: what bounds each is its issue
                # rate and its waits
                "compute": sq_compute(kt, args.steps, args.level, n, args.corpus),
            },
            "cpu_baseline": None,
        }
        if world == 1:
            line["config"]["checksum"] = checksum_rate(J, d_in, n, host, sp)
        if world == 1 and not args.no_host_api:
            line["config"]["host_api_pcie"] = host_api_rate(J, host, args.level, 256 << 20)
            line["config"]["dropin_pcie"] = dropin_rate(J, host, args.level, 256 << 20)
            line["config"]["dropin_stream_pcie"] = dropin_stream_rate(J, host, args.level,
                                                                      args.stream_sample)
            line["config"]["dropin_stream_mt_pcie"] = dropin_stream_mt_rate(
                J, host, args.level, args.stream_sample // 8, threads=8)
            line["config"]["zstrm_gzip_pcie"] = zstrm_rate(J, host, args.level, 256 << 20)
            line["config"]["foreign_stream_pcie"] = foreign_stream_rate(J, host, args.foreign_sample)
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(host, args.level, args.cpu_sample)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        raise SystemExit("round trip / parity check failed")


if __name__ == "__main__":
    main()
