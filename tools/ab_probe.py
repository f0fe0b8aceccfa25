"""A/B timing of whole engine builds on the same box (regression bisects).

    python tools/ab_probe.py LIB.so [LIB.so ...]      # one child process per library

Each child loads only the given libjdeflate_amd.so (through plain ctypes, so
builds that predate newer entry points load too), deflates + inflates 1 GiB of
the bench corpus (level 6, 64 KiB blocks) resident in HBM, and prints one JSON
line with the per-kernel ms per launch from the engine's HIP-event profiler
(the enum indices below are stable since round 2).  SIZE, LEVEL and
CORPUS=mixed select other workloads.  The order of the libraries
is repeated twice (ABBA-style) to expose box drift.
"""
import ctypes
import json
import os
import subprocess
import sys

NAMES = ["k_chains<4>", "k_chains<3>", "k_match", "k_parse", "k_emit", "k_stored", "k_scan",
         "k_compact", "k_inflate", "k_inflate_par", "k_inflate_resolve", "k_pspec", "k_psync",
         "k_pjoin", "k_checksum", "k_inflate_mp", "k_fsp_find", "k_fsp_decode", "k_fsp_window",
         "k_fsp_resolve", "k_inflate_rpar", "k_porder"]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib_path: str) -> None:
    import torch
    torch.cuda.init()
    sys.path.insert(0, ROOT)
    import jdeflate_amd as J               # only for the corpus generator
    n = int(os.environ.get("SIZE", str(1 << 30)))
    level = int(os.environ.get("LEVEL", "6"))
    gen = J.corpus_mixed if os.environ.get("CORPUS") == "mixed" else J.corpus_text
    host = gen(n, seed=1000, threads=16)
    L = ctypes.CDLL(lib_path)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.jdgpu_bound.restype = u64
    L.jdgpu_bound.argtypes = [u64, u32]
    L.jdgpu_deflate_device.restype = i32
    L.jdgpu_deflate_device.argtypes = [vp, u64, u32, i32, u32, i32, vp, u64, vp, vp, vp, vp]
    L.jdgpu_inflate_device.restype = i32
    L.jdgpu_inflate_device.argtypes = [vp, u64, vp, vp, u32, u32, vp, vp, vp, vp]
    L.jdgpu_prof_enable.argtypes = [i32]
    L.jdgpu_prof_read.argtypes = [vp, vp, i32]
    BS = 65536
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(host).to(dev)
    nb = n // BS
    cap = int(L.jdgpu_bound(n, BS))
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
    d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)

    def step():
        r = L.jdgpu_deflate_device(d_in.data_ptr(), n, BS, level, 0, 1, d_out.data_ptr(), cap,
                                   d_csz.data_ptr(), d_coff.data_ptr(), d_tot.data_ptr(), s.cuda_stream)
        assert r == 0, r
        r = L.jdgpu_inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb, BS,
                                   d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), s.cuda_stream)
        assert r == 0, r

    step()
    torch.cuda.synchronize()
    L.jdgpu_prof_enable(1)
    reps = 3
    for _ in range(reps):
        step()
    torch.cuda.synchronize()
    ms = (ctypes.c_double * 32)()
    cnt = (ctypes.c_uint64 * 32)()
    L.jdgpu_prof_read(ms, cnt, 32)
    ok = bool(torch.equal(d_back, d_in))
    import zlib
    tot = int(d_tot.item())
    out = {"lib": os.path.relpath(lib_path, ROOT), "ok": ok, "total": tot,
           "outcrc": zlib.crc32(d_out[:tot].cpu().numpy().tobytes())}
    for i, nm in enumerate(NAMES):
        if cnt[i]:
            out[nm] = round(ms[i] / reps, 3)
    print(json.dumps(out), flush=True)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(os.path.abspath(sys.argv[2]))
        return
    libs = [os.path.abspath(p) for p in sys.argv[1:]]
    for p in libs + libs[::-1]:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", p], timeout=240)
        if r.returncode:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
