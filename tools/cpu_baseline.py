"""CPU baseline check: the oracle's speed against the
reference's own container numbers, same corpus kind, same
machine class (this container's 8-core Xeon), one thread and all cores.

Corpus: every *.py under /usr/lib/python3.10 and /usr/lib/python3/dist-packages
in sorted path order, concatenated and cut at 18.8 MB (the survey's "Python
stdlib source, 18.8 MB"; its exact file list was not recorded, so the ratio
is printed beside the reference's 0.2599 as a check of the corpus's kind).
64 KiB independent blocks, fresh state per block, as BASELINE.md §2.
Writes one JSON object to stdout (profiles/r06_cpu_baseline.json)."""
import ctypes
import glob
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import jdoracle as O  # noqa: E402

REF = {  # BASELINE.md §2, Python stdlib source 18.8 MB (deflate, inflate MB/s)
    (6, 1): ((47.0, 60.0), (340.0, 396.0)),
    (6, 8): ((313.0, 328.0), (2633.0, 2704.0)),
    (9, 1): ((24.5, 24.5), (410.0, 410.0)),
    (9, 8): ((147.0, 147.0), (2487.0, 2487.0)),
}
REF_RATIO = {6: 0.2599, 9: 0.2556}
BS = 65536


def corpus(n=18_800_000):
    fs = sorted(glob.glob("/usr/lib/python3.10/**/*.py", recursive=True) +
                glob.glob("/usr/lib/python3/dist-packages/**/*.py", recursive=True))
    out = bytearray()
    for f in fs:
        with open(f, "rb") as fh:
            out += fh.read()
        if len(out) >= n:
            break
    return bytes(out[:n])


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), r


def main():
    data = corpus()
    n = len(data)
    nb = -(-n // BS)
    L = O.lib()
    src = ctypes.create_string_buffer(data, n)
    slot = L.jdo_bound(BS) + 1024
    dst = ctypes.create_string_buffer(nb * slot)
    sizes = (ctypes.c_uint32 * nb)()
    back = ctypes.create_string_buffer(nb * BS)
    rows = []
    for level in (6, 9):
        for threads in (1, 8):
            reps = 5 if threads == 8 or level == 6 else 3
            td, _ = timed(lambda: L.jdo_deflate_blocks_mt(src, n, BS, level, dst, slot, sizes, threads), reps)
            cs = list(sizes)
            coff = (ctypes.c_uint64 * nb)(*[i * slot for i in range(nb)])
            csz = (ctypes.c_uint32 * nb)(*cs)
            ti, bad = timed(lambda: L.jdo_inflate_blocks_mt(dst, coff, csz, nb, BS, back, threads), reps)
            assert bad == 0 and back.raw[:n] == data
            ratio = sum(cs) / n
            rd, ri = REF[(level, threads)]
            dm, im = n / td / 1e6, n / ti / 1e6
            rows.append({
                "level": level, "threads": threads, "deflate_MBps": round(dm, 1), "inflate_MBps": round(im, 1),
                "ratio": round(ratio, 4), "ref_deflate_MBps": list(rd), "ref_inflate_MBps": list(ri),
                "ref_ratio": REF_RATIO[level],
                "deflate_vs_ref_mid": round(dm / ((rd[0] + rd[1]) / 2), 3),
                "inflate_vs_ref_mid": round(im / ((ri[0] + ri[1]) / 2), 3),
            })
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    print(json.dumps({"corpus": "python-source", "bytes": n, "blocks": nb, "cpu": cpu,
                      "online_cpus": os.cpu_count(), "python": platform.python_version(),
                      "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
