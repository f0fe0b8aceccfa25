"""Per-kernel ms for each block kind of the mixed corpus (corpus.c jdc_mixed),
1024 blocks of one kind per run; LEVEL (default 9)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import jdeflate_amd as J

BS = 65536
M64 = (1 << 64) - 1
level = int(os.environ.get("LEVEL", "9"))
per = int(os.environ.get("PER", "1024"))


def rnext(s):
    s = (s + 0x9e3779b97f4a7c15) & M64
    z = s
    z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
    z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
    return s, z ^ (z >> 31)


def kind(seed, u):
    _, s = rnext((seed * 0x9e3779b97f4a7c15 ^ u) & M64)
    pick = s % 100
    return 0 if pick < 35 else 1 if pick < 55 else 2 if pick < 70 else 3 if pick < 85 else 4 if pick < 95 else 5


seed = 1000
nblk = per * 22
host = J.corpus_mixed(nblk * BS, seed=seed, threads=16)
kinds = np.array([kind(seed, u) for u in range(nblk)])
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(dev)
torch.cuda.set_stream(s)
names = ["text", "code", "random", "ramps", "runs", "zero"]
for k in range(6):
    idx = np.nonzero(kinds == k)[0][:per]
    buf = np.concatenate([host[i * BS:(i + 1) * BS] for i in idx])
    n = len(buf)
    nb = n // BS
    cap = J.bound(n)
    d_in = torch.from_numpy(buf).to(dev)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
    d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)

    def step():
        J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(), d_coff.data_ptr(),
                         d_tot.data_ptr(), level=level, stream=s.cuda_stream)
        J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb, d_back.data_ptr(),
                         d_us.data_ptr(), d_err.data_ptr(), stream=s.cuda_stream)
    step()
    torch.cuda.synchronize()
    J.prof_enable(True)
    step()
    torch.cuda.synchronize()
    kt = J.prof_read()
    J.prof_enable(False)
    ok = torch.equal(d_back, d_in)
    tot = int(d_tot.item())
    import zlib
    occ = zlib.crc32(d_out[:tot].cpu().numpy().tobytes())
    print(json.dumps({"kind": names[k], "blocks": nb, "total": tot, "outcrc": occ, "ok": ok,
                      **{kk: round(v[0], 3) for kk, v in kt.items()}}), flush=True)
