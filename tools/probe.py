"""Timing probe: device deflate + inflate of 1 GiB text, per-kernel ms (no checks)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import jdeflate_amd as J
BS = 65536
n = int(os.environ.get("SIZE", str(1 << 30))); level = int(os.environ.get("LEVEL", "6"))
host = (J.corpus_mixed if os.environ.get('CORPUS') == 'mixed' else J.corpus_text)(n, seed=1000, threads=16)
dev = torch.device("cuda", 0)
d_in = torch.from_numpy(host).to(dev)
nb = n // BS; cap = J.bound(n)
d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
d_csz = torch.empty(nb, dtype=torch.int32, device=dev); d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
d_back = torch.empty(n, dtype=torch.uint8, device=dev)
d_us = torch.empty(nb, dtype=torch.int32, device=dev); d_err = torch.empty(nb, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev); torch.cuda.set_stream(s)
def step():
    J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(), d_coff.data_ptr(), d_tot.data_ptr(), level=level, stream=s.cuda_stream)
    J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb, d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), stream=s.cuda_stream)
step(); torch.cuda.synchronize()
import time
torch.cuda.synchronize(); t0 = time.time()
for _ in range(3): step()
torch.cuda.synchronize(); wall = (time.time() - t0) / 3 * 1e3
J.prof_enable(True)
for _ in range(3): step()
torch.cuda.synchronize()
kt = J.prof_read()
ok = torch.equal(d_back, d_in)
import zlib
tot = int(d_tot.item())
occ = zlib.crc32(d_out[:tot].cpu().numpy().tobytes())
print(json.dumps({"wall_ms": round(wall, 3), "MBps": round(n / wall / 1e3, 1), "ok": ok,
                  "total": tot, "outcrc": occ,
                  **{k: round(v[0] / 3, 3) for k, v in kt.items()}}))
