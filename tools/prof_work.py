"""Profiling workload: device-resident deflate+inflate of SIZE bytes, REPS times."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import jdeflate_amd as J
size = int(os.environ.get("SIZE", str(256 << 20))); reps = int(os.environ.get("REPS", "3"))
level = int(os.environ.get("LEVEL", "6"))
BS = 65536
dev = torch.device("cuda", 0)
torch.cuda.init()
if os.environ.get("CORPUS") == "runs":
    # the runs kind of corpus.c's mixed corpus: runs of 1-200 bytes of {0, 1, 255}
    import numpy as np
    rng = np.random.default_rng(1000)
    k = size // 50 + 1
    host = np.repeat(rng.choice(np.array([0, 1, 255], dtype=np.uint8), k), rng.integers(1, 201, k))[:size].copy()
else:
    host = J.corpus_text(size, seed=1000, threads=16)
d_in = torch.from_numpy(host).to(dev)
nb = size // BS; cap = J.bound(size)
d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
d_csz = torch.empty(nb, dtype=torch.int32, device=dev); d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
d_back = torch.empty(size, dtype=torch.uint8, device=dev)
d_us = torch.empty(nb, dtype=torch.int32, device=dev); d_err = torch.empty(nb, dtype=torch.int32, device=dev)
s = torch.cuda.Stream(dev)
for _ in range(reps):
    J.deflate_device(d_in.data_ptr(), size, d_out.data_ptr(), cap, d_csz.data_ptr(), d_coff.data_ptr(), d_tot.data_ptr(), level=level, stream=s.cuda_stream)
    J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb, d_back.data_ptr(), d_us.data_ptr(), d_err.data_ptr(), stream=s.cuda_stream)
s.synchronize()
print("ok", torch.equal(d_back, d_in), int(d_tot.item()) / size)
