"""Diagnostic: all-zero 64 KiB blocks (the zero kind of the mixed corpus).
Each stage runs in its own process; the driver stops at the first failure.
  python tools/zero_diag.py            (driver)
  python tools/zero_diag.py STAGE NB   (one stage)"""
import os, sys, subprocess
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
BS = 65536


def stage(name, nb):
    import numpy as np
    import torch
    import jdeflate_amd as J
    from oracle import jdoracle as O
    n = nb * BS
    host = np.zeros(n, dtype=np.uint8)
    dev = torch.device("cuda", 0)
    level = 9 if "l9" in name else 6
    ref1 = O.deflate(bytes(BS), level=level, flush=2)
    if name.startswith("inflate"):
        comp = ref1 * nb
        d_c = torch.from_numpy(np.frombuffer(comp, dtype=np.uint8).copy()).to(dev)
        d_coff = torch.tensor([i * len(ref1) for i in range(nb)], dtype=torch.int64, device=dev)
        d_csz = torch.full((nb,), len(ref1), dtype=torch.int32, device=dev)
        d_back = torch.empty(n, dtype=torch.uint8, device=dev)
        d_us = torch.empty(nb, dtype=torch.int32, device=dev)
        d_err = torch.empty(nb, dtype=torch.int32, device=dev)
        J.inflate_device(d_c.data_ptr(), len(comp), d_coff.data_ptr(), d_csz.data_ptr(), nb, d_back.data_ptr(),
                         d_us.data_ptr(), d_err.data_ptr())
        torch.cuda.synchronize()
        ok = bool((d_back == 0).all()) and not bool(d_err.any())
    else:
        d_in = torch.from_numpy(host).to(dev)
        cap = J.bound(n)
        d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
        d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
        d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
        d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
        J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(), d_coff.data_ptr(),
                         d_tot.data_ptr(), level=level)
        torch.cuda.synchronize()
        csz = d_csz.cpu().numpy()
        out = d_out[:int(d_tot.item())].cpu().numpy().tobytes()
        last = O.deflate(bytes(BS), level=level, flush=1)
        ok = out == ref1 * (nb - 1) + last
        print("sizes", set(csz.tolist()), len(ref1), len(last))
    print(name, nb, "ok" if ok else "MISMATCH", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    if len(sys.argv) > 2:
        sys.exit(stage(sys.argv[1], int(sys.argv[2])))
    plan = [("inflate_l9", 1024), ("deflate_l6", 1024), ("deflate_l9", 16), ("deflate_l9", 1024)]
    for name, nb in plan:
        env = dict(os.environ)
        r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, os.path.abspath(__file__), name, str(nb)],
                           env=env)
        print("stage", name, nb, "rc", r.returncode, flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)
