"""Does deflate overlap with inflate on one GPU?  Runs N deflates of 1 GiB of
text (L6) in one process and N inflates in another, alone and at the same
time (two processes: two HIP contexts, so the engine's cross-stream ordering
does not serialise them), and prints each loop's time.  If the two together
take clearly less than the sum alone, a pipelined step (batch k's inflate
beside batch k+1's deflate) would gain.

    python tools/overlap_probe.py
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = int(os.environ.get("N", "20"))


def child(mode: str, start_at: float) -> None:
    sys.path.insert(0, ROOT)
    import torch
    import jdeflate_amd as J
    n = 1 << 30
    bs = 65536
    nb = n // bs
    host = J.corpus_text(n, seed=1000, threads=8)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(host).to(dev)
    cap = J.bound(n)
    d_out = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_csz = torch.empty(nb, dtype=torch.int32, device=dev)
    d_coff = torch.empty(nb, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(1, dtype=torch.int64, device=dev)
    d_back = torch.empty(n, dtype=torch.uint8, device=dev)
    d_us = torch.empty(nb, dtype=torch.int32, device=dev)
    d_err = torch.empty(nb, dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(dev)
    torch.cuda.set_stream(st)
    sp = st.cuda_stream

    def defl():
        J.deflate_device(d_in.data_ptr(), n, d_out.data_ptr(), cap, d_csz.data_ptr(), d_coff.data_ptr(),
                         d_tot.data_ptr(), level=6, stream=sp)

    def infl():
        J.inflate_device(d_out.data_ptr(), cap, d_coff.data_ptr(), d_csz.data_ptr(), nb, d_back.data_ptr(),
                         d_us.data_ptr(), d_err.data_ptr(), stream=sp)
    defl()
    infl()
    torch.cuda.synchronize()
    f = defl if mode == "def" else infl
    print(f"{mode} ready, {start_at - time.time():.1f} s to start", file=sys.stderr, flush=True)
    while time.time() < start_at:
        time.sleep(0.001)
    t0 = time.perf_counter()
    for _ in range(N):
        f()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ok = bool(torch.equal(d_back, d_in))
    print(json.dumps({"mode": mode, "ms_per_iter": round(el / N * 1e3, 3), "ok": ok}), flush=True)


def run(modes, delay):
    start = time.time() + delay         # every child is set up by then
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", m, repr(start)],
                           stdout=subprocess.PIPE, text=True) for m in modes]
    out = []
    for p in ps:
        o, _ = p.communicate(timeout=400)
        if p.returncode:
            raise SystemExit(f"child failed: {p.returncode}")
        out.append(json.loads(o.strip().splitlines()[-1]))
    return out


def main() -> None:
    if len(sys.argv) > 3 and sys.argv[1] == "--child":
        child(sys.argv[2], float(sys.argv[3]))
        return
    alone = run(["def"], 100.0)
    print(json.dumps(alone), flush=True)
    alone += run(["inf"], 40.0)
    print(json.dumps(alone), flush=True)
    both = run(["def", "inf"], 40.0)
    print(json.dumps({"alone": alone, "together": both, "N": N}), flush=True)


if __name__ == "__main__":
    main()
