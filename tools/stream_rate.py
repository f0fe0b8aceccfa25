"""Drop-in inflator rate with 32 KiB reads (bench.py dropin_stream_rate) on SIZE bytes."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
import jdeflate_amd as J
n = int(os.environ.get("SIZE", str(32 << 20)))
host = J.corpus_text(n, seed=1000, threads=16)
for piece in (32768, 1 << 20):
    print(json.dumps(bench.dropin_stream_rate(J, host, 6, n, piece=piece)), flush=True)
