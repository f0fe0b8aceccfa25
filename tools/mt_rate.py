"""Multi-instance drop-in inflator rate (bench.py dropin_stream_mt_rate) on
SIZE bytes per instance, THREADS instances; run once per GPU_MAX_HW_QUEUES
setting (the variable is read when HIP initialises, so set it outside)."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench
import jdeflate_amd as J
n = int(os.environ.get("SIZE", str(32 << 20)))
threads = int(os.environ.get("THREADS", "8"))
host = J.corpus_text(n, seed=1000, threads=16)
r = bench.dropin_stream_mt_rate(J, host, 6, n, threads=threads)
r["hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES", "default")
print(json.dumps(r), flush=True)
