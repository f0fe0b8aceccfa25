"""Per-kernel SQ issue counters of a tools/prof_counters.sh run as JSON
(profiles/sq_summary*.json), read by bench.py for the roofline's compute
side: VALU and LDS issue rates against the wave64 peaks, and the share of
wave cycles parked in s_waitcnt (SQ_WAIT_ANY).

    python tools/sq_json.py OUTDIR TAG SIZE LEVEL [CORPUS] > profiles/sq_summary.json

Counters are summed over a kernel's dispatches and divided by their number
(per launch); cycle counters are quad-cycles (MI355X_MICROARCH.md), so only
their ratios are used."""
import collections
import csv
import glob
import json
import sys


def main():
    d, tag, size, level = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    corpus = sys.argv[5] if len(sys.argv) > 5 else "text"
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    out = {}
    for k, c in agg.items():
        if not k.startswith("k_"):
            continue
        per = {}
        for name, v in c.items():
            n = max(1, len(disp[(k, name)]))
            per[name] = v / n
            per["dispatches"] = max(per.get("dispatches", 0), n)
        out[k] = per
    print(json.dumps({"tag": tag, "workload": {"bytes": size, "level": level, "corpus": corpus},
                      "command": "tools/prof_counters.sh (rocprofv3 --pmc passes on tools/prof_work.py, 1 rep)",
                      "kernels": out}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
