"""Per-kernel summary of SQ counter passes written by tools/prof_counters.sh."""
import collections, csv, glob, sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    v = c.get("SQ_INSTS_VALU", 0) or 1
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k[:40]:40s} waves={c.get('SQ_WAVES', 0):9.0f} valu={c.get('SQ_INSTS_VALU', 0):.3g} "
          f"lanes/valu={c.get('SQ_THREAD_CYCLES_VALU', 0) / v:5.1f} salu={c.get('SQ_INSTS_SALU', 0):.3g} "
          f"lds={c.get('SQ_INSTS_LDS', 0):.3g} vmem_rd={c.get('SQ_INSTS_VMEM_RD', 0):.3g} "
          f"busy_cu={c.get('SQ_BUSY_CU_CYCLES', 0):.3g} wave_cyc={wc:.3g} "
          f"active_any/wave={c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} wait_any/wave={c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
          f"valu_act/wave={c.get('SQ_ACTIVE_INST_VALU', 0) / wc:.2f} lds_wait/wave={c.get('SQ_WAIT_INST_LDS', 0) / wc:.2f} "
          f"bankconf={c.get('SQ_LDS_BANK_CONFLICT', 0):.3g}")
