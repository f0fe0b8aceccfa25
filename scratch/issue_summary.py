import csv,collections,glob,sys
d=sys.argv[1]; want=sys.argv[2] if len(sys.argv)>2 else 'k_match'
agg=collections.defaultdict(float)
for f in glob.glob(d+"/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if want in r['Kernel_Name']:
            agg[r['Counter_Name']]+=float(r['Counter_Value'])
for k,v in sorted(agg.items()): print("%-24s %.4g"%(k,v))
if 'SQ_INSTS_VALU' in agg and 'SQ_THREAD_CYCLES_VALU' in agg: print("lanes/valu", agg['SQ_THREAD_CYCLES_VALU']/agg['SQ_INSTS_VALU'])
