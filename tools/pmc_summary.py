"""Summarise rocprofv3 PMC csv files: mean counter value per kernel (name substring filter)."""
import csv, collections, glob, sys
root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(root + "/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            k = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("((")[0][:60]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print("   %-26s %14.4g  (n=%d)" % (c, sum(v) / len(v), len(v)))
