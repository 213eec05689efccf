"""Summarise rocprofv3 counter-collection CSVs: mean counter value per kernel."""
import csv
import collections
import glob
import sys

for path in sys.argv[1:]:
    for f in glob.glob(path + "/**/*counter_collection.csv", recursive=True) or [path]:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        durs = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
            durs[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print(f)
        for k, d in agg.items():
            print(f"  {k[:40]:40s} n={len(durs[k])} dur_us={sum(durs[k]) / len(durs[k]) / 1e3:.1f}")
            for c, v in sorted(d.items()):
                print(f"      {c:32s} {sum(v) / len(v):16.1f}")
