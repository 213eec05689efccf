"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_traffic.sh into
profiles/<name>.json: mean per dispatch and hbm_bytes = 2*FETCH + WRITE (KB)."""
import csv
import collections
import glob
import json
import sys


def means(d):
    acc = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("(anonymous namespace)::", "")
            acc[name].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


fetch, write = means(sys.argv[1]), means(sys.argv[2])
# optional: the U4 probe's passes (tools/u4_probe.py), its kernels keyed "<name>_evd"
if len(sys.argv) > 5:
    for k, v in means(sys.argv[4]).items():
        fetch[k + "_evd"] = v
    for k, v in means(sys.argv[5]).items():
        write[k + "_evd"] = v
out = {
    "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of "
              "`python3 bench.py --steps 5 --warmup 2 --skip-cpu --skip-e2e --skip-config3 --skip-u4` (the pipeline and "
              "U1 phases), mean per dispatch; *_evd: `python3 tools/u4_probe.py` (U4 alone) (tools/prof_bench.sh "
              "with PMC=1)",
    "correction": "gfx950: FETCH_SIZE counts half the bytes of wide streaming reads (MI355X_MICROARCH.md HBM "
                  "section): hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE; Infinity-Cache hits are included",
    "kernels": {k: {"FETCH_SIZE_KB": round(fetch[k], 1), "WRITE_SIZE_KB": round(write.get(k, 0.0), 1),
                    "hbm_bytes": int(round((2 * fetch[k] + write.get(k, 0.0)) * 1024))} for k in fetch},
}
json.dump(out, open(sys.argv[3], "w"), indent=1)   # argv: fetch_dir write_dir out [u4_fetch_dir u4_write_dir]
print(json.dumps(out["kernels"], indent=1))
