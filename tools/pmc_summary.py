"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE, SQ_*) into a per-kernel JSON.

  python tools/pmc_summary.py <pmc_dir> <out.json>

<pmc_dir> holds one sub-directory per pass (fetch/, write/, sq1/, ...) with
run_counter_collection.csv.  FETCH_SIZE / WRITE_SIZE are in KiB; per MI355X_MICROARCH.md
("HBM [CDNA4]") gfx950's FETCH_SIZE counts exactly half the bytes of 16-B-per-lane
reads, so fetch is doubled (`fetch_bytes`); WRITE_SIZE is exact for 16-B stores.  Values
are per dispatch: the mean over the dispatches of that kernel, and (`*_max`) the largest
dispatch, which is the large launch of a kernel that runs in both halves with very different
sizes (bench.py's roofline reads that one)."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("qmfx::", "")
    return "rocprim" if "rocprim" in n else n


def main(src, out):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(src, "*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, cs in sorted(per.items()):
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"dispatches": max(len(v) for v in cs.values())}
        if "FETCH_SIZE" in d:
            e["fetch_bytes"] = d["FETCH_SIZE"] * 1024 * 2
            e["fetch_bytes_max"] = max(cs["FETCH_SIZE"]) * 1024 * 2
        if "WRITE_SIZE" in d:
            e["write_bytes"] = d["WRITE_SIZE"] * 1024
            e["write_bytes_max"] = max(cs["WRITE_SIZE"]) * 1024
        for c, v in d.items():
            if c.startswith("SQ_") or c.startswith("GRBM"):
                e[c] = v
        res[k] = e
    json.dump({"source": "rocprofv3 --pmc, one counter group per pass (tools/pmc.sh)",
               "units": "bytes per dispatch; fetch doubled per the gfx950 FETCH_SIZE note",
               "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
