"""HBM traffic per l7g_classify call from rocprofv3 FETCH_SIZE / WRITE_SIZE
passes (separate runs, tools/run_r6_pmc.sh) -> profiles/traffic_<workload>.json,
which bench.py reports as roofline.traffic for the dominant kernel.

Per kernel name (template instantiations apart) the counters are averaged
over its dispatches; a stage launched as several kernels (the HTTP hot and
general instantiations) sums them.  gfx950 correction (MI355X_MICROARCH.md,
HBM / rocprofv3 section): FETCH_SIZE reports half the bytes of 16-byte-per-
lane reads (every classifier reads through 16-byte loads), so it is doubled;
WRITE_SIZE is taken as reported.  Both are in KiB.

usage: python tools/traffic.py <workload> <fetch pmc dir> <write pmc dir> <note>
"""
import collections
import csv
import glob
import json
import os
import sys

STAGES = {"http_classify_kernel": "http_classify_kernel", "http_grouped_kernel": "http_grouped_kernel",
          "http_group_count_kernel": "http_group_count_kernel", "http_group_scatter_kernel": "http_group_scatter_kernel",
          "kafka_classify_kernel": "kafka_classify_kernel", "memcache_classify_kernel": "memcache_classify_kernel",
          "partition_kernel": "partition_kernel"}


def per_name(root, counter):
    agg = collections.defaultdict(float)
    names = {}
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            agg[(r["Kernel_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[r["Kernel_Name"]] = 1
    out = {}
    for name in names:
        vals = [v for (k, _), v in agg.items() if k == name]
        out[name] = sum(vals) / len(vals)
    return out


def main():
    wl, fdir, wdir = sys.argv[1:4]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    fetch, write = per_name(fdir, "FETCH_SIZE"), per_name(wdir, "WRITE_SIZE")
    kernels = {}
    for stage in STAGES:
        fk = sum(v for k, v in fetch.items() if stage in k.split("(")[0])
        wk = sum(v for k, v in write.items() if stage in k.split("(")[0])
        if fk == 0 and wk == 0:
            continue
        rd, wr = int(fk * 1024 * 2), int(wk * 1024)
        kernels[stage] = {"fetch_size_kb_reported": round(fk, 1), "write_size_kb_reported": round(wk, 1),
                          "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
                          "hbm_bytes_per_launch": rd + wr}
    out = {"workload": wl, "note": note,
           "source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes (tools/run_r6_pmc.sh)",
           "correction": ("gfx950 FETCH_SIZE x2: one TCC_EA0_RDREQ per 128-byte line read, counted as 64 B -- "
                          "calibrated for these kernels' access shapes on known reads of cfg5's requests "
                          "(wave-coalesced, one lane per request in 16- and 64-byte steps: "
                          "profiles/r6/kafka_traffic_calibration_pmc.txt); WRITE_SIZE as reported; KiB -> bytes"),
           "kernels": kernels}
    if len(kernels) == 1:
        out["hbm_bytes_per_launch"] = next(iter(kernels.values()))["hbm_bytes_per_launch"]
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", f"traffic_{wl}.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
