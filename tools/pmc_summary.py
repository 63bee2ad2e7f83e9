"""Summarise rocprofv3 --pmc CSVs: per-dispatch counter sums averaged over the
dispatches of the kernels whose name contains a pattern."""
import collections
import csv
import glob
import sys


def summarize(root, pattern="http_classify"):
    out = {}
    for f in sorted(set(glob.glob(f"{root}/**/pmc_counter_collection.csv", recursive=True))):
        agg = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if pattern not in r["Kernel_Name"]:
                continue
            agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        per = collections.defaultdict(list)
        for (_, c), v in agg.items():
            per[c].append(v)
        for c, v in per.items():
            out[c] = sum(v) / len(v)
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "http_classify")
    for k in sorted(res):
        print(f"{k:28s} {res[k]:16.1f}")
