"""Per-dispatch listing of rocprofv3 --pmc CSVs (measurement tool): one line
per dispatch in order, kernel name and every counter's value summed over the
dispatch's instances.  usage: python tools/pmc_dispatches.py DIR [DIR ...] [--match PATTERN]"""
import collections
import csv
import glob
import sys


def dispatches(root, pattern=""):
    rows = collections.OrderedDict()
    for f in sorted(glob.glob(f"{root}/**/pmc_counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            if pattern and pattern not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            d = rows.setdefault(k, {"name": r["Kernel_Name"], "c": collections.defaultdict(float)})
            d["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return [rows[k] for k in sorted(rows)]


if __name__ == "__main__":
    args = sys.argv[1:]
    pat = ""
    if "--match" in args:
        i = args.index("--match")
        pat = args[i + 1]
        del args[i:i + 2]
    for root in args:
        print(f"== {root}")
        for d in dispatches(root, pat):
            cs = "  ".join(f"{k}={v:.4g}" for k, v in sorted(d["c"].items()))
            print(f"{d['name'][:60]:60s} {cs}")
