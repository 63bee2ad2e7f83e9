"""Per-kernel resources of a run (measurement tool): from a rocprofv3
--kernel-trace CSV, each kernel's first dispatch -- LDS bytes per workgroup,
scratch bytes per lane, VGPRs (the trace's VGPR_Count is in units of 2
registers on this ROCm: 128 = 256 VGPRs; the 'vgprs' column doubles it), SGPRs,
workgroup size -- and its dispatch count and mean duration.
usage: python tools/kernel_resources.py TRACE.csv [pattern]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "l7::"
    first, durs = {}, collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        first.setdefault(k, r)
    print(f"{'kernel':70s} {'lds_B':>7s} {'scratch_B':>9s} {'vgprs':>5s} {'sgprs':>5s} {'wg':>5s} {'calls':>5s} {'mean_ms':>9s}")
    for k, r in sorted(first.items(), key=lambda kv: -sum(durs[kv[0]])):
        print(f"{k[:70]:70s} {int(r['LDS_Block_Size']):7d} {int(r['Scratch_Size']):9d} {2 * int(r['VGPR_Count']):5d} "
              f"{int(r['SGPR_Count']):5d} {int(r['Workgroup_Size_X']):5d} {len(durs[k]):5d} {sum(durs[k]) / len(durs[k]):9.4f}")


if __name__ == "__main__":
    main()
