set -o pipefail
O=gpurun_out/mx; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 -u tools/exp_mixed.py 8000000 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
grep -E "ms/step" $O/log
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/mx/prof/**/prof_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/mx/prof/prof_kernel_trace.csv")
rows = list(csv.DictReader(open(f[0])))
hs = [r for r in rows if "http_classify" in r["Kernel_Name"]]
for r in hs:
    print(r["Kernel_Name"][:40], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r.get("Grid_Size", r.get("Grid_Size_X", "")))
PY
