# Round 6, call T (GPU box): lat_fast's phase split (timing build, tools/exp_lat.py).
set -o pipefail
O=gpurun_out/${TAG:-r6t}; mkdir -p $O; export TMPDIR=/tmp
L7G_LIB=cilium_amd/libl7gpu_timing.so timeout -k 10 200 python -u tools/exp_lat.py > $O/lat_timing.log 2>&1 || { tail -5 $O/lat_timing.log; exit 2; }
grep -v amdgpu.ids $O/lat_timing.log
