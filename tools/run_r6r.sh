# Round 6, call R (GPU box): where a one-request HTTP call's device time goes
# with lat_fast (tools/exp_lat.py: product, then the phase-stamped build).
set -o pipefail
O=gpurun_out/${TAG:-r6r}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u tools/exp_lat.py > $O/lat_prod.log 2>&1 || { tail -5 $O/lat_prod.log; exit 1; }
L7G_LIB=cilium_amd/libl7gpu_timing.so timeout -k 10 200 python -u tools/exp_lat.py > $O/lat_timing.log 2>&1 || { tail -5 $O/lat_timing.log; exit 2; }
grep -v amdgpu.ids $O/lat_prod.log $O/lat_timing.log
