# device framing throughput: product vs variants (GPU box)
set -o pipefail
for k in ${KINDS:-http memcache}; do
  for lib in libl7gpu.so $VARLIBS; do
    echo "== $lib"; L7G_LIB=$PWD/cilium_amd/$lib timeout -k 10 300 python -u tools/exp_frame.py $k 1000000 16384 2>&1 | grep -E "frame_streams|requests in" || exit 1
  done
done
