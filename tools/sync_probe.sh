# one-request sync path breakdown (GPU box)
set -o pipefail
O=gpurun_out/${TAG:-probe}; mkdir -p $O
python -c "
import sys, json; sys.path.insert(0, '.')
from cilium_amd import gen
h = gen.http_workload(2, 512)
c0 = h.conns[0]
reqs = [bytes(h.arena[int(o):int(o) + int(n)]) for o, n in zip(h.offsets, h.lengths)]
print(json.dumps(h.policy)); print(int(c0['policy']), int(c0['port']), int(c0['ingress']), int(c0['src_id']), int(c0['dst_id']))
print('mc x 0 0')
for r in reqs: print(r.hex())
" > $O/in.txt || exit 1
for m in block; do echo "== $m"; timeout -k 10 60 tools/experiments/sync_probe $m < $O/in.txt || exit 1; done
