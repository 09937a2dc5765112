#!/bin/bash
# The frame scan at uniform frame sizes (tools/bench_sizes.py) with the one-pass path by default and
# off (NETC_SCAN_ONEPASS=0), two interleaved rounds (through gpurun, repo root)
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
D=$R/gpurun_out/${TAG:-r06_sizes}; mkdir -p $D
for r in 1 2; do for v in def 0; do
 ( [ $v = 0 ] && export NETC_SCAN_ONEPASS=0; exec timeout -k 10 300 python -u tools/bench_sizes.py --sizes 16,64,128,256,1024,4096 > $D/sizes_$v.$r.log 2>&1 ) || { tail -5 $D/sizes_$v.$r.log; exit 1; }
 python3 -c "
import json
for l in open('$D/sizes_$v.$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', $r, d.get('frame_bytes', d.get('size')), {k: v for k, v in d.items() if 'scan' in k})
"
done; done
