#!/bin/bash
# Round-2 probe 19: throughput-kernel workgroup pairs per CU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/stream_timeline.py --workloads cfg5,131072x1024 --footprint-mib 640 > gpurun_out/stl_pairs.log 2>&1
rc=$?; echo "[stl_pairs] rc=$rc"; grep -v amdgpu.ids gpurun_out/stl_pairs.log | grep -v '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    k, _, j = l.partition(' ')
    try: d = json.loads(j)
    except Exception: print(l[:300]); continue
    print(k, json.dumps(d['by_place'].get('cu_pairs')), json.dumps(d['by_place']['simd_of_wave0']))
"
exit $rc
