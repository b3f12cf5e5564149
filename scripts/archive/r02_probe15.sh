#!/bin/bash
# Round-2 probe 15: s_memrealtime span of the last launch vs HIP events.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/stream_timeline.py --workloads cfg5,262144x1024,131072x1024 --footprint-mib 640 > gpurun_out/stl_ev.log 2>&1
rc=$?; echo "[stl_ev] rc=$rc"; grep -v amdgpu.ids gpurun_out/stl_ev.log | grep -v '^{' | python3 -c "
import sys, json
for l in sys.stdin:
    k, _, j = l.partition(' ')
    try: d = json.loads(j)
    except Exception: print(l[:300]); continue
    print(k, 'span', d['span_us'], 'event', d['last_launch_event_us'], 'clk', d['clock_ghz']['med'])
"
exit $rc
