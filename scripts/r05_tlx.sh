#!/bin/bash
# Window kernel: per-XCC chain cycles per byte (kernel_timeline --placement),
# cfg2 and 3 072 x 1 KiB, three separate runs.
set -u
OUT=gpurun_out/r05/${RUN:-tlx}; mkdir -p $OUT
for r in 1 2 3; do
  timeout -k 10 200 python tools/kernel_timeline.py --placement --workloads cfg2,3072x1024 > $OUT/tl_$r.log 2>&1 || exit $?
done
grep -h placement $OUT/tl_*.log | python3 -c "
import sys, json
for line in sys.stdin:
    wl, js = line.split(' placement: ')
    print(wl, json.dumps(json.loads(js)['by_xcc']))
"
