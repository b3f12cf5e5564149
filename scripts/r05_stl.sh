#!/bin/bash
# cfg5 prologue evidence: per-pair timelines of the
# persistent kernel (range and grouped) and a timing-only A/B in which the
# first group's image is never loaded (the whole image burst gone).
set -u
OUT=gpurun_out/r05/stl; mkdir -p $OUT
timeout -k 10 300 python tools/stream_timeline.py --workloads cfg5,262144x1024 --dump $OUT/tl_range > $OUT/tl_range.log 2>&1 &&
timeout -k 10 300 python tools/stream_timeline.py --workloads cfg5 --ids grouped --dump $OUT/tl_grouped > $OUT/tl_grouped.log 2>&1 &&
timeout -k 10 500 python tools/ab_bench.py --variant prod: --variant noimg0:ZRC4_AB_NOIMG0=1 --no-check --workloads cfg5,262144x1024 --rounds 11 --launches 20 --segment > $OUT/ab_noimg0.log 2>&1
rc=$?; for f in $OUT/*.log; do echo "== $f"; grep -v amdgpu.ids $f | tail -3 | cut -c1-1500; done; exit $rc
