#!/bin/bash
# BASELINE config 1 on the round-6 tree: the frameStressTest-shaped loopback
# (tools/frame_stress.cpp, 1 KiB proto4z packets, RC4 both directions) with the
# gfx950 hooks (adaptive default), the reference's own RC4 on the CPU
# (oracle/_ref) and RC4 off, interleaved, 3 repetitions of 2 s per point.
set -u
OUT=gpurun_out/r06/${RUN:-loop}; mkdir -p $OUT
REF=oracle/_ref/libzrc4_ref.so
[ -f "$REF" ] || { echo "no $REF"; exit 1; }
: > $OUT/frame_loopback.jsonl
for rep in 1 2 3; do
  for cfg in "2 1" "2 4" "64 1" "512 1" "2048 2"; do
    set -- $cfg
    for hooks in device "host:$REF" off; do
      timeout -k 10 60 zsummerx_amd/bin/frame_stress --rc4 "$hooks" --sessions $1 --depth $2 \
          --seconds 2 --warmup 0.5 >> $OUT/frame_loopback.jsonl 2>> $OUT/frame_loopback.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "[loopback $cfg $hooks] rc=$rc"; exit $rc; fi
    done
  done
  echo "rep $rep done"
done
python3 - "$OUT/frame_loopback.jsonl" <<'PY'
import json, statistics, sys, collections
rows = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    assert d["mismatches"] == 0, d
    rows[(d["sessions"], d["depth"], d["rc4"].split(":")[0])].append(d["echo_per_s"])
for k in sorted(rows):
    print(k, round(statistics.median(rows[k])), [round(v) for v in rows[k]])
PY
