#!/bin/bash
# Round-6 A/B: the reservoir hooks' refill piece per slot ($ZSX_REFILL_CHUNK,
# default 8192; at most a quarter of the ring) in the config-1 loopback and
# larger shapes, interleaved with the reference's CPU RC4, REPS repetitions
# of 2 s per point.  VARIANTS: chunk:ring pairs (ring = --ring bytes per slot).
set -u
OUT=gpurun_out/r06/${RUN:-refill}; mkdir -p $OUT
REF=oracle/_ref/libzrc4_ref.so
[ -f "$REF" ] || { echo "no $REF"; exit 1; }
export HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS=${VARIANTS:-"8192:65536 16384:65536 ref:65536"}
CFGS=${CFGS:-"2 1;2 4;64 1"}
: > $OUT/refill_ab.jsonl
for rep in $(seq 1 ${REPS:-5}); do
  IFS=';' read -ra CL <<< "$CFGS"
  for cfg in "${CL[@]}"; do
    set -- $cfg
    for vr in $VARIANTS; do
      v=${vr%%:*}; ring=${vr#*:}
      if [ $v = ref ]; then hooks="host:$REF"; else hooks=device; fi
      ZSX_REFILL_CHUNK=$v timeout -k 10 60 zsummerx_amd/bin/frame_stress --rc4 "$hooks" --sessions $1 --depth $2 \
          --ring $ring --seconds 2 --warmup 0.5 | sed "s/^{/{\"chunk\": \"$v\", \"ring_arg\": $ring, /" \
          >> $OUT/refill_ab.jsonl 2>> $OUT/refill_ab.err
      rc=$?
      if [ $rc -ne 0 ]; then echo "[refill $cfg $vr] rc=$rc"; exit $rc; fi
    done
  done
  echo "rep $rep done"
done
python3 - "$OUT/refill_ab.jsonl" <<'PY'
import json, statistics, sys, collections
rows = collections.defaultdict(list)
for l in open(sys.argv[1]):
    d = json.loads(l)
    assert d["mismatches"] == 0, d
    rows[(d["sessions"], d["depth"], d["chunk"], d["ring_arg"])].append(d["echo_per_s"])
for k in sorted(rows, key=lambda k: (k[0], k[1], str(k[2]), k[3])):
    print(k, round(statistics.median(rows[k])), [round(v) for v in rows[k]])
PY
