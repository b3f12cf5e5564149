#!/bin/bash
# Round-3 engine session: frame/hooks GPU tests (adaptive hooks default), then
# the config-1 loopback sweep with the adaptive hooks (default), the reservoir
# alone (ZSX_RC4_DIRECT_BYTES=0), the direct hooks, the reference's CPU RC4
# and RC4 off.  usage: scripts/r03_engine.sh [seconds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03
OUT=gpurun_out/r03
SECS="${1:-2}"
REF=oracle/_ref/libzrc4_ref.so
[ -f "$REF" ] || REF=oracle/liboracle.so
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 400 python -u -m pytest tests/test_frame.py tests/test_hooks.py -m gpu -x -v --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $OUT/frame_tests.log 2>&1
rc=$?; tail -3 $OUT/frame_tests.log; echo "[frame-tests] rc=$rc"; [ $rc -eq 0 ] || exit $rc
fi
: > $OUT/frame_loopback.jsonl
for cfg in ${CFGS:-"2 1" "2 4" "64 1" "64 4" "512 1" "512 4" "2048 2"}; do
  set -- ${cfg//_/ }
  for mode in ${MODES:-adaptive reservoir direct adaptive reservoir direct adaptive reservoir direct reference off}; do
    case $mode in
      adaptive)  H=device;        E="" ;;
      reservoir) H=device;        E="ZSX_RC4_DIRECT_BYTES=0" ;;
      direct)    H=device-direct; E="" ;;
      reference) H="host:$REF";   E="" ;;
      off)       H=off;           E="" ;;
    esac
    env $E timeout -k 10 60 zsummerx_amd/bin/frame_stress --rc4 "$H" --sessions $1 --depth $2 \
        --seconds $SECS --warmup 0.5 > $OUT/one.json 2>> $OUT/frame_loopback.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "[loopback $cfg $mode] rc=$rc"; exit $rc; fi
    python3 -c "import json,sys; d=json.loads(open('$OUT/one.json').read().strip().splitlines()[-1]); d['mode']='$mode'; print(json.dumps(d))" >> $OUT/frame_loopback.jsonl
  done
done
python3 - <<'PY'
import json, collections
import statistics
rows = [json.loads(l) for l in open("gpurun_out/r03/frame_loopback.jsonl")]
by = collections.defaultdict(lambda: collections.defaultdict(list))
for d in rows:
    by[(d["sessions"], d["depth"])][d["mode"]].append(d)
print("median echo/s over the repetitions (runs interleaved by mode)")
print("%8s %6s %11s %11s %11s %11s %11s %8s" % ("sessions", "depth", "adaptive", "reservoir", "direct", "reference", "off", "adapt/best"))
for (s, dp), m in by.items():
    e = {k: statistics.median(x["echo_per_s"] for x in v) for k, v in m.items()}
    best = max(e["reservoir"], e["direct"])
    bad = [k for k, v in m.items() for x in v if x.get("mismatches", 0)]
    print("%8d %6d %11.0f %11.0f %11.0f %11.0f %11.0f %8.3f %s" % (s, dp, e["adaptive"], e["reservoir"], e["direct"],
          e.get("reference", 0), e.get("off", 0), e["adaptive"] / best, "MISMATCH " + str(bad) if bad else ""))
PY
echo done
