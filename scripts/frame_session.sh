#!/bin/bash
# GPU-box session for the batched session engine:
# wire-parity tests against the oracle peer, then the config-1 loopback
# (example/frameStressTest analogue) at several session counts with the gfx950
# hooks (reservoir = keystream rings in pinned host memory, and direct), the
# reference's own RC4 on the CPU (oracle/_ref) and RC4 off; then a rocprofv3
# kernel trace of the 2-session loopback.
#   usage: scripts/frame_session.sh [seconds] [skip-tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
SECS="${1:-2}"
REF=oracle/_ref/libzrc4_ref.so
[ -f "$REF" ] || REF=oracle/liboracle.so

if [ "${2:-}" != "skip-tests" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_frame.py tests/test_hooks.py -m gpu -x -v --timeout 120 \
      --timeout-method thread -p no:cacheprovider > $OUT/frame_tests.log 2>&1
  rc=$?; tail -3 $OUT/frame_tests.log; echo "[frame-tests] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi

: > $OUT/frame_loopback.jsonl
for cfg in "2 1" "2 4" "64 1" "64 4" "512 1" "512 4" "2048 2"; do
  set -- $cfg
  for hooks in device device-direct "host:$REF" off; do
    timeout -k 10 60 zsummerx_amd/bin/frame_stress --rc4 "$hooks" --sessions $1 --depth $2 \
        --seconds $SECS --warmup 0.5 >> $OUT/frame_loopback.jsonl 2>> $OUT/frame_loopback.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "[loopback $cfg $hooks] rc=$rc"; exit $rc; fi
  done
done
python3 - <<'PY'
import json
print("%-20s %8s %6s %12s %10s %8s" % ("hooks", "sessions", "depth", "echo/s", "us/call", "spans"))
for l in open("gpurun_out/frame_loopback.jsonl"):
    d = json.loads(l)
    print("%-20s %8d %6d %12.0f %10.1f %8.1f %s %s" % (d["rc4"], d["sessions"], d["depth"], d["echo_per_s"],
          d["rc4_us_per_call"], d["spans_per_call"], "" if d["mismatches"] == 0 else "MISMATCH",
          json.dumps(d.get("hooks", {}))))
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof_loopback -o run --output-format csv \
    -- $GRAFT_REPO_ROOT/zsummerx_amd/bin/frame_stress --rc4 device --sessions 2 --depth 1 --seconds $SECS --warmup 0.5 \
    > $GRAFT_REPO_ROOT/$OUT/prof_loopback.log 2>&1
rc=$?; echo "[rocprof loopback] rc=$rc"; tail -1 $GRAFT_REPO_ROOT/$OUT/prof_loopback.log
echo done
