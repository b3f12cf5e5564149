#!/bin/bash
# Round-2 probe 26: same-box A/B of the reservoir's host XOR threads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/xor_ab.jsonl
: > $OUT
for rep in 1 2; do
for cfg in "64 4" "512 4" "2048 2"; do
  set -- $cfg
  for t in 1 2 4 8; do
    ZSX_XOR_THREADS=$t timeout -k 10 60 zsummerx_amd/bin/frame_stress --rc4 device --sessions $1 --depth $2 \
        --seconds 2 --warmup 0.5 | sed "s/^{/{\"xor_threads_env\": $t, /" >> $OUT
    rc=$?; [ $rc -eq 0 ] || { echo "[xor $cfg $t] rc=$rc"; exit $rc; }
  done
  timeout -k 10 60 zsummerx_amd/bin/frame_stress --rc4 device-direct --sessions $1 --depth $2 --seconds 2 --warmup 0.5 \
      | sed 's/^{/{"xor_threads_env": -1, /' >> $OUT
done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/xor_ab.jsonl"):
    d = json.loads(l)
    print(d["sessions"], d["depth"], d["xor_threads_env"], round(d["echo_per_s"]), round(d["rc4_us_per_call"], 1))
PY
