#!/bin/bash
# Round-6 rehearsal of bench.py's multi-rank path on a one-GPU box: the
# driver's scaling run launches `torch.distributed.run --nproc-per-node N
# bench.py --gpus N` on an 8-GPU node (RCCL); here every rank runs its real
# GpuRunner shard on cuda:0 over gloo (`--rehearse-one-gpu`), through both
# launchers, with the configs[4] companion split over the ranks.  The lines
# are checked for shape (n_gpus, one per_gpu entry per rank, the companion's
# split), not for speed: the ranks share one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${REH_OUT:-gpurun_out/r06/rehearse}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name, seconds, command...
    local name=$1 secs=$2; shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "[$name] rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -2 | cut -c1-400
    if [ $rc -ne 0 ]; then echo "[$name] failed: stopping GPU work in this call"; exit $rc; fi
}
check() {  # name, N: the last JSON line has N ranks and the companion split N ways
    python3 - "$OUT/$1.log" "$2" <<'EOF' || exit 1
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d, n = json.loads(line), int(sys.argv[2])
c = d["configs4_strong"]
assert d["n_gpus"] == n and d["config"]["world_size_seen"] == n and len(d["per_gpu"]) == n, d["per_gpu"]
assert c["n_gpus"] == n and c["config"]["sessions_per_gpu"] * n == c["config"]["global_sessions_per_step"] == 524288
assert "rehearsal" in d["config"] and d["config"]["dist_backend"] == "gloo"
print(f"[check {n}] ok: value {d['value']} GiB/s, companion {c['value']} GiB/s (shared GPU: shape only)")
EOF
}
step self_launch_2 400 python bench.py --gpus 2 --steps 20 --warmup 5 --rehearse-one-gpu
check self_launch_2 2
step torchrun_4 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 4 --steps 20 --warmup 5 --rehearse-one-gpu
check torchrun_4 4
echo rehearse done
