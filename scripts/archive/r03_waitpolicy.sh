set -u
# Host wait policy vs the bench's fixed per-region cost: the HIP runtime spins
# for ROC_ACTIVE_WAIT_TIMEOUT us before sleeping on an interrupt (default 50).
mkdir -p gpurun_out/r03/wait
timeout -k 10 200 python -u tools/sync_probe.py --ks 20,200 --reps 11 > gpurun_out/r03/wait/default.log 2>&1 || exit 1
ROC_ACTIVE_WAIT_TIMEOUT=20000 timeout -k 10 200 python -u tools/sync_probe.py --ks 20,200 --reps 11 > gpurun_out/r03/wait/spin20ms.log 2>&1 || exit 2
for f in default spin20ms; do echo "== $f"; grep -v amdgpu.ids gpurun_out/r03/wait/$f.log | grep -v '^{'; done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --companion-workload none > gpurun_out/r03/wait/bench_default.log 2>&1 || exit 3
ROC_ACTIVE_WAIT_TIMEOUT=20000 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --companion-workload none > gpurun_out/r03/wait/bench_spin.log 2>&1 || exit 4
for f in bench_default bench_spin; do grep '^{' gpurun_out/r03/wait/$f.log | cut -c1-200; done
