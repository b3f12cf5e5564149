set -u
# Host-inclusive rates with the size-chosen chunking, and the box's pinned
# copy ceiling (H2D, D2H, both at once).
mkdir -p gpurun_out/r03/hostinc
timeout -k 10 120 python -u tools/hostinc_sweep.py --pcie-only > gpurun_out/r03/hostinc/pcie.log 2>&1 || exit 1
grep '^pcie' gpurun_out/r03/hostinc/pcie.log
for wl in cfg2 cfg3 cfg5; do
  timeout -k 10 200 python -u bench.py --host-inclusive --workload $wl --steps 15 --warmup 3 > gpurun_out/r03/hostinc/copy_$wl.json 2>gpurun_out/r03/hostinc/copy_$wl.err || exit 2
  timeout -k 10 200 python -u bench.py --host-inclusive --zero-copy --workload $wl --steps 15 --warmup 3 > gpurun_out/r03/hostinc/zc_$wl.json 2>gpurun_out/r03/hostinc/zc_$wl.err || exit 3
  cat gpurun_out/r03/hostinc/copy_$wl.json gpurun_out/r03/hostinc/zc_$wl.json
done
