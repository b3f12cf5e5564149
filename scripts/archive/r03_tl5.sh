set -u
# cfg5 stream-kernel timeline at the bench's footprint (640 MiB: one batch,
# R = 1) and at 1200 MiB (R = 2), raw stamps dumped for offline analysis.
mkdir -p gpurun_out/r03/tl5
for fp in 640 1200; do
  timeout -k 10 200 python -u tools/stream_timeline.py --workloads cfg5 --footprint-mib $fp --dump gpurun_out/r03/tl5/fp$fp > gpurun_out/r03/tl5/fp$fp.log 2>&1 || exit 1
  grep '^cfg5 ' gpurun_out/r03/tl5/fp$fp.log | cut -c1-700
done
