set -u
# cfg5: issue priority to the CU's later-starting workgroup (ZRC4_PRIO 2/3)
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u tools/ab_bench.py --variant base: --variant p2:ZRC4_PRIO=2 --variant p3:ZRC4_PRIO=3 \
    --workloads cfg5,262144x1024,131072x1024 --rounds 11 --launches 20 --segment > gpurun_out/r03/ab_prio_late.log 2>&1 || { tail -20 gpurun_out/r03/ab_prio_late.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/ab_prio_late.log | grep -v '^{'
timeout -k 10 200 python -u tools/stream_timeline.py --workloads cfg5 --footprint-mib 640 --define ZRC4_PRIO=2 --dump gpurun_out/r03/tl5/p2 > gpurun_out/r03/tl5/p2.log 2>&1 || exit 2
grep '^cfg5 ' gpurun_out/r03/tl5/p2.log | cut -c1-400
