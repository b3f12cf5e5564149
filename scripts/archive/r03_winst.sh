set -u
# Window-kernel store cache policy A/B (ZRC4_WIN_ST), back-to-back launches
# like bench.py (--segment) and one event pair per launch.
mkdir -p gpurun_out/r03
V="--variant base: --variant nt:ZRC4_WIN_ST=1 --variant scsc:ZRC4_WIN_ST=2 --variant sc1:ZRC4_WIN_ST=3"
timeout -k 10 300 python -u tools/ab_bench.py $V --workloads cfg2,cfg4,8192x1024 --rounds 11 --launches 20 --segment > gpurun_out/r03/ab_winst_seg.log 2>&1 || { tail -20 gpurun_out/r03/ab_winst_seg.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/ab_winst_seg.log | grep -v '^{'
timeout -k 10 300 python -u tools/ab_bench.py $V --workloads cfg2 --rounds 11 --launches 20 > gpurun_out/r03/ab_winst.log 2>&1 || { tail -20 gpurun_out/r03/ab_winst.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r03/ab_winst.log | grep -v '^{'
