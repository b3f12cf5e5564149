set -u
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k dispatch --timeout 120 --timeout-method thread > gpurun_out/r03/dispatch_tests.log 2>&1 || { echo dispatch_fail; tail -30 gpurun_out/r03/dispatch_tests.log; exit 1; }
tail -3 gpurun_out/r03/dispatch_tests.log
timeout -k 10 120 python tools/kernel_timeline.py --workloads cfg2 --footprint-mib 8 > gpurun_out/r03/tl_win_fp8.log 2>&1 || exit 2
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python tools/kernel_timeline.py --workloads cfg2 > gpurun_out/r03/tl_win_devkarg.log 2>&1 || exit 3
timeout -k 10 120 python tools/kernel_timeline.py --workloads cfg2 > gpurun_out/r03/tl_win_base.log 2>&1 || exit 4
for f in fp8 devkarg base; do grep '^cfg2 ' gpurun_out/r03/tl_win_$f.log | cut -c1-420; done
