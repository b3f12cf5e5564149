set -u
# xcd_run_map (ZRC4_WMAP=1) for crypt_kernel and crypt_half_kernel: parity
# subset on the variant, then same-process timing.
mkdir -p gpurun_out/r03/wmap
ZSX_ZRC4_VARIANT=wm timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/wmap/tests_wm.log 2>&1 || { tail -30 gpurun_out/r03/wmap/tests_wm.log; exit 1; }
tail -1 gpurun_out/r03/wmap/tests_wm.log
timeout -k 10 500 python -u tools/ab_bench.py --variant base: --variant wm:ZRC4_WMAP=1 \
  --workloads 65536x128,cfg3,65536x1024,65536x2048,16384x1024,32768x1024,16384x256,32768x256,12288x1024,65536x512 --rounds 9 --launches 20 --segment > gpurun_out/r03/wmap/ab5.log 2>&1 || { tail -20 gpurun_out/r03/wmap/ab5.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r03/wmap/ab5.log | grep -v '^{'
