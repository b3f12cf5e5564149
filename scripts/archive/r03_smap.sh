set -u
# crypt_stream_kernel: XCD-contiguous groups per round (ZRC4_SMAP=1)
mkdir -p gpurun_out/r03/smap
ZSX_ZRC4_VARIANT=sm timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "ragged or baseline_configs or dispatch or staged" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/smap/tests_sm.log 2>&1 || { tail -30 gpurun_out/r03/smap/tests_sm.log; exit 1; }
tail -1 gpurun_out/r03/smap/tests_sm.log
timeout -k 10 500 python -u tools/ab_bench.py --variant base: --variant sm:ZRC4_SMAP=1 \
  --workloads cfg5,262144x1024,131072x1024,1048576x256,524288x512 --rounds 9 --launches 20 --segment > gpurun_out/r03/smap/ab.log 2>&1 || { tail -20 gpurun_out/r03/smap/ab.log; exit 2; }
grep -v amdgpu.ids gpurun_out/r03/smap/ab.log | grep -v '^{'
