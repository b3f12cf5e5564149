set -u
# crypt_kernel workgroup -> group map: WPERM (97k mod grid, product) vs XCD-
# contiguous groups (ZRC4_WMAP=1) vs identity; cfg3 write traffic per variant.
mkdir -p gpurun_out/r03/wmap
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "ragged or baseline_configs or dispatch" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/wmap/tests_base.log 2>&1 || { tail -20 gpurun_out/r03/wmap/tests_base.log; exit 1; }
ZSX_ZRC4_VARIANT=xmap timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "ragged or baseline_configs or dispatch" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/wmap/tests_xmap.log 2>&1 || { tail -20 gpurun_out/r03/wmap/tests_xmap.log; exit 2; }
tail -1 gpurun_out/r03/wmap/tests_base.log gpurun_out/r03/wmap/tests_xmap.log
timeout -k 10 300 python -u tools/ab_bench.py --variant base: --variant xmap:ZRC4_WMAP=1 --variant noperm:ZRC4_WPERM=0 \
   --workloads cfg3,65536x512,65536x1024,32768x256,262144x128 --rounds 9 --launches 20 --segment > gpurun_out/r03/wmap/ab.log 2>&1 || { tail -20 gpurun_out/r03/wmap/ab.log; exit 3; }
grep -v amdgpu.ids gpurun_out/r03/wmap/ab.log | grep -v '^{'
cd /tmp && export TMPDIR=/tmp
for V in base xmap noperm; do
  for C in WRITE_SIZE FETCH_SIZE; do
    ZSX_ZRC4_VARIANT=$V timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03/wmap/${V}_$C -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload cfg3 --steps 20 --warmup 2 --cpu-seconds 0 --companion-workload none > $GRAFT_REPO_ROOT/gpurun_out/r03/wmap/${V}_$C.log 2>&1 || exit 4
  done
done
echo pmc done
