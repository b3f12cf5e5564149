set -u
# WMAP block size B (contiguous groups per XCD turn): 1 (identity) .. 32 (one run per XCD at 256 groups)
mkdir -p gpurun_out/r03/wmap
V="--variant base: --variant b2:ZRC4_WMAP=2 --variant b4:ZRC4_WMAP=4 --variant b8:ZRC4_WMAP=8 --variant b32:ZRC4_WMAP=32"
timeout -k 10 400 python -u tools/ab_bench.py $V --workloads 65536x128,cfg3,65536x512,65536x1024,65536x2048 --rounds 9 --launches 20 --segment > gpurun_out/r03/wmap/ab3.log 2>&1 || { tail -20 gpurun_out/r03/wmap/ab3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/wmap/ab3.log | grep -v '^{'
cd /tmp && export TMPDIR=/tmp
for V in b2 b4 b8; do
  ZSX_ZRC4_VARIANT=$V timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03/wmap/${V}_WRITE_SIZE -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload cfg3 --steps 20 --warmup 2 --cpu-seconds 0 --companion-workload none > $GRAFT_REPO_ROOT/gpurun_out/r03/wmap/${V}_WRITE_SIZE.log 2>&1 || exit 4
done
echo pmc done
