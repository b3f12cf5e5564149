set -u
# WMAP sweep over message sizes at 256 groups (crypt_kernel), two repetitions.
mkdir -p gpurun_out/r03/wmap
for rep in 1 2; do
timeout -k 10 400 python -u tools/ab_bench.py --variant base: --variant xmap:ZRC4_WMAP=1 \
   --workloads 65536x128,cfg3,65536x384,65536x512,65536x768,65536x1024,65536x2048,49152x1024,49152x256 --rounds 9 --launches 20 --segment > gpurun_out/r03/wmap/ab2_$rep.log 2>&1 || { tail -20 gpurun_out/r03/wmap/ab2_$rep.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/wmap/ab2_$rep.log | grep -v '^{'
done
