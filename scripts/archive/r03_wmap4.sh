set -u
# WMAP=8 with and without streaming (nt) payload stores in crypt_kernel
mkdir -p gpurun_out/r03/wmap
V="--variant base: --variant b8:ZRC4_WMAP=8 --variant b8nt:ZRC4_WMAP=8,ZRC4_ST_NT=1 --variant nt:ZRC4_ST_NT=1"
timeout -k 10 400 python -u tools/ab_bench.py $V --workloads 65536x128,cfg3,65536x512,65536x1024,65536x2048,49152x1024 --rounds 9 --launches 20 --segment > gpurun_out/r03/wmap/ab4.log 2>&1 || { tail -20 gpurun_out/r03/wmap/ab4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/wmap/ab4.log | grep -v '^{'
