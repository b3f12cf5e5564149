set -u
# Operating envelope of the product dispatch: kernel time over session count x message size.
mkdir -p gpurun_out/r03/env
W=""
for S in 1024 4096 16384 65536 262144 524288; do
  for L in 64 256 1024 4096 16384; do
    B=$((S * L))
    if [ $B -le 2147483648 ]; then W="$W,${S}x${L}"; fi
  done
done
W=${W#,}
timeout -k 10 900 python -u tools/ab_bench.py --variant base: --workloads $W --rounds 5 --launches 10 --segment --footprint-mib 256 > gpurun_out/r03/env/envelope.log 2>&1 || { tail -20 gpurun_out/r03/env/envelope.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03/env/envelope.log | grep -v '^{' | cut -c1-160
