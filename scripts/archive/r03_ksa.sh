set -u
# KSA (zrc4_ksa_range) time by key length on this box: register-pattern
# lengths (16, 32, 8) against the generic fetch path (13, 24, 40, 100).
mkdir -p gpurun_out/r03/ksa
for kl in 16 32 8 13 24 40 100; do
  timeout -k 10 200 python -u tools/ab_bench.py --variant base: --workloads cfg2,cfg5 --rounds 5 --launches 10 --ksa --key-len $kl > gpurun_out/r03/ksa/kl$kl.log 2>&1 || { tail -5 gpurun_out/r03/ksa/kl$kl.log; exit 1; }
  echo "kl=$kl $(grep _ksa gpurun_out/r03/ksa/kl$kl.log | grep -v '^{' | tr '\n' ' ')"
done
