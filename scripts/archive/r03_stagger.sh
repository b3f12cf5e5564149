set -u
# cfg2 prologue probe (scripts/r03_prologue.sh), then the cfg5 prologue-stagger
# A/B (ZRC4_PSTAGGER) and the stream timeline with CU placement.
mkdir -p gpurun_out/r03
bash scripts/r03_prologue.sh || exit 1
timeout -k 10 300 python -u tools/ab_bench.py --variant base: --variant s4:ZRC4_PSTAGGER=4 \
    --variant s8:ZRC4_PSTAGGER=8 --variant s12:ZRC4_PSTAGGER=12 --variant p8:ZRC4_PSTAGGER=8,ZRC4_PSTAGGER_SEL=1 \
    --workloads cfg5,262144x1024 --rounds 9 --launches 20 > gpurun_out/r03/ab_pstagger.log 2>&1 || { tail -20 gpurun_out/r03/ab_pstagger.log; exit 5; }
cat gpurun_out/r03/ab_pstagger.log | grep -v amdgpu.ids
timeout -k 10 200 python -u tools/stream_timeline.py --workloads cfg5 > gpurun_out/r03/tl_stream_place.log 2>&1 || exit 6
timeout -k 10 200 python -u tools/stream_timeline.py --workloads cfg5 --define ZRC4_PSTAGGER=8 > gpurun_out/r03/tl_stream_s8.log 2>&1 || exit 7
for f in place s8; do grep '^cfg5 ' gpurun_out/r03/tl_stream_$f.log | cut -c1-900; done
