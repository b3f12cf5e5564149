set -u
# Stream kernel at 4 KiB vs 1 KiB messages: HBM traffic per launch
mkdir -p gpurun_out/r03/pmc4k
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  for W in 524288x1024 524288x4096; do
    timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03/pmc4k/${W}_$C -o run -- \
      python3 $GRAFT_REPO_ROOT/tools/ab_bench.py --variant base: --workloads $W --rounds 2 --launches 6 --segment --footprint-mib 256 \
      > $GRAFT_REPO_ROOT/gpurun_out/r03/pmc4k/${W}_$C.log 2>&1 || exit 3
    echo "$W $C ok"
  done
done
