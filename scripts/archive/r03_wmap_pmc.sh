set -u
# cfg3 L2 behaviour by workgroup->group order: r02 order (ZRC4_WMAP=0) vs the XCD runs (product)
mkdir -p gpurun_out/r03/wmap_pmc
cd /tmp && export TMPDIR=/tmp
for V in wm0 prod; do
  for SET in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"; do
    tag=$(echo $SET | cut -c1-6)
    if [ $V = prod ]; then unset ZSX_ZRC4_VARIANT; else export ZSX_ZRC4_VARIANT=$V; fi
    timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r03/wmap_pmc/${V}_$tag -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --workload cfg3 --steps 20 --warmup 2 --cpu-seconds 0 --companion-workload none > $GRAFT_REPO_ROOT/gpurun_out/r03/wmap_pmc/${V}_$tag.log 2>&1 || exit 3
    echo "$V $tag ok"
  done
done
