# The resident grid against the launched record layer, one window per submit (rapido's operating point, one
# connection: lib/rapido.c:2115-2126), depths 1 / 4 / 16, seal and open from one box.
#   launched, dma_in: coalescing on (default 16 windows per launch), inputs by DMA, outputs in place
#   launched, direct: coalescing on, inputs read in place
#   resident:         every window's runs (and an open's delivery) as jobs of the persistent grid -- measured on the
#                     round-5 start build (profiles/r05a_resident_vs_launched.json), then removed with the grid; set
#                     TRANSPORTS to re-run the launched ones alone
#   gpurun -- 'bash scripts/rl_resident_ab.sh' -> gpurun_out/${TAG:-rlres}/
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-rlres}
mkdir -p $OUT
for rep in 1 2; do
  for d in 1 4 16; do
    for tr in ${TRANSPORTS:-dma_in direct}; do
      timeout -k 10 60 scripts/_build/rl_stream 64 $d 16 $tr 1 > $OUT/${tr}_d${d}_r$rep.json
      echo "$tr depth $d rep $rep: $(tail -c 300 $OUT/${tr}_d${d}_r$rep.json)"
    done
  done
done
