# Window-kernel latency A/B across engine builds (scripts/ablate.py build): one window_bench per variant, twice.
#   gpurun -- 'VARIANTS="base head" bash scripts/gpu_win_ab.sh'
set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${TAG:-winab}
mkdir -p $OUT
for rep in 1 2; do
  for v in ${VARIANTS:-base head}; do
    PTLS_MI355X_LIB=rapido_amd/_lib/variants/$v.so timeout -k 10 200 python scripts/window_bench.py --reps 300 --out $OUT/${v}_$rep.json > $OUT/${v}_$rep.log 2>&1
  done
done
