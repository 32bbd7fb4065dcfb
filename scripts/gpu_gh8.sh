# round 3: GH8 latin tables against the nibble tables (interleaved A/B on one box), then the full GPU suite,
# smoke and the bench line on the GH8 build.   gpurun --timeout 1200 -- 'bash scripts/gpu_gh8.sh'
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r03p}
mkdir -p $OUT
for w in 1400 16k-aes128 16k; do
  ABLATE_VARIANTS=nogh8,gh8 timeout -k 10 240 python -u scripts/ablate.py run --workload $w --rounds 6 >> $OUT/ablate_gh8.txt 2>&1
done
cat $OUT/ablate_gh8.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > $OUT/bench_1400.json 2> $OUT/bench.err
cat $OUT/bench_1400.json
