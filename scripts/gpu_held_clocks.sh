# The clock each side workload's kernels hold (profiles/held_clock.json, bench.py's lds_roofline): for every workload,
# its bench line (the roofline kernel's un-profiled launch time), a counter-free kernel trace (the other direction's
# launches) and one GRBM_GUI_ACTIVE pass (GPU-busy cycles per dispatch).  scripts/collect_profiles.py --clocks-only.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-clocks}
mkdir -p $OUT
for w in ${WORKLOADS:-16k 16k-max 16k-max-aes128 ragged}; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-workloads >> $OUT/bench_other.jsonl 2>> $OUT/bench.err
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-workloads > $OUT/trace_$w.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE --kernel-trace -d $OUT/pmc_clk_$w -o run --output-format csv -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_clk_$w.log 2>&1
done
