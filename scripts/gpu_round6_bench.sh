# Round-end style measurement: bench lines for every workload, rocprofv3 kernel-trace summary
# of the default bench, and the PMC passes (FETCH_SIZE / WRITE_SIZE separately) for traffic.
set -e
# (round 6: the multi-key workload 1400-mk64 in every loop)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}
mkdir -p $OUT
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --e2e > $OUT/bench_1400.json 2> $OUT/bench.err
for w in 16k 16k-aes128 16k-max 16k-max-aes128 ragged 1400-mk64; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-workloads >> $OUT/bench_other.jsonl 2>> $OUT/bench.err
done
# the same steps, warmups and pre-warm as the bench lines, so the timed launches' durations reproduce roofline.frac
# (PMC passes: no pre-warm, bytes per launch do not depend on the clock)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-workloads > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_sq -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_sq.log 2>&1
# SQ counters of the north-star workload (16 KiB AES-128): LDS busy cycles per block
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_sq_16k-aes128 -o run --output-format csv -- python bench.py --workload 16k-aes128 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_sq_16k-aes128.log 2>&1
# HBM traffic of the other workloads (roofline.traffic of their bench lines): FETCH / WRITE in separate passes
for w in 16k 16k-aes128 16k-max 16k-max-aes128 ragged 1400-mk64; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch_$w -o run --output-format csv -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_fetch_$w.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write_$w -o run --output-format csv -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_write_$w.log 2>&1
done
# GPU-busy cycles of the other workloads' kernels (profiles/held_clock.json: the clock their lds_roofline is priced at)
for w in 16k 16k-max 16k-max-aes128 ragged 1400-mk64; do
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE --kernel-trace -d $OUT/pmc_clk_$w -o run --output-format csv -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 --prewarm-ms 0 > $OUT/pmc_clk_$w.log 2>&1
done
# rocprofv3 kernel-trace summaries of the other workloads (profiles/<label>_kernel_stats_<w>.csv)
for w in 16k 16k-aes128 16k-max 16k-max-aes128 ragged 1400-mk64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$w -o run --output-format csv -- python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-workloads > $OUT/trace_$w.log 2>&1
done
