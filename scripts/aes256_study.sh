# AES-256 at 16 KiB (configs[2], the kernel furthest below its roofline): what binds it -- package power, LDS, VALU --
# and whether the mixed bitsliced + T-table engine (scripts/probe_bs.hip) would lift it on today's box.
#   gpurun -- 'bash scripts/aes256_study.sh'  ->  gpurun_out/${TAG:-aes256}/   (summarised by scripts/aes256_summary.py)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-aes256}
mkdir -p $OUT
timeout -k 5 20 amd-smi metric -p -c --json > $OUT/idle.json 2>&1 || true
# 1. compute-only sweep (no HBM traffic): T-table waves per 16-wave workgroup, the rest bitsliced
PROBE_NTT=16,12,10,8,6,0 timeout -k 10 200 python scripts/probe_bs.py run > $OUT/probe_sweep.log 2>&1
# 2. power and clock under the probe, AES-256, T-table only (16) vs the best mix (8 + 8), ~20 s each
for ntt in 16 8; do
  PROBE_KEYS=32 PROBE_NTT=$ntt PROBE_REPS=1400 PROBE_UNITS_MULT=64 timeout -k 10 150 python scripts/probe_bs.py run > $OUT/probe_power_$ntt.log 2>&1 &
  pid=$!
  sleep 15
  for i in 1 2 3 4 5; do timeout -k 5 20 amd-smi metric -p -c --json > $OUT/probe_${ntt}_$i.json 2>&1 || true; sleep 1; done
  wait $pid
done
# 3. power and clock under the AES-256 batch kernels (bench.py, 16 KiB records)
timeout -k 10 150 python bench.py --workload 16k --steps 2500 --warmup 2 --no-cpu-baseline --no-e2e --no-workloads --check 0 > $OUT/bench_16k.json 2> $OUT/bench_16k.err &
pid=$!
sleep 12
for i in 1 2 3 4 5; do timeout -k 5 20 amd-smi metric -p -c --json > $OUT/bench_16k_$i.json 2>&1 || true; sleep 1; done
wait $pid
# 4. PMC of the AES-256 batch launches, one counter set per pass
B="python bench.py --workload 16k --steps 3 --warmup 1 --prewarm-ms 0 --no-cpu-baseline --no-e2e --no-workloads --check 0"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $set --kernel-trace -d $OUT/pmc_$i -o run --output-format csv -- $B > $OUT/pmc_$i.log 2>&1
done
