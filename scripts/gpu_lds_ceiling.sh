# The LDS ceiling of the batch kernels' read mix, pinned: the probe (scripts/lds_ceiling.hip) and the
# batch kernels under the same LDS counters, one box: LDS-array active cycles (SQ_LDS_IDX_ACTIVE) per 64 blocks are the
# mix's LDS work, and the wall cycles per 64 blocks (GRBM_GUI_ACTIVE / 8 per launch, in-kernel clock for the probe) what
# each achieves.   gpurun -- 'bash scripts/gpu_lds_ceiling.sh' -> gpurun_out/${TAG:-ldsceil}/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ldsceil}
mkdir -p $OUT
C="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
timeout -k 10 120 python scripts/lds_ceiling.py run $OUT/probe.json > $OUT/probe.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_probe -o run --output-format csv -- python scripts/lds_ceiling.py run > $OUT/pmc_probe.log 2>&1
for w in 16k-aes128 1400 16k; do
  timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace -d $OUT/pmc_$w -o run --output-format csv -- python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 > $OUT/pmc_$w.log 2>&1
done
