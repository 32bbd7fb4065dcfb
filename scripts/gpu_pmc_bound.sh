# SQ counters (LDS busy, VALU, bank conflicts, clock) of the batch seal at 1400 B and 16 KiB AES-128, then the power
# and clock the board holds under each workload.   gpurun -- 'TAG=r03q bash scripts/gpu_pmc_bound.sh'
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-bound}
mkdir -p $OUT
for w in 1400 16k-aes128; do
  ABLATE_VARIANTS=${ABLATE_VARIANTS:-gh8,gh8pair,gh8nt} timeout -k 10 240 python -u scripts/ablate.py run --workload $w --rounds 6 >> $OUT/ablate.txt 2>&1
done
cat $OUT/ablate.txt
for w in 1400 16k-aes128; do
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_sq_$w -o run --output-format csv -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 > $OUT/pmc_sq_$w.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc_sq2_$w -o run --output-format csv -- python bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-workloads --check 0 > $OUT/pmc_sq2_$w.log 2>&1
done
TAG=${TAG:-bound} bash scripts/power_probe.sh
