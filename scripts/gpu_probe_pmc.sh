# PMC passes over the bitsliced/T-table probe (scripts/probe_bs.py), one counter set per pass
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-probe_pmc}
mkdir -p $OUT
for ntt in ${NTTS:-0 16 8}; do
  PROBE_KEYS=16 PROBE_NTT=$ntt timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS:-SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE} --kernel-trace -d $OUT/ntt$ntt -o run --output-format csv -- python scripts/probe_bs.py run > $OUT/ntt$ntt.log 2>&1
done
