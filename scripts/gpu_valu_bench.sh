set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/valu_bench
mkdir -p $OUT
timeout -k 10 120 python scripts/valu_bench.py run > $OUT/out.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc -o run --output-format csv -- python scripts/valu_bench.py run > $OUT/pmc.log 2>&1
