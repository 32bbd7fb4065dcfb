set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/lds_bench
mkdir -p $OUT
LDS_THREADS=1024 timeout -k 10 120 python scripts/lds_bench.py run > $OUT/out.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d $OUT/pmc -o run --output-format csv -- python scripts/lds_bench.py run > $OUT/pmc.log 2>&1
