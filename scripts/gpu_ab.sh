# Interleaved A/B of two engine builds on one box (the same bench command, alternating):
#   A = rapido_amd/_lib/libptls_mi355x.so (HEAD), B = $B_LIB
#   gpurun -- 'B_LIB=scripts/_bin/r1/libptls_mi355x.so ARGS="--workload 1400" bash scripts/gpu_ab.sh'
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --no-workloads --steps 10 --warmup 2 $ARGS >> $OUT/a.jsonl
  PTLS_MI355X_LIB=$B_LIB timeout -k 10 120 python bench.py --no-cpu-baseline --no-e2e --no-workloads --steps 10 --warmup 2 $ARGS >> $OUT/b.jsonl
done
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
for f in ("a", "b"):
    rows = [json.loads(l) for l in open(f"{out}/{f}.jsonl")]
    print(f, [r["value"] for r in rows], [r["seal_gibps"] for r in rows], [r["open_gibps"] for r in rows])
PY
