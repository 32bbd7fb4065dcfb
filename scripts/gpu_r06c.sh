#!/bin/bash
# round 6: the 1400-B single-key A/B again (more rounds), then the default bench line (with the multi-key workload)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-r06c}
mkdir -p "$out"
for i in 1 2; do
    ABLATE_VARIANTS=base,head timeout -k 10 300 python scripts/ablate.py run --workload 1400 --rounds 20 >> "$out/ablate.txt" 2>&1 || exit 1
done
grep -v '^{' "$out/ablate.txt" | grep K=
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 1; }
python - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "frac", d["roofline"]["frac"])
for k, w in d.get("workloads", {}).items():
    print(k, w["value"], w["seal_gibps"], w["open_gibps"], w["roofline"]["frac"], w["roofline"]["kernel"])
PY
