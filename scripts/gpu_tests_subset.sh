#!/bin/bash
# A subset of the GPU suite (the files given), one pytest process, stopping at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${TAG:-subset}
mkdir -p "$out"
timeout -k 10 ${LIMIT:-900} python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu "$@" > "$out/tests.log" 2>&1
rc=$?
tail -5 "$out/tests.log"
exit $rc
