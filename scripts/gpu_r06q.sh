# Round 6: the record layer's host-to-host stream with the windows of 8 sessions
# per launch (multi-key) against 8 connections of one session and against the same sessions submitted apart.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06q}
mkdir -p $OUT
# a launch of 8 windows is one of a layer's 4 launch slots: 4 in flight; submitted apart, the 8 sessions' layers have
# 4 slots each (and coalesce their own queued windows)
for t in dma_in direct; do
  for run in "4 16 $t 8" "4 16 $t 8 sessions" "4 16 $t 8 sessions_apart" "16 16 $t 8 sessions_apart" "32 16 $t 8 sessions_apart"; do
    timeout -k 10 120 scripts/_build/rl_stream 64 $run >> $OUT/rl_sessions.jsonl 2>> $OUT/rl_sessions.err || { tail -5 $OUT/rl_sessions.err; exit 1; }
  done
done
cat $OUT/rl_sessions.jsonl
