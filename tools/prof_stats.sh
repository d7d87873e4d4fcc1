#!/bin/bash
# rocprofv3 kernel-trace statistics of one bench.py configuration on the GPU box:
#   bash tools/prof_stats.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/ (CSV) + <tag>_stats.log
set -o pipefail
tag=$1; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o p -- \
  python3 "$root/bench.py" --no-cpu-baseline --no-kernel-timing --no-full-loop --no-exact --no-bf16 "$@" \
  > "$out/run.log" 2>&1
rc=$?
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && head -40 "$f" > "$root/gpurun_out/${tag}_stats.log"
exit $rc
