#!/bin/bash
# Collect the round's rocprofv3 evidence for bench.py on the GPU box (run from the repo root):
#   kernel-trace stats, then FETCH_SIZE, WRITE_SIZE and SQ counter passes, each its own run.
#   bash tools/profile_round.sh r01
# Outputs land in gpurun_out/prof_<tag>/; copy the summaries into profiles/ afterwards with
#   python tools/pmc_summary.py ....
set -o pipefail
tag=${1:-r01}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
B="python3 $root/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-full-loop ${BENCH_ARGS:-}"
run() {  # name seconds rocprof-args...
  local name=$1 secs=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 -s KILL "$secs" rocprofv3 "$@" --output-format csv -d "$out/$name" -o p -- $B \
    > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >&2
  return $rc
}
run stats 240 --kernel-trace --stats &&
run fetch 120 --pmc FETCH_SIZE &&
run write 120 --pmc WRITE_SIZE &&
run sq 120 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
rc=$?
find "$out" -name '*.csv' | sort >&2
exit $rc
