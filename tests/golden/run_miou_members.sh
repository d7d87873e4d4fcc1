#!/bin/bash
# Reference mIoU runs on the CPU (make_golden.py imports the reference): the selective-metric set's
# unperturbed run, then perturbed members of both 256x256 sets, PAR processes of THREADS threads at a time.
#   bash tests/golden/run_miou_members.sh "s:1 s:2 ... h:3 ..."      (1e-7 input-perturbed members)
#   bash tests/golden/run_miou_members.sh "h:c1 h:c2 ..."             (3e-7 conv-output-noise members)
# then: python tests/golden/make_golden.py miou256x_collect s 1 2 ...  (miou256c_collect h 1 2 ... for c)
cd "$(dirname "$0")/../.." || exit 1
export OMP_NUM_THREADS=${THREADS:-4}
mkdir -p gpurun_out/miou_ref
jobs=${1:-"s:0 s:1 s:2 s:3 s:4 s:5 s:6 s:7 s:8 h:3 h:4 h:5 h:6 h:7 h:8"}
for j in $jobs; do echo "$j"; done | xargs -P "${PAR:-2}" -I{} bash -c '
  tag=${1%%:*}; k=${1##*:}
  if [ "$k" = 0 ]; then cmd="python tests/golden/make_golden.py miou256$tag"
  elif [ "${k:0:1}" = c ]; then cmd="python tests/golden/make_golden.py miou256c_member $tag ${k:1}"
  else cmd="python tests/golden/make_golden.py miou256x_member $tag $k"; fi
  t0=$(date +%s); $cmd > gpurun_out/miou_ref/$tag$k.log 2>&1; rc=$?
  echo "$1 rc=$rc $(( $(date +%s) - t0 )) s: $(tail -1 gpurun_out/miou_ref/$tag$k.log)"
' _ {}
