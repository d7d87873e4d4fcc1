#!/bin/bash
# SQ/GRBM counters (clock, MFMA busy) of the split-fp16 conv under the build and two ablation libraries
# (_ab/libselunet_a64.so: constant fragments, _ab/libselunet_a16.so: no MFMAs; tools/ablate.sh). GPU box.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in base a64 a16; do
  lib=$R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so
  [ $v != base ] && lib=$R/_ab/libselunet_$v.so
  SELUNET_LIB=$lib timeout -k 10 -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_$v -o p -- python3 $R/tools/conv_bench.py --dtype fp32 --x2 --iters 10 --only fwd --layers dec3_1,enc1_2 > $R/gpurun_out/pmc_$v.log 2>&1 || exit 1
  echo "$v done"
done
