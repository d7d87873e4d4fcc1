# SQ counters of the 3x3 conv kernels on a few bench layers (two passes, each its own run):
#   bash tools/pmc_conv.sh [conv_bench args...]   (default: --layers enc1_2,enc2_2,dec3_2 --only fwd)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ARGS=${*:-"--layers enc1_2,enc2_2,dec3_2 --only fwd"}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcA -o p -- python3 $R/tools/conv_bench.py --iters 3 $ARGS > $R/gpurun_out/pmcA.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcB -o p -- python3 $R/tools/conv_bench.py --iters 3 $ARGS > $R/gpurun_out/pmcB.log 2>&1
