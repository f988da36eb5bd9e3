#!/bin/bash
# PMC passes over the verify kernel (one counter group per rocprofv3 run; see MI355X_MICROARCH.md).
set -e
OUT=${1:-gpurun_out/pmc}
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--n ${CV_PMC_N:-1000000} --reps 2"
K="--kernel-include-regex (scalars_kernel|points_one_kernel|points_kernel|hs_straus_kernel)"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT $K -d $OUT/p1 -o p1 --output-format csv -- python3 tools/pmc_probe.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_LEVEL_WAVES $K -d $OUT/p2 -o p2 --output-format csv -- python3 tools/pmc_probe.py $ARGS > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE $K -d $OUT/p3 -o p3 --output-format csv -- python3 tools/pmc_probe.py $ARGS > $OUT/p3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE $K -d $OUT/p4 -o p4 --output-format csv -- python3 tools/pmc_probe.py $ARGS > $OUT/p4.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_I8 SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA $K -d $OUT/p5 -o p5 --output-format csv -- python3 tools/pmc_probe.py $ARGS > $OUT/p5.log 2>&1
echo pmc done
