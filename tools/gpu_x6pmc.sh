#!/bin/bash
# rocprofv3 passes over one bf16x6 GEMM shape (tools/gemm_x6_pmc.py); output under gpurun_out/x6pmc_$TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/x6pmc_${TAG:-a}
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p1.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d $O/p2 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p2.log 2>&1 || exit 3
python3 $R/tools/gemm_x6_pmc.py --summary $O/p1 $O/p2 > $O/summary.json
grep -h "gemm_x6" $O/trace/run_kernel_stats.csv | cut -c1-200 >> $O/summary.json
cat $O/summary.json
