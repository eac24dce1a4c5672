#!/bin/bash
# rocprofv3 passes over the update's backward / weight-gradient x6 shapes at 2,097,152 rows
# (tools/gemm_x6_pmc.py): kernel-trace stats, MFMA busy + clock, the stall mix, and FETCH_SIZE /
# WRITE_SIZE in separate passes (gfx950: the two do not fit one pass); summary by tools/x6_shapes_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-r05}
for s in ${SHAPES:-bwd:256:512 bwd:512:512 bwd:512:256 wgrad:512:256 wgrad:512:512 wgrad:256:512}; do
  IFS=: read d k n <<< "$s"
  O=$R/gpurun_out/x6shape_${T}_${d}_${k}_${n}; mkdir -p $O
  export GEMM_DIR=$d K=$k N=$n
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/trace.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p1.log 2>&1 || exit 2
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS --output-format csv -d $O/p2 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p2.log 2>&1 || exit 3
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p3.log 2>&1 || exit 4
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/p4 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p4.log 2>&1 || exit 5
  echo "done $s"
done
python3 $R/tools/x6_shapes_summary.py $R/gpurun_out x6shape_${T}_ > $R/gpurun_out/x6shape_${T}_summary.json
cat $R/gpurun_out/x6shape_${T}_summary.json
