#!/bin/bash
# GRBM_GUI_ACTIVE + MFMA-busy pass over the forward 512->512 x6 GEMM of the product and of ablated
# builds (tools/x6_ablate.py): the clock each build runs at (cycles / kernel time)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in product ${VARIANTS:-noglobal nosplit_noglobal}; do
  O=$R/gpurun_out/x6clk_$v; mkdir -p $O
  L=""; [ $v != product ] && L=$R/tools/_build/libx6_$v.so
  LIB=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/trace.log 2>&1 || exit 1
  LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/tools/gemm_x6_pmc.py > $O/p1.log 2>&1 || exit 2
  python3 $R/tools/gemm_x6_pmc.py --summary $O/p1 > $O/summary.json
  echo "== $v"; grep -E "GRBM|mfma_util" $O/summary.json; grep -h gemm_x6 $O/trace/run_kernel_stats.csv | cut -d, -f2-4
done
