#!/bin/bash
# K2 GEMM counter profile of selected variants vs hipBLASLt: two PMC passes
# (kernel-trace only, no sys/runtime trace), summarised by tools/pmc_summary.py
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gemm_pmc}
shift
V=${@:-0 6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  -d $O/p1 -o run --output-format csv -- python3 $R/tools/gemm_prof.py --n 8192 --variants $V > $O/p1.log 2>&1
rc=$?; echo "pass1 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/p1.log; exit $rc; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE \
  -d $O/p2 -o run --output-format csv -- python3 $R/tools/gemm_prof.py --n 8192 --variants $V > $O/p2.log 2>&1
rc=$?; echo "pass2 rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/p2.log; exit $rc; }
python3 $R/tools/pmc_summary.py $(find $O/p1 $O/p2 -name "*counter_collection.csv") > $O/summary.json
echo done
