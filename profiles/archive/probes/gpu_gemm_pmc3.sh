#!/bin/bash
# K2 GEMM counters of selected variants vs hipBLASLt at 8192^3, three passes
# (kernel-trace only): SQ issue/wait, SQ LDS/MFMA, TCC (L2) hits/misses and
# fabric reads.  Summarised by tools/pmc_summary.py.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-gemm_pmc3}
shift
V=${@:-15 6}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/p$P -o run --output-format csv -- \
    python3 $R/tools/gemm_prof.py --n 8192 --variants $V > $O/p$P.log 2>&1
  rc=$?; echo "pass$P rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/p$P.log; exit $rc; }
}
P=1 run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE
P=2 run TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE
P=3 run SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
python3 $R/tools/pmc_summary.py $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") > $O/summary.json
echo done
