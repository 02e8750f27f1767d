#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp

timeout -k 10 300 python3 $R/tools/kernel_bench.py > $O/kbench.json 2> $O/kbench.err
rc=$?; echo "kbench rc=$rc"; cat $O/kbench.json; tail -20 $O/kbench.err
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof1 -o kb --output-format csv -- python3 $R/tools/kernel_bench.py --quick > $O/prof1.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -5 $O/prof1.log
exit $rc
