#!/bin/bash
# Round 2: the driver container's SMI table on the real MI355X (what the reference reads off nvidia-smi,
# README.md:152-167), and rocprofv3 kernel stats of whole bring-ups (every validator process torn down so
# the profiler can write its records)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r2s34
mkdir -p $O
cd $R
HOST_ROOT=/ VALIDATIONS_DIR=/tmp/amd-val timeout -k 10 60 python3 -m amdgpu_operator driver smi > $O/driver_smi.txt 2> $O/driver_smi.err
rc=$?; echo "smi rc=$rc"; cat $O/driver_smi.txt
[ $rc -ne 0 ] && { tail -5 $O/driver_smi.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
AMDGPU_VALIDATOR_TEARDOWN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u $R/bench.py --steps 3 --warmup 1 --kubelet-status-s 0 > $O/prof_bench.out 2> $O/prof_bench.err
rc=$?; echo "rocprof rc=$rc"; cut -c1-200 $O/prof_bench.out
find $O/prof -name "*kernel_stats.csv" | head -20
exit $rc
