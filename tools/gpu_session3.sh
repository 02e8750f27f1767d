#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s3
mkdir -p $O
export TMPDIR=/tmp
V=$R/amdgpu_operator/_native/amdgpu-validator
ls /sys/module/amdgpu/ > $O/sysmodule.txt 2>&1; cat /sys/module/amdgpu/initstate >> $O/sysmodule.txt 2>&1
$R/amdgpu_operator/_native/amdgpu-probe --json > $O/probe.json 2> $O/probe.err; echo "probe rc=$?"
/usr/bin/time -v timeout -k 10 120 $V --rendezvous /tmp/rv1 > $O/validator_plain.json 2> $O/validator_plain.err
echo "plain rc=$?"; cat $O/validator_plain.json; grep -E "Elapsed|Maximum resident" $O/validator_plain.err
AMDGPU_VALIDATOR_COUNTERS=1 timeout -k 10 120 $V --rendezvous /tmp/rv2 --counter-gate --steps hip,gemm > $O/validator_gate.json 2> $O/validator_gate.err
echo "gate rc=$?"; cat $O/validator_gate.json; tail -5 $O/validator_gate.err
timeout -k 10 120 $V --rendezvous /tmp/rv3 --gemm 8192 --hbm-bytes 4294967296 --steps hip,gemm,hbm > $O/validator_big.json 2> $O/validator_big.err
echo "big rc=$?"; cat $O/validator_big.json
