#!/bin/bash
# librccl load: plain dlopen without HIP, then the validator's rccl step with
# the library loaded on the main thread before HIP init.
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-s35}
mkdir -p $O /tmp/rdvC
V=$GRAFT_REPO_ROOT/amdgpu_operator/_native/amdgpu-validator
timeout -k 5 30 python3 -c "
import ctypes, time
t=time.perf_counter(); ctypes.CDLL('/opt/rocm/lib/librccl.so.1'); print('plain dlopen s', round(time.perf_counter()-t,3))" > $O/plain.log 2>&1
rc=$?; echo "plain rc=$rc"; cat $O/plain.log
[ $rc -ne 0 ] && exit $rc
timeout -k 5 40 $V --rendezvous /tmp/rdvC --steps hip,rccl --rccl-elems 1048576 > $O/c.out 2> $O/c.err
rc=$?; echo "validator rc=$rc"; tail -c 1500 $O/c.out; tail -5 $O/c.err
exit $rc
