#!/bin/bash
# HIP start-up breakdown of a fresh process under a few runtime settings (5 runs each)
P=/root/repo/tools/native/hip_init_probe
UUID=$(rocminfo 2>/dev/null | grep -m1 -o "GPU-[0-9a-f]\{16\}")
for v in "" "ROCR_VISIBLE_DEVICES=$UUID" "HIP_ENABLE_DEFERRED_LOADING=0" "HIP_ENABLE_DEFERRED_LOADING=1" "HSA_ENABLE_INTERRUPT=0" "AMD_DIRECT_DISPATCH=0"; do
  for i in 1 2 3 4 5; do
    echo "[$v] $(env $v timeout -k 5 30 $P)"
  done
done
