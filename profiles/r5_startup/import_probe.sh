#!/bin/bash
# cost of argparse and logging on a fresh interpreter (-S), interleaved, on the box's CPU
O=gpurun_out/r5_import
mkdir -p $O
for i in $(seq 1 12); do
  for mods in "json,threading" "json,threading,argparse" "json,threading,logging" "json,threading,argparse,logging"; do
    t=$(python3 -S -c "import time; t=time.perf_counter(); import $mods; print(round(time.perf_counter()-t, 5))")
    echo "$mods $t" >> $O/imports.txt
  done
done
cd $GRAFT_REPO_ROOT && for i in 1 2 3 4 5 6; do python3 -S -X importtime -c "import amdgpu_operator.cli.main" 2>> $O/importtime_cli_main.$i.txt; done
echo done
