set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r3_exporter_ab; mkdir -p $O; cd $R
for arm in default no_metrics; do
  extra=""; [ $arm = no_metrics ] && extra="--set dcgmExporter.enabled=false"
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 10 --warmup 2 --compare 0 $extra --detail $O/${arm}_detail.json > $O/${arm}.json 2> $O/${arm}.err || exit 1
  echo "$arm $(cut -c1-160 $O/${arm}.json)"
done
