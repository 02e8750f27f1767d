set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r3_podexit; mkdir -p $O; cd $R; export TMPDIR=/tmp
timeout -k 10 120 python3 -u tools/pod_exit_probe.py 8 > $O/pod_exit_probe.json 2> $O/pod_exit_probe.err
rc=$?; echo "probe rc=$rc"; python3 -c "import json;d=json.load(open('$O/pod_exit_probe.json'));print({k:v['median'] for k,v in d.items()})"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 10 --warmup 2 --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $O/bench.json
exit $rc
