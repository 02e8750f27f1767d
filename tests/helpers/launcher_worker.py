"""torchrun worker for tests/test_launcher.py: rank 0 submits one process per
device and checks that the owner rank (device % world) ran it."""
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch.distributed as dist  # noqa: E402

from amdgpu_operator.parallel.launcher import DistributedLauncher  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo")
L = DistributedLauncher(rank, world, dist.group.WORLD)
results = {}


def driver():
    threads = []
    for dev in range(2 * world):
        def one(d=dev):
            r = L([sys.executable, "-c", "import os,json;print(json.dumps({'rank': os.environ['RANK'], 'x': os.environ['X']}))"],
                  {"X": str(d)}, d, 30)
            results[d] = json.loads(r.stdout)
        th = threading.Thread(target=one)
        th.start()
        threads.append(th)
    for th in threads:
        th.join()
    # a child that reports, closes its pipes and then takes 3 s to exit (GPU
    # teardown) is complete at its report when it asks for that
    early = {}

    def slow(d):
        r = L([sys.executable, "-c", EARLY_CHILD], {"AMDGPU_REPORT_EARLY": "1"}, d, 30)
        early[d] = (r.rc, r.seconds, json.loads(r.stdout)["ok"])

    threads = [threading.Thread(target=slow, args=(d,)) for d in range(world)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    results["early"] = early
    L.request_stop()


EARLY_CHILD = ("import json,os,sys,time;print(json.dumps({'ok': True}));sys.stdout.flush();"
               "n=os.open(os.devnull,os.O_WRONLY);os.dup2(n,1);os.dup2(n,2);time.sleep(3)")


if rank == 0:
    th = threading.Thread(target=driver)
    th.start()
    L.serve()
    th.join()
    ok = all(int(results[d]["rank"]) == d % world and results[d]["x"] == str(d) for d in range(2 * world))
    ok = ok and len(results["early"]) == world and all(rc == 0 and sec < 2.0 and rep for rc, sec, rep in
                                                       results["early"].values())
    print("LAUNCHER_OK" if ok else f"LAUNCHER_BAD {results}")
else:
    L.serve()
dist.destroy_process_group()
