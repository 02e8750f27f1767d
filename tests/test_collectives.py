"""RCCL sweep logic (amdgpu_operator/parallel/collectives.py) on CPU gloo ranks,
world 1 and 2; the GPU run of the same code is in test_native_gpu.py."""

import json
import os
import socket
import subprocess
import sys

import pytest

from amdgpu_operator.parallel import collectives as C

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_default_sizes():
    assert C.default_sizes(8, 1 << 10, 4) == [8, 32, 128, 512, 1024]
    assert C.default_sizes(8, 8) == [8]
    assert C.default_sizes()[-1] == 1 << 30


def test_elem_count_divisible():
    for world in (1, 2, 3, 8):
        for b in (1, 8, 100, 4096):
            n = C._elem_count(b, 4, world)
            assert n >= world and n % world == 0


@pytest.mark.parametrize("world", [1, 2])
def test_sweep_cli_gloo(world):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["PYTHONPATH"] = REPO
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", "-m", "amdgpu_operator", "collectives",
           "--backend", "gloo", "--min-bytes", "8", "--max-bytes", "65536", "--factor", "16", "--iters", "2",
           "--json"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    rows = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("[")][-1])
    assert {r["op"] for r in rows} == {"allreduce", "allgather", "reducescatter"}
    assert all(r["ok"] and r["world"] == world for r in rows)
    assert len(rows) == 3 * len(C.default_sizes(8, 65536, 16))
    if world == 1:
        assert all(r["busbw_gbps"] == 0 for r in rows)
    else:
        assert all(r["busbw_gbps"] > 0 for r in rows)
