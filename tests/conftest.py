"""Shared pytest configuration.

``gpu``-marked tests need a real MI355X (run on the GPU box with
``pytest -m gpu``); everything else runs on the CPU-only build container.
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


# threads of a gRPC server (rpc/wire.py ``<name>-accept``) or of a device
# plugin's kubelet watch that a test started must be gone when it ends: a
# leaked plugin re-registers with whatever kubelet socket appears later (and
# logs into a closed stream), and under -n N it can reach another test's
# kubelet through a shared temp dir
_SERVER_THREADS = ("amdgpu-dp-watch", "amdgpu-dp-health", "amdgpu-health-hub")


def _server_threads():
    import threading

    return {t for t in threading.enumerate()
            if t.is_alive() and (t.name in _SERVER_THREADS or t.name.endswith("-accept"))}


@pytest.fixture(autouse=True)
def no_leaked_servers(request):
    import time

    before = _server_threads()
    yield
    deadline = time.monotonic() + 10.0  # a loaded CI box (pytest -n 8) can take seconds to end a watch thread
    left = _server_threads() - before
    while left and time.monotonic() < deadline:
        time.sleep(0.02)
        left = {t for t in left if t.is_alive()}
    if left:
        pytest.fail(f"{request.node.nodeid} left server threads running: {sorted(t.name for t in left)}",
                    pytrace=False)
