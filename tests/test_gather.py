"""must-gather archive (cli/gather.py) on a simulated cluster."""

import json
import tarfile

from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags
from amdgpu_operator.cli.gather import must_gather
from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster


def test_must_gather_archive(tmp_path):
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-1", 2), NodeSpec("cpu-1", 0)], fake_gpu=True).start()
    try:
        c.install_operator(parse_set_flags(REFERENCE_SET_FLAGS))
        c.wait_ready(60, {"gpu-1": 2})
        env = c.nodes["gpu-1"].env
        out = str(tmp_path / "mg.tar.gz")
        summary = must_gather(c.client, c.namespace, out, node_root=env.host_root, validations_dir=env.validations_dir)
        assert summary["gpu_nodes"] == 1 and summary["not_validated"] == []
        assert summary["allocatable"] == {"gpu-1": {"amd.com/gpu": "2"}}
        assert summary["policy_state"] == [["cluster-policy", "ready"]] or summary["policy_state"] == [
            ("cluster-policy", "ready")]
        with tarfile.open(out) as tar:
            names = {m.name.split("/", 1)[1] for m in tar.getmembers()}
            assert {"summary.json", "cluster/clusterpolicies.json", "cluster/pods.json", "node/node.json"} <= names
            node = json.load(tar.extractfile([m for m in tar.getmembers() if m.name.endswith("node/node.json")][0]))
        assert len(node["gpus"]) == 2 and node["probe"]["ok"]
        assert "workload-ready" in node["validations"] or any("workload" in k for k in node["validations"])
    finally:
        c.stop()
