"""The simulated node as an operand process sees it (SimCluster
``process_containers``): what a real node has as hardware, stood in.

Kept apart from :mod:`.simcluster` on purpose: every operand process of a
simulated bring-up imports this at start-up, inside the measured
time-to-Ready, and the cluster harness pulls in the operator (pydantic, the
ClusterPolicy model: ~0.3 s of imports) that no operand image carries.
"""

from __future__ import annotations

import os
import sys

from ..nodeenv import NodeEnv, run_local


def adopt_sim_node_env(env: NodeEnv) -> None:
    """In an operand process started by a ``process_containers`` SimCluster
    (``AMDGPU_SIM_NODE=1``): the fake kernel module and PCI kernel of the
    synthetic sysfs tree, the metrics fixture where amd-smi is absent,
    stand-in validator processes where there is no GPU - and ephemeral ports
    (several simulated nodes share one host)."""
    e = os.environ
    if e.get("AMDGPU_SIM_KMOD") == "1":
        from . import fakesys

        env.extra["kmod"] = fakesys.SimModule(env.host_root)
        env.extra["pci_backend"] = fakesys.FakePciKernel(env.host_root)
        if sys.argv[1:2] == ["partition-manager"]:  # partition switches act on the fake tree too
            from ..discovery import topology
            from ..partition import manager as PM

            gpus = len({g.physical_index for g in topology.enumerate_gpus(env.host_root)})
            env.extra["partition_backend"] = PM.SysfsBackend(
                env.host_root, PM.sysfs_partition_rebuilder(env.host_root, gpus), env.validations_dir)
    if e.get("AMDGPU_SIM_METRICS_FIXTURE"):
        env.extra["metrics_fixture"] = e["AMDGPU_SIM_METRICS_FIXTURE"]
    env.extra["ephemeral_ports"] = True
    if e.get("AMDGPU_SIM_FAKE_VALIDATOR") == "1":
        def launch(argv, penv, device, timeout):
            if os.path.basename(argv[0]) == "amdgpu-validator":
                argv = [sys.executable, "-m", "amdgpu_operator.testing.fake_validator", *argv[1:]]
            elif os.path.basename(argv[0]) == "amdgpu-gpu-check":
                expect = argv[argv.index("--expect-devices"):][:2] if "--expect-devices" in argv else []
                argv = [sys.executable, "-m", "amdgpu_operator.testing.fake_validator", "--steps", "hsa,vecadd",
                        "--pod-check", *expect]
            return run_local(argv, penv, timeout)

        env.launcher = launch
