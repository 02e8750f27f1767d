"""``AMDGPUDriver`` (``amd.com/v1``, cluster-scoped): per-node-pool driver.

Reference parity: the reference deploys one driver DaemonSet for the whole
cluster (/root/reference/README.md:104,132-143).  Clusters that mix node pools
(different kernels, a canary pool on a newer amdgpu/ROCm) need one driver
configuration per pool, which upstream solves with a driver CRD next to the
ClusterPolicy.  With ``driver.useDriverCRD: true`` the operator creates one
``amd-driver-daemonset-<name>`` per AMDGPUDriver, restricted to the GPU nodes
its ``nodeSelector`` matches and owned by the object (deleting it removes its
DaemonSet).  A GPU node matched by two AMDGPUDriver objects is a conflict:
both report it in their status and neither is deployed there.
"""

from __future__ import annotations

from pydantic import Field

from .clusterpolicy import DriverSpec

KIND = "AMDGPUDriver"
PLURAL = "amdgpudrivers"


class AMDGPUDriverSpec(DriverSpec):
    """DriverSpec plus the nodes it applies to (empty selector = every GPU node)."""

    nodeSelector: dict[str, str] = Field(default_factory=dict)


def amdgpu_driver(name: str, spec: AMDGPUDriverSpec | dict | None = None) -> dict:
    from .. import API_GROUP, API_VERSION

    if isinstance(spec, dict) or spec is None:
        spec = AMDGPUDriverSpec.model_validate(spec or {})
    return {"apiVersion": f"{API_GROUP}/{API_VERSION}", "kind": KIND, "metadata": {"name": name},
            "spec": spec.model_dump(mode="json")}
