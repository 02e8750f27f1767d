"""Kubelet pod-resources API (``v1.PodResourcesLister``) client.

``GetAllocatableResources`` is the kubelet device manager's own view: the
devices every registered plugin reported, available the moment ListAndWatch
delivers them.  ``Node.status.allocatable`` trails it - the kubelet publishes
node status on its ``nodeStatusUpdateFrequency`` tick (10 s by default), not
on a device-plugin registration - and pods bound to the node are admitted
against the device manager, not against the Node object.  The validator
therefore starts its plugin-validation pods from this view (the upstream
validator polls the Node object, which adds up to one status period to
time-to-Ready); ``Node.status.allocatable`` is what the scheduler and the
verify CLI read (/root/reference/README.md:122).
"""

from __future__ import annotations

import os

from ..rpc import wire
from . import api


class KubeletDevices:
    """Polls the kubelet's allocatable devices over one reused channel."""

    def __init__(self, socket_path: str = api.POD_RESOURCES_SOCKET):
        self.socket_path = socket_path
        self._ch = None
        self._call = None

    def available(self) -> bool:
        return os.path.exists(self.socket_path)

    def _channel(self):
        if self._call is None:
            req, resp, _ = api.POD_RESOURCES_METHODS["GetAllocatableResources"]
            self._ch = wire.Channel(self.socket_path)
            self._call = self._ch.unary_unary(
                api.method_path(api.POD_RESOURCES_SERVICE, "GetAllocatableResources"),
                request_serializer=req.SerializeToString, response_deserializer=resp.FromString)
        return self._call

    def allocatable(self, timeout: float = 2.0) -> dict[str, list[str]] | None:
        """resource name -> device IDs the kubelet can allocate, or None when
        the API is not reachable (no socket, kubelet < 1.23 without the
        ``KubeletPodResourcesGetAllocatable`` gate: UNIMPLEMENTED)."""
        if not self.available():
            return None
        try:
            call = self._channel()
            req = api.POD_RESOURCES_METHODS["GetAllocatableResources"][0]
            out = call(req(), timeout=timeout)
        except wire.RpcError:
            self.close()
            return None
        devs: dict[str, list[str]] = {}
        for d in out.devices:
            devs.setdefault(d.resource_name, []).extend(d.device_ids)
        return devs

    def count(self, resource: str, timeout: float = 2.0) -> int | None:
        devs = self.allocatable(timeout)
        return None if devs is None else len(devs.get(resource, []))

    def close(self) -> None:
        if self._ch is not None:
            self._ch.close()
        self._ch = self._call = None
