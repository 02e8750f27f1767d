"""Kubelet device-plugin API ``v1beta1`` and pod-resources API ``v1``.

Wire-compatible hand declarations (SURVEY.md §7.1 lists the field numbers),
encoded by the operator's own codec (rpc/proto.py); the same schema built
through google.protobuf (:func:`protobuf_classes`, deviceplugin/protodef.py)
is the reference the codec is tested against.
The reference relies on the NVIDIA device plugin speaking this API to turn
GPUs into the ``nvidia.com/gpu`` extended resource
(/root/reference/README.md:122,205,211,220); this operator speaks the same API
for ``amd.com/gpu``.
"""

from __future__ import annotations

from ..rpc.proto import build_file

VERSION = "v1beta1"
DEVICE_PLUGIN_PATH = "/var/lib/kubelet/device-plugins/"
KUBELET_SOCKET = DEVICE_PLUGIN_PATH + "kubelet.sock"
POD_RESOURCES_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
REPLICA_SEP = "::"  # time-sliced replica IDs: "<device id>::<replica>" (config.py)
HEALTHY = "Healthy"
UNHEALTHY = "Unhealthy"

_MESSAGES = {
    "Empty": [],
    "DevicePluginOptions": [("pre_start_required", 1, "bool", "opt"),
                            ("get_preferred_allocation_available", 2, "bool", "opt")],
    "RegisterRequest": [("version", 1, "string", "opt"), ("endpoint", 2, "string", "opt"),
                        ("resource_name", 3, "string", "opt"), ("options", 4, "DevicePluginOptions", "opt")],
    "ListAndWatchResponse": [("devices", 1, "Device", "rep")],
    "TopologyInfo": [("nodes", 1, "NUMANode", "rep")],
    "NUMANode": [("ID", 1, "int64", "opt")],
    "Device": [("ID", 1, "string", "opt"), ("health", 2, "string", "opt"), ("topology", 3, "TopologyInfo", "opt")],
    "PreStartContainerRequest": [("devices_ids", 1, "string", "rep")],
    "PreStartContainerResponse": [],
    "PreferredAllocationRequest": [("container_requests", 1, "ContainerPreferredAllocationRequest", "rep")],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, "string", "rep"),
                                            ("must_include_deviceIDs", 2, "string", "rep"),
                                            ("allocation_size", 3, "int32", "opt")],
    "PreferredAllocationResponse": [("container_responses", 1, "ContainerPreferredAllocationResponse", "rep")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, "string", "rep")],
    "AllocateRequest": [("container_requests", 1, "ContainerAllocateRequest", "rep")],
    "ContainerAllocateRequest": [("devices_ids", 1, "string", "rep")],
    "CDIDevice": [("name", 1, "string", "opt")],
    "AllocateResponse": [("container_responses", 1, "ContainerAllocateResponse", "rep")],
    "ContainerAllocateResponse": [("envs", 1, "map<string,string>", "rep"), ("mounts", 2, "Mount", "rep"),
                                  ("devices", 3, "DeviceSpec", "rep"), ("annotations", 4, "map<string,string>", "rep"),
                                  ("cdi_devices", 5, "CDIDevice", "rep")],
    "Mount": [("container_path", 1, "string", "opt"), ("host_path", 2, "string", "opt"), ("read_only", 3, "bool", "opt")],
    "DeviceSpec": [("container_path", 1, "string", "opt"), ("host_path", 2, "string", "opt"),
                   ("permissions", 3, "string", "opt")],
}

_SERVICES = {
    "Registration": [("Register", "RegisterRequest", "Empty", False)],
    "DevicePlugin": [
        ("GetDevicePluginOptions", "Empty", "DevicePluginOptions", False),
        ("ListAndWatch", "Empty", "ListAndWatchResponse", True),
        ("GetPreferredAllocation", "PreferredAllocationRequest", "PreferredAllocationResponse", False),
        ("Allocate", "AllocateRequest", "AllocateResponse", False),
        ("PreStartContainer", "PreStartContainerRequest", "PreStartContainerResponse", False),
    ],
}

pb = build_file("v1beta1", _MESSAGES)

REGISTRATION_SERVICE = "v1beta1.Registration"
DEVICE_PLUGIN_SERVICE = "v1beta1.DevicePlugin"

# method -> (request class, response class, server streaming)
DEVICE_PLUGIN_METHODS = {name: (pb[i], pb[o], s) for name, i, o, s in _SERVICES["DevicePlugin"]}
REGISTRATION_METHODS = {name: (pb[i], pb[o], s) for name, i, o, s in _SERVICES["Registration"]}

# ---------------------------------------------------------------- pod resources v1
_PR_MESSAGES = {
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, "PodResources", "rep")],
    "PodResources": [("name", 1, "string", "opt"), ("namespace", 2, "string", "opt"),
                     ("containers", 3, "ContainerResources", "rep")],
    "ContainerResources": [("name", 1, "string", "opt"), ("devices", 2, "ContainerDevices", "rep"),
                           ("cpu_ids", 3, "int64", "rep"), ("memory", 4, "ContainerMemory", "rep"),
                           ("dynamic_resources", 5, "DynamicResource", "rep")],
    "ContainerMemory": [("memory_type", 1, "string", "opt"), ("size", 2, "uint64", "opt"),
                        ("topology", 3, "TopologyInfo", "opt")],
    # DRA claims prepared for the container (kubelet >= 1.27 behind the
    # KubeletPodResourcesDynamicResources gate; driver/pool/device since 1.31)
    "DynamicResource": [("class_name", 1, "string", "opt"), ("claim_name", 2, "string", "opt"),
                        ("claim_namespace", 3, "string", "opt"), ("claim_resources", 4, "ClaimResource", "rep")],
    "ClaimResource": [("cdi_devices", 1, "CDIDevice", "rep"), ("driver_name", 2, "string", "opt"),
                      ("pool_name", 3, "string", "opt"), ("device_name", 4, "string", "opt")],
    "CDIDevice": [("name", 1, "string", "opt")],
    "ContainerDevices": [("resource_name", 1, "string", "opt"), ("device_ids", 2, "string", "rep"),
                         ("topology", 3, "TopologyInfo", "opt")],
    "TopologyInfo": [("nodes", 1, "NUMANode", "rep")],
    "NUMANode": [("ID", 1, "int64", "opt")],
    "AllocatableResourcesRequest": [],
    "AllocatableResourcesResponse": [("devices", 1, "ContainerDevices", "rep"), ("cpu_ids", 2, "int64", "rep")],
}
_PR_SERVICES = {
    "PodResourcesLister": [("List", "ListPodResourcesRequest", "ListPodResourcesResponse", False),
                           ("GetAllocatableResources", "AllocatableResourcesRequest", "AllocatableResourcesResponse", False)],
}
podres = build_file("v1", _PR_MESSAGES)
POD_RESOURCES_SERVICE = "v1.PodResourcesLister"
POD_RESOURCES_METHODS = {name: (podres[i], podres[o], s) for name, i, o, s in _PR_SERVICES["PodResourcesLister"]}


def method_path(service: str, method: str) -> str:
    return f"/{service}/{method}"


def protobuf_classes() -> tuple[dict, dict]:
    """The same messages as google.protobuf classes (tests: the codec's reference)."""
    from .protodef import build_file as pb_build

    dp, _ = pb_build("v1beta1", "deviceplugin/v1beta1/api.proto", _MESSAGES, _SERVICES)
    pr, _ = pb_build("v1", "podresources/v1/api.proto", _PR_MESSAGES, _PR_SERVICES)
    return dp, pr
