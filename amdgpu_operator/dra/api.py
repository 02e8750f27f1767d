"""Kubelet DRA plugin API ``v1beta1`` and plugin-registration API ``v1``.

Dynamic Resource Allocation with structured parameters (Kubernetes >= 1.32,
``resource.k8s.io/v1beta1``) is the successor of the device-plugin API the
reference's operator advertises GPUs through (/root/reference/README.md:122,
205,211); upstream ships it as a separate GPU DRA driver next to the device
plugin.  A DRA driver talks to the kubelet over two unix sockets:

* ``pluginregistration.Registration`` (``GetInfo``,
  ``NotifyRegistrationStatus``) on a socket in
  ``/var/lib/kubelet/plugins_registry``, which the kubelet's plugin watcher
  finds and dials;
* ``k8s.io.kubelet.pkg.apis.dra.v1beta1.DRAPlugin`` (``NodePrepareResources``,
  ``NodeUnprepareResources``) on the endpoint ``GetInfo`` names.

Field numbers from the upstream ``api.proto`` files [EXT, recollection; no
copy is available in this environment - parity unpinned against a real
kubelet].  Proto3 ``map<string, Message>`` fields are declared as repeated
``*Entry`` messages (key = 1, value = 2), which is their wire form.
"""

from __future__ import annotations

from ..rpc.proto import build_file

DRIVER_NAME = "gpu.amd.com"
DRA_VERSION = "v1beta1.DRAPlugin"
PLUGIN_TYPE = "DRAPlugin"
REGISTRY_DIR = "/var/lib/kubelet/plugins_registry"
PLUGINS_DIR = "/var/lib/kubelet/plugins"

_DRA_MESSAGES = {
    "Claim": [("namespace", 1, "string", "opt"), ("uid", 2, "string", "opt"), ("name", 3, "string", "opt")],
    "NodePrepareResourcesRequest": [("claims", 1, "Claim", "rep")],
    "NodePrepareResourcesResponse": [("claims", 1, "PrepareClaimsEntry", "rep")],
    "PrepareClaimsEntry": [("key", 1, "string", "opt"), ("value", 2, "NodePrepareResourceResponse", "opt")],
    "NodePrepareResourceResponse": [("devices", 1, "Device", "rep"), ("error", 2, "string", "opt")],
    "Device": [("request_names", 1, "string", "rep"), ("pool_name", 2, "string", "opt"),
               ("device_name", 3, "string", "opt"), ("cdi_device_ids", 4, "string", "rep")],
    "NodeUnprepareResourcesRequest": [("claims", 1, "Claim", "rep")],
    "NodeUnprepareResourcesResponse": [("claims", 1, "UnprepareClaimsEntry", "rep")],
    "UnprepareClaimsEntry": [("key", 1, "string", "opt"), ("value", 2, "NodeUnprepareResourceResponse", "opt")],
    "NodeUnprepareResourceResponse": [("error", 1, "string", "opt")],
}
_DRA_SERVICES = {
    "DRAPlugin": [("NodePrepareResources", "NodePrepareResourcesRequest", "NodePrepareResourcesResponse", False),
                  ("NodeUnprepareResources", "NodeUnprepareResourcesRequest", "NodeUnprepareResourcesResponse", False)],
}
dra = build_file("k8s.io.kubelet.pkg.apis.dra.v1beta1", _DRA_MESSAGES)
DRA_SERVICE = "k8s.io.kubelet.pkg.apis.dra.v1beta1.DRAPlugin"
DRA_METHODS = {name: (dra[i], dra[o], s) for name, i, o, s in _DRA_SERVICES["DRAPlugin"]}
# Kubernetes 1.31's kubelet speaks the same messages as service v1alpha4.Node;
# the driver serves both and advertises both versions (the kubelet picks)
DRA_SERVICE_V1ALPHA4 = "k8s.io.kubelet.pkg.apis.dra.v1alpha4.Node"
DRA_VERSIONS = [DRA_VERSION, "v1alpha4.Node"]

_REG_MESSAGES = {
    "InfoRequest": [],
    "PluginInfo": [("type", 1, "string", "opt"), ("name", 2, "string", "opt"), ("endpoint", 3, "string", "opt"),
                   ("supported_versions", 4, "string", "rep")],
    "RegistrationStatus": [("plugin_registered", 1, "bool", "opt"), ("error", 2, "string", "opt")],
    "RegistrationStatusResponse": [],
}
_REG_SERVICES = {
    "Registration": [("GetInfo", "InfoRequest", "PluginInfo", False),
                     ("NotifyRegistrationStatus", "RegistrationStatus", "RegistrationStatusResponse", False)],
}
reg = build_file("pluginregistration", _REG_MESSAGES)
REGISTRATION_SERVICE = "pluginregistration.Registration"
REGISTRATION_METHODS = {name: (reg[i], reg[o], s) for name, i, o, s in _REG_SERVICES["Registration"]}


def method_path(service: str, method: str) -> str:
    return f"/{service}/{method}"


def _as_proto_maps(messages: dict) -> dict:
    """The schema as upstream's .proto writes it: ``*Entry`` fields back to
    ``map<string, V>`` (same wire bytes)."""
    entries = {n: dict((f[0], f[2]) for f in fs) for n, fs in messages.items() if n.endswith("Entry")}
    return {n: [(f[0], f[1], f"map<string,{entries[f[2]]['value']}>" if f[2] in entries else f[2], f[3]) for f in fs]
            for n, fs in messages.items() if n not in entries}


def protobuf_classes() -> tuple[dict, dict]:
    """The same messages as google.protobuf classes (tests: the codec's reference)."""
    from ..deviceplugin.protodef import build_file as pb_build

    d, _ = pb_build("k8s.io.kubelet.pkg.apis.dra.v1beta1", "dra/v1beta1/api.proto", _as_proto_maps(_DRA_MESSAGES),
                    _DRA_SERVICES)
    r, _ = pb_build("pluginregistration", "pluginregistration/v1/api.proto", _REG_MESSAGES, _REG_SERVICES)
    return d, r
