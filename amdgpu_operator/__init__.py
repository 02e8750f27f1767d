"""amd-gpu-operator: a Kubernetes GPU operator built from scratch for AMD
Instinct MI355X (gfx950 / CDNA4).

Capability parity target: the NVIDIA GPU Operator deployment of
``thanatchon36/nvidia-gpu-operator-k8s-cluster``.  Python
control plane (operator, device plugin, discovery, exporters, CLI) + native
C++/HIP components (validator kernels, OCI hook, topology/metrics/health
library, readiness probe) under ``native/``.
"""

__version__ = "0.1.0"

# Kubernetes API surface (reference name -> MI355X name)
RESOURCE_NAME = "amd.com/gpu"
LABEL_PREFIX = "amd.com/gpu"
LABEL_PRESENT = "amd.com/gpu.present"
API_GROUP = "amd.com"
API_VERSION = "v1"
DEFAULT_NAMESPACE = "gpu-operator-resources"
