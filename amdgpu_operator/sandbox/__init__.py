"""Sandbox (VM passthrough) workloads: the MI355X counterpart of the NVIDIA
GPU Operator's ``sandboxWorkloads`` mode (vfio-manager, sandbox device plugin,
sandbox validator).  A GPU node labelled
``amd.com/gpu.workload.config=vm-passthrough`` gets its GPUs bound to
``vfio-pci`` and advertised per product (``amd.com/MI355X``) for KubeVirt-style
VMs instead of ``amd.com/gpu`` for containers."""

WORKLOAD_CONFIG_LABEL = "amd.com/gpu.workload.config"
WORKLOAD_CONTAINER = "container"
WORKLOAD_VM_PASSTHROUGH = "vm-passthrough"
WORKLOADS = (WORKLOAD_CONTAINER, WORKLOAD_VM_PASSTHROUGH)
