#!/bin/bash
# Install + load the amdgpu kernel module for the running host kernel and the
# ROCm userspace (gfx950 / MI355X), then wait for /dev/kfd.  Invoked by
# `amdgpu-operator driver install` (amdgpu_operator/driver/manager.py) when the
# N1 probe says the driver is not live.  Inputs (env, from the ClusterPolicy):
#   ROCM_VERSION, AMDGPU_DRIVER_VERSION, AMDGPU_USE_PRECOMPILED,
#   AMDGPU_BLACKLIST_INBOX, AMDGPU_MODULE_PARAMS
set -euo pipefail
HOST=/host
KVER=$(uname -r)
log() { echo "{\"ts\": $(date +%s), \"msg\": \"$*\"}"; }

if [ "$(cat /sys/module/amdgpu/initstate 2>/dev/null || true)" = "live" ]; then
  log "amdgpu already live ($(cat /sys/module/amdgpu/version 2>/dev/null || echo inbox)); nothing to install"
  exit 0
fi
if [ "${AMDGPU_BLACKLIST_INBOX:-true}" = "true" ]; then
  echo "blacklist amdgpu" > /etc/modprobe.d/amd-gpu-operator-blacklist.conf || true
fi
. /etc/os-release
REPO="https://repo.radeon.com/amdgpu/${AMDGPU_DRIVER_VERSION}/ubuntu"
log "installing amdgpu-dkms ${AMDGPU_DRIVER_VERSION} for kernel ${KVER} (${VERSION_CODENAME})"
mkdir -p /etc/apt/keyrings
curl -fsSL https://repo.radeon.com/rocm/rocm.gpg.key | gpg --dearmor -o /etc/apt/keyrings/rocm.gpg
echo "deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] ${REPO} ${VERSION_CODENAME} main" > /etc/apt/sources.list.d/amdgpu.list
apt-get update
apt-get install -y "linux-headers-${KVER}" "linux-modules-extra-${KVER}" || log "host headers from /host"
if [ "${AMDGPU_USE_PRECOMPILED:-false}" = "true" ]; then
  apt-get install -y "amdgpu-dkms-firmware" "amdgpu-${KVER}"
else
  apt-get install -y amdgpu-dkms
fi
modprobe -r amdgpu 2>/dev/null || true
# shellcheck disable=SC2086
modprobe amdgpu ${AMDGPU_MODULE_PARAMS:-}
for _ in $(seq 1 600); do
  [ -e /dev/kfd ] && [ "$(cat /sys/module/amdgpu/initstate 2>/dev/null)" = "live" ] && break
  sleep 1
done
[ -e /dev/kfd ] || { log "amdgpu loaded but /dev/kfd missing"; exit 1; }
log "amdgpu $(cat /sys/module/amdgpu/version) live"
