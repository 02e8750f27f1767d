#!/bin/bash
# Install + load the amdgpu kernel module for the running host kernel and the
# ROCm userspace (gfx950 / MI355X), then wait for /dev/kfd.  Invoked by
# `amdgpu-operator driver install` (amdgpu_operator/driver/manager.py) when the
# N1 probe says the driver is not live, or the live one is not the requested one.  Reference parity: the driver
# DaemonSet "installs the NVIDIA driver on the node" (README.md:212 of the
# reference); here it is the amdgpu DKMS module + ROCm for gfx950.
#
# Inputs (env, from the ClusterPolicy driver spec):
#   AMDGPU_DRIVER_VERSION   amdgpu repo release (e.g. 7.2)          [required]
#   ROCM_VERSION            ROCm userspace release                  [optional]
#   AMDGPU_USE_PRECOMPILED  true: prebuilt amdgpu-<kernel> package, no DKMS build
#   AMDGPU_BLACKLIST_INBOX  true (default): keep the distro's inbox amdgpu from
#                           auto-loading ahead of the operator's module
#   AMDGPU_MODULE_PARAMS    extra `modprobe amdgpu` parameters
#   AMDGPU_REPO_BASE        package mirror (air-gapped clusters); default repo.radeon.com
#   AMDGPU_WAIT_SECONDS     how long to wait for /dev/kfd after modprobe (default 600)
#   AMDGPU_FORCE_RELOAD     true: replace a live module even when its version
#                           matches (the driver spec changed, e.g. module params)
# Test hooks (tests/test_driver.py runs this script against a fake root):
#   AMDGPU_SYS_ROOT / AMDGPU_DEV_ROOT / AMDGPU_ETC_ROOT  replace /sys, /dev, /etc
#   KVER overrides `uname -r`; apt-get, modprobe, curl, gpg come from PATH.
set -euo pipefail
SYS=${AMDGPU_SYS_ROOT:-/sys}
DEV=${AMDGPU_DEV_ROOT:-/dev}
ETC=${AMDGPU_ETC_ROOT:-/etc}
KVER=${KVER:-$(uname -r)}
WAIT=${AMDGPU_WAIT_SECONDS:-600}
REPO_BASE=${AMDGPU_REPO_BASE:-https://repo.radeon.com}
log() { echo "{\"ts\": $(date +%s), \"component\": \"amd-driver-install\", \"msg\": \"$*\"}"; }
live() { [ "$(cat "$SYS/module/amdgpu/initstate" 2>/dev/null || true)" = "live" ]; }

loaded_version() { cat "$SYS/module/amdgpu/version" 2>/dev/null || true; }

# A live module is kept only when it is the requested one.  An inbox module
# (no version file) is kept unless the manager asks for a reload, as it does
# when the driver spec changed (AMDGPU_FORCE_RELOAD=true).
if live && [ -e "$DEV/kfd" ] && [ "${AMDGPU_FORCE_RELOAD:-false}" != "true" ]; then
  LV=$(loaded_version)
  if [ -z "$LV" ] || [ -z "${AMDGPU_DRIVER_VERSION:-}" ] || [ "$LV" = "$AMDGPU_DRIVER_VERSION" ]; then
    log "amdgpu already live (${LV:-inbox}); nothing to install"
    exit 0
  fi
  log "amdgpu ${LV} live, ${AMDGPU_DRIVER_VERSION} requested: replacing it"
fi
: "${AMDGPU_DRIVER_VERSION:?AMDGPU_DRIVER_VERSION is required}"

mkdir -p "$ETC/modprobe.d"
if [ "${AMDGPU_BLACKLIST_INBOX:-true}" = "true" ]; then
  echo "blacklist amdgpu" > "$ETC/modprobe.d/amd-gpu-operator-blacklist.conf"
fi
# (a blacklist entry stops alias-based autoload at boot only; the explicit
# modprobe below still loads the operator's module)
if [ -f "$ETC/os-release" ]; then . "$ETC/os-release"; fi
CODENAME=${VERSION_CODENAME:-jammy}

log "installing amdgpu ${AMDGPU_DRIVER_VERSION} for kernel ${KVER} (${CODENAME})"
mkdir -p "$ETC/apt/keyrings" "$ETC/apt/sources.list.d"
curl -fsSL "${REPO_BASE}/rocm/rocm.gpg.key" | gpg --dearmor -o "$ETC/apt/keyrings/rocm.gpg"
echo "deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] ${REPO_BASE}/amdgpu/${AMDGPU_DRIVER_VERSION}/ubuntu ${CODENAME} main" \
  > "$ETC/apt/sources.list.d/amdgpu.list"
if [ -n "${ROCM_VERSION:-}" ]; then
  echo "deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] ${REPO_BASE}/rocm/apt/${ROCM_VERSION} ${CODENAME} main" \
    > "$ETC/apt/sources.list.d/rocm.list"
fi
apt-get update
if [ "${AMDGPU_USE_PRECOMPILED:-false}" = "true" ]; then
  apt-get install -y "amdgpu-dkms-firmware" "amdgpu-${KVER}"
else
  apt-get install -y "linux-headers-${KVER}" "linux-modules-extra-${KVER}" || log "headers for ${KVER} not packaged; using /host headers"
  apt-get install -y amdgpu-dkms
fi
if [ -n "${ROCM_VERSION:-}" ]; then
  apt-get install -y amd-smi-lib rocm-smi-lib
fi

if live; then
  # loading the new module over a live one would leave the old one in place
  if ! modprobe -r amdgpu; then
    log "could not unload the running amdgpu (GPU in use?)"
    exit 1
  fi
fi
# shellcheck disable=SC2086
modprobe amdgpu ${AMDGPU_MODULE_PARAMS:-}
for _ in $(seq 1 "$WAIT"); do
  if [ -e "$DEV/kfd" ] && live; then break; fi
  sleep 1
done
if ! [ -e "$DEV/kfd" ]; then
  log "amdgpu loaded but $DEV/kfd missing after ${WAIT}s"
  exit 1
fi
LV=$(loaded_version)
if [ -n "$LV" ] && [ "$LV" != "$AMDGPU_DRIVER_VERSION" ]; then
  log "amdgpu ${LV} loaded, ${AMDGPU_DRIVER_VERSION} requested"
  exit 1
fi
log "amdgpu ${LV:-unknown} live"
