#!/bin/bash
# Install + load the amdgpu kernel module for the running host kernel (gfx950 /
# MI355X), then wait for /dev/kfd.  Invoked by `amdgpu-operator driver install`
# (amdgpu_operator/driver/manager.py) when the N1 probe says the driver is not
# live, or the live one is not the requested one.  Reference parity: the driver
# DaemonSet "installs the NVIDIA driver on the node" (README.md:212 of the
# reference); here it is the amdgpu module + its firmware.
#
# Two flows, both with nothing fetched at pod start when the image has what the
# node needs:
#
#   precompiled (AMDGPU_USE_PRECOMPILED=true): the image was built for one
#     kernel (Dockerfile.precompiled, tag <driverVersion>-<kernel>) and holds
#     the built modules under $PRECOMPILED_ROOT/lib/modules/<kernel> plus the
#     firmware.  `modprobe -d $PRECOMPILED_ROOT` loads them; no network, no
#     compiler.  A node whose kernel the image was not built for fails with
#     the kernels it was built for.
#   dkms (default): the amdgpu-dkms package (baked in the image under
#     $DEB_DIR, or fetched) builds the module for the node's kernel against
#     its headers: the image's own, the host's /usr/src (mounted at
#     $HOST_SRC), or the distro's linux-headers package, in that order.  A
#     module already built for this kernel and version (host /lib/modules
#     survives container restarts) is loaded without a rebuild.
#
# Firmware: the MI355X firmware ships in the image (amdgpu-dkms-firmware at
# image build time).  The kernel's firmware loader resolves paths in the host's
# mount namespace, so the firmware is staged to a host directory
# ($HOST_FW_DIR, /run/amd is a hostPath at the same path) and that directory
# is written to /sys/module/firmware_class/parameters/path BEFORE modprobe.
# amdgpu keeps the images it requested for the device's lifetime (GPU reset
# reuses them), so the previous search path is restored when this script exits.
#
# Inputs (env, from the ClusterPolicy driver spec):
#   AMDGPU_DRIVER_VERSION   amdgpu release (e.g. 6.12.12)                 [required]
#   AMDGPU_USE_PRECOMPILED  true: precompiled flow (above)
#   AMDGPU_BLACKLIST_INBOX  true (default): keep the distro's inbox amdgpu from
#                           auto-loading ahead of the operator's module
#   AMDGPU_MODULE_PARAMS    extra `modprobe amdgpu` parameters
#   AMDGPU_REPO_BASE        package mirror (air-gapped clusters); default repo.radeon.com
#   AMDGPU_WAIT_SECONDS     how long to wait for /dev/kfd after modprobe (default 600)
#   AMDGPU_FORCE_RELOAD     true: replace a live module even when its version
#                           matches (the driver spec changed, e.g. module params)
# Image layout (Dockerfile / Dockerfile.precompiled):
#   AMDGPU_FIRMWARE_SRC     firmware shipped in the image (default /lib/firmware/updates)
#   AMDGPU_HOST_FIRMWARE_DIR  host directory the firmware is staged to (default /run/amd/firmware)
#   AMDGPU_PRECOMPILED_ROOT modprobe root of the precompiled modules (default /opt/amdgpu)
#   AMDGPU_DEB_DIR          amdgpu-dkms .deb baked at image build (default /opt/amdgpu/debs)
#   AMDGPU_HOST_SRC         the host's /usr/src (default /host/usr/src)
# Test hooks (tests/test_driver.py runs this script against a fake root):
#   AMDGPU_SYS_ROOT / AMDGPU_DEV_ROOT / AMDGPU_ETC_ROOT / AMDGPU_USR_SRC
#   replace /sys, /dev, /etc, /usr/src; KVER overrides `uname -r`; apt-get,
#   dpkg, dkms, modinfo, modprobe, curl, gpg come from PATH.
set -euo pipefail
SYS=${AMDGPU_SYS_ROOT:-/sys}
DEV=${AMDGPU_DEV_ROOT:-/dev}
ETC=${AMDGPU_ETC_ROOT:-/etc}
USR_SRC=${AMDGPU_USR_SRC:-/usr/src}
HOST_SRC=${AMDGPU_HOST_SRC:-/host/usr/src}
FW_SRC=${AMDGPU_FIRMWARE_SRC:-/lib/firmware/updates}
HOST_FW_DIR=${AMDGPU_HOST_FIRMWARE_DIR:-/run/amd/firmware}
PRECOMPILED_ROOT=${AMDGPU_PRECOMPILED_ROOT:-/opt/amdgpu}
DEB_DIR=${AMDGPU_DEB_DIR:-/opt/amdgpu/debs}
KVER=${KVER:-$(uname -r)}
WAIT=${AMDGPU_WAIT_SECONDS:-600}
REPO_BASE=${AMDGPU_REPO_BASE:-https://repo.radeon.com}
FW_PARAM="$SYS/module/firmware_class/parameters/path"
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

REPO_READY=false
ensure_repo() {  # the package repository, only when something must be fetched
  $REPO_READY && return 0
  log "fetching from ${REPO_BASE} (amdgpu ${AMDGPU_DRIVER_VERSION}, ${CODENAME})"
  mkdir -p "$ETC/apt/keyrings" "$ETC/apt/sources.list.d"
  curl -fsSL "${REPO_BASE}/rocm/rocm.gpg.key" | gpg --dearmor -o "$ETC/apt/keyrings/rocm.gpg"
  echo "deb [arch=amd64 signed-by=/etc/apt/keyrings/rocm.gpg] ${REPO_BASE}/amdgpu/${AMDGPU_DRIVER_VERSION}/ubuntu ${CODENAME} main" \
    > "$ETC/apt/sources.list.d/amdgpu.list"
  apt-get update
  REPO_READY=true
}

# ------------------------------------------------------------------ firmware
FW_PREV=""
FW_SET=false
restore_fw_path() {
  if $FW_SET; then
    echo "$FW_PREV" > "$FW_PARAM" 2>/dev/null || true
  fi
}
trap restore_fw_path EXIT

stage_firmware() {
  local src=$1 fetch=$2
  if ! [ -d "$src/amdgpu" ] && $fetch; then
    ensure_repo
    apt-get install -y amdgpu-dkms-firmware
  fi
  if ! [ -d "$src/amdgpu" ]; then
    log "no amdgpu firmware in $src; relying on the host's /lib/firmware"
    return 0
  fi
  # copy next to the live set, then swap: a GPU reset in another process never
  # sees a half-written directory
  mkdir -p "$HOST_FW_DIR"
  rm -rf "$HOST_FW_DIR/.amdgpu.new"
  cp -a "$src/amdgpu" "$HOST_FW_DIR/.amdgpu.new"
  rm -rf "$HOST_FW_DIR/amdgpu"
  mv "$HOST_FW_DIR/.amdgpu.new" "$HOST_FW_DIR/amdgpu"
  if [ -e "$FW_PARAM" ]; then
    FW_PREV=$(cat "$FW_PARAM" 2>/dev/null || true)
    FW_SET=true
    echo "$HOST_FW_DIR" > "$FW_PARAM"
    log "firmware search path ${HOST_FW_DIR} ($(ls "$HOST_FW_DIR/amdgpu" | wc -l) files)"
  else
    log "firmware_class has no path parameter; firmware staged to ${HOST_FW_DIR} only"
  fi
}

# ------------------------------------------------------------------- headers
ensure_headers() {
  if [ -e "$USR_SRC/linux-headers-$KVER" ]; then
    return 0  # in the image (a kernel-tagged DKMS image)
  fi
  if [ -d "$HOST_SRC/linux-headers-$KVER" ]; then
    # /lib/modules/<kver>/build (host mount) names /usr/src/linux-headers-<kver>
    # by absolute path: make every host headers tree visible there
    mkdir -p "$USR_SRC"
    for d in "$HOST_SRC"/linux-headers-*; do
      [ -e "$USR_SRC/$(basename "$d")" ] || ln -s "$d" "$USR_SRC/$(basename "$d")"
    done
    log "using the host's headers for ${KVER}"
    return 0
  fi
  ensure_repo
  if apt-get install -y "linux-headers-${KVER}" "linux-modules-extra-${KVER}"; then
    return 0
  fi
  log "no headers for ${KVER}: install linux-headers-${KVER} on the host (mounted at ${HOST_SRC}) or use usePrecompiled"
  exit 1
}

MODPROBE=(modprobe)
if [ "${AMDGPU_USE_PRECOMPILED:-false}" = "true" ]; then
  if ! [ -d "$PRECOMPILED_ROOT/lib/modules/$KVER" ]; then
    built=$(ls "$PRECOMPILED_ROOT/lib/modules" 2>/dev/null | tr '\n' ' ' || true)
    log "precompiled image has no modules for kernel ${KVER} (built for: ${built:-none}); use the image tagged ${AMDGPU_DRIVER_VERSION}-${KVER}"
    exit 1
  fi
  log "precompiled amdgpu ${AMDGPU_DRIVER_VERSION} for ${KVER}"
  stage_firmware "$PRECOMPILED_ROOT/firmware" false  # never fetched at pod start
  MODPROBE=(modprobe -d "$PRECOMPILED_ROOT")
else
  built=$(modinfo -k "$KVER" -F version amdgpu 2>/dev/null || true)
  stage_firmware "$FW_SRC" true
  if [ "$built" = "$AMDGPU_DRIVER_VERSION" ]; then
    log "amdgpu ${built} already built for ${KVER}; no rebuild"
  else
    ensure_headers
    deb=$(ls "$DEB_DIR"/amdgpu-dkms_*.deb 2>/dev/null | head -n1 || true)
    if [ -n "$deb" ]; then
      dpkg -i "$deb"
    else
      ensure_repo
      apt-get install -y amdgpu-dkms
    fi
    dkms autoinstall -k "$KVER"
  fi
fi

if live; then
  # loading the new module over a live one would leave the old one in place
  if ! modprobe -r amdgpu; then
    log "could not unload the running amdgpu (GPU in use?)"
    exit 1
  fi
fi
# shellcheck disable=SC2086
"${MODPROBE[@]}" amdgpu ${AMDGPU_MODULE_PARAMS:-}
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
