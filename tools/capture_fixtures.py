"""Capture real MI355X device fixtures (run on the GPU box via gpurun).

Writes, under the output directory:
  rocminfo.txt, amd-smi-{static,metric,topology,list,partition}.json,
  rocprofv3-counters.txt, sysfs/ (KFD topology, DRM, PCI, module copies of
  small readable files), devnodes.txt
These back the fake-sysfs/fake-amd-smi fixtures in tests/fixtures.
"""

import json
import os
import shutil
import stat
import subprocess
import sys


def run(cmd, out, timeout=60):
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        with open(out, "w") as f:
            f.write(r.stdout)
            if r.returncode:
                f.write(f"\n# rc={r.returncode}\n{r.stderr[-4000:]}")
    except Exception as e:  # noqa: BLE001
        with open(out, "w") as f:
            f.write(f"# failed: {e}\n")


def copy_tree(src, dst, max_files=20000, max_bytes=65536, skip=()):
    n = 0
    for root, dirs, files in os.walk(src, followlinks=False):
        dirs[:] = [d for d in dirs if d not in skip and not d.startswith("power")]
        for fn in files:
            if n >= max_files:
                return
            p = os.path.join(root, fn)
            try:
                st = os.lstat(p)
                if not stat.S_ISREG(st.st_mode) or not (st.st_mode & stat.S_IRUSR):
                    continue
                with open(p, "rb") as f:
                    data = f.read(max_bytes)
            except Exception:  # noqa: BLE001
                continue
            rel = os.path.relpath(p, "/")
            q = os.path.join(dst, rel)
            os.makedirs(os.path.dirname(q), exist_ok=True)
            with open(q, "wb") as f:
                f.write(data)
            n += 1


def copy_links(src, dst):
    """Record symlink targets of a directory (e.g. /sys/class/drm/*)."""
    out = {}
    if os.path.isdir(src):
        for fn in sorted(os.listdir(src)):
            p = os.path.join(src, fn)
            out[fn] = os.readlink(p) if os.path.islink(p) else None
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)


def main(out):
    os.makedirs(out, exist_ok=True)
    run(["rocminfo"], f"{out}/rocminfo.txt")
    for sub in ("static", "metric", "topology", "list", "partition", "firmware", "bad-pages", "process", "xgmi"):
        run(["amd-smi", sub, "--json"], f"{out}/amd-smi-{sub}.json")
    run(["amd-smi", "version"], f"{out}/amd-smi-version.txt")
    run(["rocm-smi", "--showallinfo", "--json"], f"{out}/rocm-smi-all.json")
    run(["rocprofv3", "-L"], f"{out}/rocprofv3-counters.txt", timeout=120)
    run(["bash", "-c", "ls -l /dev/kfd /dev/dri /dev/dri/by-path; id; uname -a; cat /proc/cpuinfo | grep 'model name' | head -1; nproc; free -g"],
        f"{out}/devnodes.txt")
    sysd = f"{out}/sysfs"
    copy_tree("/sys/class/kfd/kfd/topology", sysd, skip=("caches",))
    copy_links("/sys/class/drm", f"{out}/drm-links.json")
    for card in sorted(os.listdir("/sys/class/drm")) if os.path.isdir("/sys/class/drm") else []:
        base = f"/sys/class/drm/{card}"
        for fn in ("dev", "uevent"):
            copy_tree_file(f"{base}/{fn}", sysd)
        dev = f"{base}/device"
        if os.path.isdir(dev):
            for fn in ("vendor", "device", "subsystem_vendor", "subsystem_device", "class", "numa_node", "unique_id",
                       "current_link_speed", "current_link_width", "mem_info_vram_total", "mem_info_vram_used",
                       "product_name", "product_number", "serial_number", "vbios_version", "uevent",
                       "current_compute_partition", "available_compute_partition", "current_memory_partition",
                       "available_memory_partition", "xgmi_hive_id", "xgmi_device_id", "ras/features"):
                copy_tree_file(f"{dev}/{fn}", sysd, rel_as=f"sys/class/drm/{card}/device/{fn}")
    copy_tree("/sys/module/amdgpu/version", sysd) if os.path.isfile("/sys/module/amdgpu/version") else None
    for fn in ("/sys/module/amdgpu/version", "/sys/module/amdgpu/srcversion", "/proc/version"):
        copy_tree_file(fn, sysd)
    pci = "/sys/bus/pci/devices"
    if os.path.isdir(pci):
        for d in sorted(os.listdir(pci)):
            try:
                vendor = open(f"{pci}/{d}/vendor").read().strip()
            except Exception:  # noqa: BLE001
                continue
            if vendor != "0x1002":
                continue
            for fn in ("vendor", "device", "class", "numa_node", "subsystem_vendor", "subsystem_device", "revision"):
                copy_tree_file(f"{pci}/{d}/{fn}", sysd, rel_as=f"sys/bus/pci/devices/{d}/{fn}")
    # one archive instead of thousands of files (gpurun merges <= 2000 files)
    shutil.make_archive(f"{out}/sysfs", "gztar", root_dir=sysd)
    shutil.rmtree(sysd)
    print("fixtures written to", out)


def copy_tree_file(p, sysd, rel_as=None):
    try:
        with open(p, "rb") as f:
            data = f.read(65536)
    except Exception:  # noqa: BLE001
        return
    q = os.path.join(sysd, rel_as or os.path.relpath(p, "/"))
    os.makedirs(os.path.dirname(q), exist_ok=True)
    with open(q, "wb") as f:
        f.write(data)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fixtures")
