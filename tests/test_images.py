"""Slim per-role operand images (tools/image_manifest.py): each image's
Dockerfile copies exactly the ROCm libraries, native artefacts, distro and
Python packages its sub-commands need - derived from ``ldd`` of the built
artefacts (plus the libraries they dlopen) and from importing the role's
modules - and no runtime image inherits the multi-GB ROCm development image."""

import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import image_manifest as IM  # noqa: E402


def test_every_image_copies_what_its_artefacts_need():
    assert IM.check() == []


@pytest.mark.parametrize("role", sorted(IM.ROLES))
def test_generated_dockerfile_is_current(role):
    with open(os.path.join(IM.IMAGES, role, "Dockerfile")) as f:
        assert f.read() == IM.dockerfile(role, IM.requirements(role)), "run: python tools/image_manifest.py generate"


@pytest.mark.parametrize("role", [*sorted(IM.ROLES), "amd-driver"])
def test_runtime_stage_is_not_the_rocm_dev_image(role):
    with open(os.path.join(IM.IMAGES, role, "Dockerfile")) as f:
        text = f.read()
    final = re.findall(r"^FROM (\S+)", text, re.M)[-1]
    assert "rocm/dev" not in final and final in ("ubuntu:22.04", "${BASE}")


def test_roles_need_what_they_run():
    val = IM.requirements("amd-operator-validator")
    # HIP runtime + HSA + the AQL profiler it dlopens + the trimmed RCCL's own deps
    assert {"libamdhip64.so.7", "libhsa-runtime64.so.1", "libhsa-amd-aqlprofile64.so.1",
            "librocm_smi64.so.1"} <= set(val["rocm_libs"])
    assert "librocprofiler-sdk.so.1" not in val["rocm_libs"]  # the SDK counter gate is not shipped
    assert "libamd_comgr.so.3" in val["rocm_libs"]  # HIP dlopens it at init (the MI355X trace below)
    assert {"libdrm-amdgpu1", "libnuma1", "libelf1"} <= set(val["apt"])
    assert IM.requirements("amd-gpu-operator")["rocm_libs"] == []
    assert {"pydantic", "pyyaml"} <= set(IM.requirements("amd-gpu-operator")["python"])
    # the kubelet gRPC runs on the operator's own HTTP/2 stack (rpc/): no grpcio / protobuf in any operand image
    for role in ("amd-device-plugin", "amd-operator-validator", "amd-metrics-exporter", "amd-sandbox-device-plugin"):
        assert not {"grpcio", "protobuf"} & set(IM.requirements(role)["python"]), role
    assert IM.requirements("amd-device-plugin")["rocm_libs"] == ["libamd_smi.so"]
    assert IM.requirements("amd-container-toolkit")["rocm_libs"] == []


def test_dockerfile_parser_sees_a_missing_library():
    with open(os.path.join(IM.IMAGES, "amd-operator-validator", "Dockerfile")) as f:
        text = f.read()
    broken = text.replace("COPY --from=build /opt/rocm/lib/libhsa-runtime64.so.1 /opt/rocm/lib/\n", "")
    assert "libhsa-runtime64.so.1" not in IM.parse_dockerfile(broken)["rocm_libs"]
    assert "libhsa-runtime64.so.1" in IM.parse_dockerfile(text)["rocm_libs"]


# the interpreter's own extension libraries (python3 package) and the GPU
# pool's preloaded guard library are not part of a role's closure
PYTHON_RUNTIME = {"libffi.so.8", "libexpat.so.1", "libbz2.so.1.0", "liblzma.so.5", "libz.so.1"}


@pytest.mark.parametrize("run,role", [("validator", "amd-operator-validator"), ("smi", "amd-device-plugin")])
def test_every_library_loaded_on_the_mi355x_is_in_the_image(run, role):
    """profiles/r3_images/loaded_libs_mi355x.json: `image_manifest.py trace`
    on the box (LD_DEBUG=files) - the validator's full step list with the
    counter gate, and the amd-smi reader.  Each library those processes
    loaded, dlopen'ed ones included, must be in the role's image."""
    import json

    with open(os.path.join(ROOT, "profiles/r3_images/loaded_libs_mi355x.json")) as f:
        trace = json.load(f)[run]
    assert trace["rc"] == 0
    req = IM.requirements(role)
    have = set(req["rocm_libs"]) | set(req["system_libs"]) | {os.path.basename(a) for a in req["native"]}
    loaded = {os.path.basename(p) for p in trace["loaded"]}
    loaded = {n for n in loaded if ".cpython-" not in n and "graft" not in n} - PYTHON_RUNTIME
    assert loaded - have == set()
