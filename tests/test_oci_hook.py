"""N2 OCI hook / CDI generator on synthetic bundles (SURVEY.md §4.2 native tier)."""

import json
import os
import stat
import subprocess

import pytest

from amdgpu_operator import native
from amdgpu_operator.testing import fakesys

HOOK = str(native.binary("amdgpu-oci-hook"))


@pytest.fixture
def root(tmp_path):
    r = str(tmp_path / "host")
    fakesys.build_node(r, 4)
    return r


def bundle(tmp_path, env=None, annotations=None, extra=None):
    b = tmp_path / "bundle"
    b.mkdir(exist_ok=True)
    spec = {"ociVersion": "1.1.0", "process": {"args": ["sh"], "env": env or ["PATH=/usr/bin"]},
            "root": {"path": "rootfs"}, "linux": {"resources": {"devices": [{"allow": False, "access": "rwm"}]}}}
    if annotations:
        spec["annotations"] = annotations
    if extra:
        spec.update(extra)
    (b / "config.json").write_text(json.dumps(spec))
    return str(b)


def run(args, input_=None):
    return subprocess.run([HOOK, *args], capture_output=True, text=True, input=input_, timeout=30)


def spec_of(b):
    with open(os.path.join(b, "config.json")) as f:
        return json.load(f)


def test_version():
    assert run(["--version"]).stdout.startswith("amdgpu-oci-hook")


def test_cdi_spec(root):
    p = run(["cdi", "--root", root])
    assert p.returncode == 0, p.stderr
    spec = json.loads(p.stdout)
    assert spec["cdiVersion"] == "0.6.0" and spec["kind"] == "amd.com/gpu"
    names = [d["name"] for d in spec["devices"]]
    assert names == ["0", "1", "2", "3", "all"]
    dev0 = spec["devices"][0]["containerEdits"]["deviceNodes"][0]
    assert dev0 == {"path": "/dev/dri/renderD128", "type": "c", "major": 226, "minor": 128, "permissions": "rw"}
    kfd = spec["containerEdits"]["deviceNodes"][0]
    assert kfd["path"] == "/dev/kfd" and kfd["major"] == 241
    assert len(spec["devices"][-1]["containerEdits"]["deviceNodes"]) == 4


def test_cdi_to_file_with_rocm_mount(root, tmp_path):
    out = str(tmp_path / "cdi" / "amd.json")
    os.makedirs(os.path.dirname(out))
    p = run(["cdi", "--root", root, "--output", out, "--mount-rocm", "--rocm-dir", "/opt/rocm"])
    assert p.returncode == 0, p.stderr
    spec = json.load(open(out))
    assert spec["containerEdits"]["mounts"][0]["hostPath"] == "/opt/rocm"


def test_apply_from_env_is_idempotent(root, tmp_path):
    b = bundle(tmp_path, env=["PATH=/usr/bin", "AMD_VISIBLE_DEVICES=1,3"])
    for _ in range(2):
        p = run(["apply", "--bundle", b, "--root", root])
        assert p.returncode == 0, p.stderr
    s = spec_of(b)
    paths = [d["path"] for d in s["linux"]["devices"]]
    assert paths == ["/dev/kfd", "/dev/dri/renderD136", "/dev/dri/renderD152"]
    rules = [r for r in s["linux"]["resources"]["devices"] if r["allow"]]
    assert {(r["major"], r["minor"]) for r in rules} == {(241, 0), (226, 136), (226, 152)}
    assert s["annotations"]["amd.com/gpu.injected"] == "1,3"
    assert s["linux"]["resources"]["devices"][0] == {"allow": False, "access": "rwm"}  # existing deny-all kept


def _proc_tree(tmp_path, pid, cgroup_text):
    """Fake /proc/<pid>/{root,cgroup} for the prestart stage."""
    proc = tmp_path / "proc"
    (proc / str(pid) / "root").mkdir(parents=True)
    (proc / str(pid) / "cgroup").write_text(cgroup_text)
    return str(proc)


def test_precreate_edits_the_spec_on_stdin(root, tmp_path):
    spec = {"ociVersion": "1.1.0", "process": {"args": ["sh"], "env": ["AMD_VISIBLE_DEVICES=1,3"]},
            "root": {"path": "rootfs"}, "linux": {}}
    p = run(["precreate", "--root", root], json.dumps(spec))
    assert p.returncode == 0, p.stderr
    out = json.loads(p.stdout)
    assert [d["path"] for d in out["linux"]["devices"]] == ["/dev/kfd", "/dev/dri/renderD136", "/dev/dri/renderD152"]
    assert "AMD_VISIBLE_DEVICES=1,3" in out["process"]["env"]
    # a non-GPU container comes back unchanged (the runtime uses whatever is on stdout)
    plain = {"ociVersion": "1.1.0", "process": {"args": ["sh"], "env": ["PATH=/bin"]}, "linux": {}}
    p = run(["precreate", "--root", root], json.dumps(plain))
    assert p.returncode == 0 and json.loads(p.stdout) == plain
    assert run(["precreate", "--root", root], "not json").returncode == 1


def test_prestart_creates_nodes_in_the_container_and_allows_them(root, tmp_path):
    """prestart runs after the runtime loaded config.json: it acts on the live
    container (device nodes under /proc/<pid>/root, cgroup-v1 devices.allow)
    and leaves config.json alone."""
    b = bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=2"])
    before = open(os.path.join(b, "config.json")).read()
    proc = _proc_tree(tmp_path, 4242, "12:devices:/kubepods/pod1/c1\n11:memory:/kubepods/pod1/c1\n")
    cg = tmp_path / "cgroup"
    (cg / "devices/kubepods/pod1/c1").mkdir(parents=True)
    state = json.dumps({"ociVersion": "1.1.0", "id": "c1", "status": "created", "pid": 4242, "bundle": b})
    args = ["prestart", "--root", root, "--proc-root", proc, "--cgroup-root", str(cg)]
    p = run([*args, "--dry-run"], state)
    assert p.returncode == 0, p.stderr
    plan = json.loads(p.stdout)
    assert [m["path"] for m in plan["mknod"]] == [f"{proc}/4242/root/dev/kfd", f"{proc}/4242/root/dev/dri/renderD144"]
    assert plan["rules"] == ["c 241:0 rwm", "c 226:144 rwm"] and plan["injected"] == "2"
    assert plan["devices.allow"] == f"{cg}/devices/kubepods/pod1/c1/devices.allow"
    p = run(args, state)
    allow = (cg / "devices/kubepods/pod1/c1/devices.allow").read_text()
    assert allow == "c 241:0 rwmc 226:144 rwm"  # two writes (cgroupfs takes one rule per write)
    node = tmp_path / "proc/4242/root/dev/dri/renderD144"
    if p.returncode == 0:  # this process may create device nodes
        assert stat.S_ISCHR(os.stat(node).st_mode) and os.major(os.stat(node).st_rdev) == 226
    else:  # no CAP_MKNOD here: the failure names the node
        assert "mknod" in p.stderr and "renderD" in p.stderr or "kfd" in p.stderr
    assert open(os.path.join(b, "config.json")).read() == before


@pytest.mark.parametrize("attack", ["dri-dir", "node", "dev-dir"])
def test_prestart_does_not_follow_container_symlinks(root, tmp_path, attack):
    """The hook runs as host root: a container-controlled symlink at /dev,
    /dev/dri or the node's own name (an absolute link resolves against the
    HOST root) must not make it create nodes in, or chmod, host paths."""
    b = bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=2"])
    proc = _proc_tree(tmp_path, 4243, "12:devices:/kubepods/pod1/c2\n")
    cg = tmp_path / "cgroup"
    (cg / "devices/kubepods/pod1/c2").mkdir(parents=True)
    croot = tmp_path / "proc/4243/root"
    victim_dir = tmp_path / "host-etc"
    victim_dir.mkdir()
    victim = victim_dir / "shadow"
    victim.write_text("secret")
    victim.chmod(0o600)
    if attack == "dri-dir":
        (croot / "dev").mkdir()
        os.symlink(str(victim_dir), croot / "dev/dri")
    elif attack == "dev-dir":
        os.symlink(str(victim_dir), croot / "dev")
    else:
        (croot / "dev/dri").mkdir(parents=True)
        os.symlink(str(victim), croot / "dev/dri/renderD144")
    state = json.dumps({"ociVersion": "1.1.0", "id": "c2", "pid": 4243, "bundle": b})
    p = run(["prestart", "--root", root, "--proc-root", proc, "--cgroup-root", str(cg)], state)
    assert p.returncode == 1 and "refused" in p.stderr, p.stderr
    assert stat.S_IMODE(os.stat(victim).st_mode) == 0o600 and victim.read_text() == "secret"
    assert sorted(os.listdir(victim_dir)) == ["shadow"]  # nothing created in the host directory


def test_prestart_accepts_an_existing_matching_node_and_refuses_a_wrong_one(root, tmp_path):
    b = bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=2"])
    proc = _proc_tree(tmp_path, 4244, "12:devices:/kubepods/pod1/c3\n")
    cg = tmp_path / "cgroup"
    (cg / "devices/kubepods/pod1/c3").mkdir(parents=True)
    state = json.dumps({"ociVersion": "1.1.0", "id": "c3", "pid": 4244, "bundle": b})
    args = ["prestart", "--root", root, "--proc-root", proc, "--cgroup-root", str(cg)]
    first = run(args, state)
    if first.returncode != 0:
        pytest.skip("no CAP_MKNOD in this environment")
    assert run(args, state).returncode == 0  # idempotent: the nodes are there and right
    node = tmp_path / "proc/4244/root/dev/dri/renderD144"
    os.unlink(node)
    node.write_text("not a device")
    p = run(args, state)
    assert p.returncode == 1 and "not char device 226:144" in p.stderr


def test_prestart_refuses_cgroup_v2(root, tmp_path):
    b = bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=0"])
    proc = _proc_tree(tmp_path, 77, "0::/kubepods.slice/pod1/c1\n")
    state = json.dumps({"ociVersion": "1.1.0", "id": "c1", "pid": 77, "bundle": b})
    p = run(["prestart", "--root", root, "--proc-root", proc], state)
    assert p.returncode == 1 and "precreate" in p.stderr and "cgroup-v1" in p.stderr
    # a non-GPU container needs nothing from the hook, whatever the cgroup version
    b2 = tmp_path / "b2"
    b2.mkdir()
    (b2 / "config.json").write_text(json.dumps({"process": {"env": []}}))
    st2 = json.dumps({"pid": 77, "bundle": str(b2)})
    assert run(["prestart", "--root", root, "--proc-root", proc], st2).returncode == 0


def test_annotation_needs_privilege_with_envvar_privileged_only(root, tmp_path):
    """Runtimes copy pod annotations into the spec: with --envvar-privileged-only
    an unprivileged container cannot name GPUs through amd.com/gpu.devices."""
    b = bundle(tmp_path, annotations={"amd.com/gpu.devices": "all"})
    p = run(["apply", "--bundle", b, "--root", root, "--dry-run", "--envvar-privileged-only"])
    assert p.returncode == 0 and json.loads(p.stdout) == {"devices": []}
    b = bundle(tmp_path, annotations={"amd.com/gpu.devices": "all"},
               extra={"process": {"args": ["sh"], "env": [], "capabilities": {"bounding": ["CAP_SYS_ADMIN"]}}})
    p = run(["apply", "--bundle", b, "--root", root, "--dry-run", "--envvar-privileged-only"])
    assert json.loads(p.stdout)["annotations"]["amd.com/gpu.injected"] == "0,1,2,3"
    # without the policy flag the annotation still selects devices (trusted runtimes)
    b = bundle(tmp_path, annotations={"amd.com/gpu.devices": "1"})
    p = run(["apply", "--bundle", b, "--root", root, "--dry-run"])
    assert json.loads(p.stdout)["annotations"]["amd.com/gpu.injected"] == "1"


def test_selectors_bdf_and_unknown(root, tmp_path):
    b = bundle(tmp_path)
    p = run(["apply", "--bundle", b, "--root", root, "--devices", "0000:0a:00.0"])
    assert p.returncode == 0, p.stderr
    assert [d["path"] for d in spec_of(b)["linux"]["devices"]][1] == "/dev/dri/renderD136"
    p = run(["apply", "--bundle", b, "--root", root, "--devices", "7"])
    assert p.returncode == 1 and "unknown device" in p.stderr


def test_non_gpu_container_untouched(root, tmp_path):
    b = bundle(tmp_path)
    before = open(os.path.join(b, "config.json")).read()
    assert run(["apply", "--bundle", b, "--root", root]).returncode == 0
    assert open(os.path.join(b, "config.json")).read() == before
    assert run(["apply", "--bundle", b, "--root", root, "--devices", "none"]).returncode == 0


def test_mount_rocm_and_dry_run(root, tmp_path):
    b = bundle(tmp_path, env=["AMD_VISIBLE_DEVICES=0"])
    p = run(["apply", "--bundle", b, "--root", root, "--mount-rocm", "--dry-run"])
    assert p.returncode == 0
    out = json.loads(p.stdout)
    assert out["mounts"][0]["destination"] == "/opt/rocm" and "ro" in out["mounts"][0]["options"]
    assert "devices" not in spec_of(b)["linux"]  # dry run did not write


@pytest.mark.parametrize("bad", ['{"bundle": 5}', "not json", "{}", '{"bundle": "/nonexistent"}'])
def test_bad_state(root, bad):
    p = run(["prestart", "--root", root], bad)
    assert p.returncode == 1


def test_bad_config_json(root, tmp_path):
    b = tmp_path / "bb"
    b.mkdir()
    (b / "config.json").write_text('{"process": {"env": ["AMD_VISIBLE_DEVICES=0"]}, "x": [1, 2,')
    p = run(["apply", "--bundle", str(b), "--root", root])
    assert p.returncode == 1 and "json" in p.stderr


def test_json_roundtrip_escapes(root, tmp_path):
    b = bundle(tmp_path, env=['AMD_VISIBLE_DEVICES=0', 'X=a"b\\cé\n'], extra={"hostname": "h☃"})
    assert run(["apply", "--bundle", b, "--root", root]).returncode == 0
    s = spec_of(b)
    assert 'X=a"b\\cé\n' in s["process"]["env"] and s["hostname"] == "h☃"
