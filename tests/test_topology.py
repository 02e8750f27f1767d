"""N3 topology library + N1 probe on real and synthetic MI355X sysfs trees."""

import os

import pytest

from amdgpu_operator.discovery import topology as T
from amdgpu_operator.testing import fakesys


@pytest.fixture
def real_root(tmp_path):
    return fakesys.build_from_real_fixture(str(tmp_path / "real"))


def test_real_fixture_enumerates_the_visible_mi355x(real_root):
    gpus = T.enumerate_gpus(real_root)
    assert len(gpus) == 1
    g = gpus[0]
    assert g.arch == "gfx950" and g.gfx_target_version == 90500
    assert g.cu_count == 256 and g.num_xcc == 8 and g.lds_size_kib == 160
    assert g.vram_bytes == 309220868096  # 288 GiB HBM3E
    assert g.bdf == "0000:a4:00.0" and g.render_minor == 184
    assert g.xgmi_links == 7  # the other 7 OAMs of the hive, hidden from this container
    assert g.device_id == 0x75A3
    assert g.max_engine_clk_mhz == 2400


def test_real_fixture_probe_accepts_renumbered_render_node(real_root):
    ok, msg = T.probe(real_root)
    assert ok, msg
    assert "re-numbered" in msg


def test_probe_fails_without_driver(tmp_path):
    root = fakesys.build_from_real_fixture(str(tmp_path / "nodrv"), driver_loaded=False)
    ok, msg = T.probe(root)
    assert not ok and "amdgpu" in msg


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_synthetic_hive(tmp_path, n):
    root = str(tmp_path / f"h{n}")
    fakesys.build_node(root, n)
    gpus = T.enumerate_gpus(root)
    assert len(gpus) == n
    assert all(g.partition_count == 1 and g.compute_partition == "SPX" for g in gpus)
    assert [g.physical_index for g in gpus] == list(range(n))
    links = T.links(root)
    assert len(links) == n * (n - 1)
    assert all(lk.is_xgmi and lk.weight == 15 and lk.max_bandwidth_mbps == 76000 for lk in links)
    ok, _ = T.probe(root, expect_gpus=n)
    assert ok
    ok, msg = T.probe(root, expect_gpus=n + 1)
    assert not ok and "expected" in msg


@pytest.mark.parametrize("mode,split", [("DPX", 2), ("QPX", 4), ("CPX", 8)])
def test_partition_modes(tmp_path, mode, split):
    root = str(tmp_path / mode)
    fakesys.build_node(root, 8, mode)
    gpus = T.enumerate_gpus(root)
    assert len(gpus) == 8 * split
    assert all(g.partition_count == split for g in gpus)
    assert all(g.cu_count == 256 // split for g in gpus)
    # partitions of one GPU share the BDF, get distinct stable device ids
    ids = [g.device_id_str for g in gpus]
    assert len(set(ids)) == len(ids)
    assert ids[1] == f"{gpus[0].bdf}-p1"


def test_visible_gpus_allow_list(tmp_path, monkeypatch):
    root = str(tmp_path / "v")
    fakesys.build_node(root, 8)
    monkeypatch.setenv("AMDGPU_VISIBLE_GPUS", "0,0000:a4:00.0")
    gpus = T.enumerate_gpus(root)
    assert [g.bdf for g in gpus] == ["0000:72:00.0", "0000:a4:00.0"]
    assert T.probe(root)[0]


def test_no_gpus(tmp_path):
    root = str(tmp_path / "empty")
    os.makedirs(root)
    assert T.enumerate_gpus(root) == []
    assert T.links(root) == []
    assert not T.probe(root)[0]


def test_smi_unavailable_is_explicit():
    # no GPU / amd-smi device in the build container: opening must fail loudly
    try:
        s = T.Smi()
    except Exception as e:  # noqa: BLE001
        assert "unavailable" in str(e)
    else:  # on a GPU box it works
        assert s.count() >= 1
        s.close()
