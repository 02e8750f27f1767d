"""Randomized fault injection on the simulated cluster (tools/chaos_sim.py):
pod deletions, driver loss, kubelet restarts, container <-> vm-passthrough
switches and ClusterPolicy edits, each followed by convergence to Ready."""

import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("seed", [2, 3])
def test_cluster_converges_after_each_fault(seed):
    import chaos_sim

    assert chaos_sim.run_seed(seed, steps=6, settle_s=0.3, timeout=60.0)
