"""Randomized fault injection on the simulated cluster (tools/chaos_sim.py):
pod deletions, driver loss, kubelet restarts, container <-> vm-passthrough
switches, ClusterPolicy edits, driver upgrades and partition changes (also
while a process holds the GPU), each followed by convergence to Ready and,
where the fault must revalidate the node, a fresh validation record."""

import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.parametrize("seed", [2, 3])
def test_cluster_converges_after_each_fault(seed):
    import chaos_sim

    assert chaos_sim.run_seed(seed, steps=6, settle_s=0.3, timeout=60.0)


def test_a_fault_that_does_not_land_fails_the_harness():
    """Ready again is not enough: a step that must revalidate the node and
    leaves no fresh validation record (here a no-op posing as one) fails."""
    import chaos_sim

    assert not chaos_sim.run_seed(1, steps=2, settle_s=0.1, timeout=3.0, inject_noop=1)


def test_dra_cluster_converges_after_each_fault():
    """The same with the DRA driver advertising the GPUs: Ready includes each
    node's ResourceSlice listing its devices (2 or 16 after a partition
    change), and claimpod faults run a user's claim workload in between."""
    import chaos_sim

    assert chaos_sim.run_seed(51, steps=6, settle_s=0.3, timeout=60.0, dra=True)
