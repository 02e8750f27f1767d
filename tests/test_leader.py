"""Operator leader election on a coordination.k8s.io/v1 Lease (kube/leader.py):
one active controller among replicas, takeover after expiry, clean release."""

import threading
import time

import pytest

from amdgpu_operator.kube import resources as R
from amdgpu_operator.kube.client import LocalClient
from amdgpu_operator.kube.fakeapi import FakeApiServer
from amdgpu_operator.kube.leader import LEASE_API, LeaderElector, micro_time, parse_micro_time

NS = "gpu-operator-resources"


class Clock:
    def __init__(self):
        self.t = 1_700_000_000.0

    def __call__(self):
        return self.t


@pytest.fixture
def client():
    c = LocalClient(FakeApiServer())
    c.create(R.new("v1", "Namespace", NS))
    return c


def elector(client, ident, clock, mono=None, **kw):
    # the fake clock drives both the written timestamps and the local expiry clock
    mono = mono or (clock if isinstance(clock, Clock) else time.monotonic)
    return LeaderElector(client, "amd-gpu-operator-leader", NS, ident, clock=clock, mono=mono, **kw)


def test_micro_time_round_trip():
    t = 1_700_000_123.456789
    assert abs(parse_micro_time(micro_time(t)) - t) < 1e-5
    assert parse_micro_time("2024-01-01T00:00:00Z") == 1704067200.0 and parse_micro_time(None) is None


def test_one_holder_and_takeover_after_expiry(client):
    clock = Clock()
    a, b = elector(client, "a", clock), elector(client, "b", clock)
    assert a.try_acquire_or_renew() and not b.try_acquire_or_renew()
    clock.t += 10
    assert a.try_acquire_or_renew()  # renewed
    clock.t += 0.1
    assert not b.try_acquire_or_renew()  # b sees the renewal 0.1 s after it happened
    clock.t += 14.8
    assert not b.try_acquire_or_renew()  # unchanged for 14.8 s of b's clock, lease 15 s
    clock.t += 0.2
    assert b.try_acquire_or_renew()  # expired: b takes over
    spec = client.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)["spec"]
    assert spec["holderIdentity"] == "b" and spec["leaseTransitions"] == 1
    assert not a.try_acquire_or_renew()


class SkewedClock:
    def __init__(self, base: Clock, skew: float):
        self.base, self.skew = base, skew

    def __call__(self):
        return self.base.t + self.skew


@pytest.mark.parametrize("skew", [-60.0, +60.0])
def test_clock_skew_does_not_hand_over_a_live_lease(client, skew):
    """The holder's wall clock is a minute off: its renewTime looks long
    expired (or far in the future) to the standby.  Expiry is measured on the
    standby's own clock from the moment it saw the record change, so the
    standby takes over only after the holder has really stopped renewing."""
    clock = Clock()
    a = elector(client, "a", SkewedClock(clock, skew), mono=clock)
    b = elector(client, "b", clock)
    assert a.try_acquire_or_renew()
    for _ in range(10):  # a keeps renewing every 2 s; b keeps looking
        assert not b.try_acquire_or_renew()
        clock.t += 2
        assert a.try_acquire_or_renew()
    # a dies: the record stops changing; b takes over one lease duration later
    assert not b.try_acquire_or_renew()
    clock.t += 14.9
    assert not b.try_acquire_or_renew()
    clock.t += 0.2
    assert b.try_acquire_or_renew()


def test_racing_candidates_one_wins(client):
    clock = Clock()
    a = elector(client, "a", clock)
    assert a.try_acquire_or_renew()
    # b and c have watched the lease; a stops renewing and is long gone
    b, c = elector(client, "b", clock), elector(client, "c", clock)
    assert not b.try_acquire_or_renew() and not c.try_acquire_or_renew()
    clock.t += 60
    lease = client.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)
    # b and c both read the expired lease; both try to take it on the same resourceVersion
    orig_get = client.get
    client.get = lambda *a_, **k: R.deep(lease)
    try:
        wins = [b.try_acquire_or_renew(), c.try_acquire_or_renew()]
    finally:
        client.get = orig_get
    assert sorted(wins) == [False, True]


def test_release_lets_a_standby_take_over_at_once(client):
    clock = Clock()
    a, b = elector(client, "a", clock), elector(client, "b", clock)
    assert a.try_acquire_or_renew()
    a.release()
    assert b.try_acquire_or_renew()  # no need to wait out the 15 s lease
    assert client.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)["spec"]["holderIdentity"] == "b"


def test_run_loop_leads_loses_and_releases(client):
    """run(): leads while renewing; a lost renewal ends the lead callback;
    a stop releases the lease."""
    clock = time.time
    kw = dict(lease_s=1.5, renew_deadline_s=0.6, retry_period_s=0.05)
    a = elector(client, "a", clock, **kw)
    stop = threading.Event()
    led = []

    def lead(ended):
        led.append(time.monotonic())
        ended.wait(10)

    th = threading.Thread(target=lambda: led.append(a.run(stop, lead)))
    th.start()
    deadline = time.time() + 5
    while not a.leading.is_set() and time.time() < deadline:
        time.sleep(0.01)
    assert a.leading.is_set()
    # another writer steals the lease behind a's back: renewals now fail
    lease = client.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)
    lease["spec"]["holderIdentity"] = "intruder"
    lease["spec"]["renewTime"] = micro_time(time.time() + 30)
    client.update(lease)
    th.join(5)
    assert not th.is_alive() and led[-1] is True  # leadership lost while still running
    assert not a.leading.is_set()
    # a clean stop releases
    b = elector(client, "b", clock, **kw)
    lease = client.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)
    lease["spec"].update({"holderIdentity": "", "renewTime": micro_time(0)})
    client.update(lease)
    stop2 = threading.Event()
    th = threading.Thread(target=lambda: b.run(stop2, lambda ended: ended.wait(10)))
    th.start()
    while not b.leading.is_set() and time.time() < deadline + 5:
        time.sleep(0.01)
    stop2.set()
    th.join(10)
    assert client.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)["spec"]["holderIdentity"] == ""


def test_bad_timings_rejected(client):
    with pytest.raises(ValueError):
        LeaderElector(client, "x", NS, "a", lease_s=5, renew_deadline_s=6, retry_period_s=1)


def test_chart_runs_the_operator_with_leader_election():
    from amdgpu_operator.helm.render import render_chart

    objs = render_chart(set_flags=["operator.replicas=2"])
    dep = [o for o in objs if o["kind"] == "Deployment" and o["metadata"]["name"] == "amd-gpu-operator"][0]
    assert dep["spec"]["replicas"] == 2
    args = dep["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "--leader-elect" in args
    role = [o for o in objs if o["kind"] == "ClusterRole" and o["metadata"]["name"] == "amd-gpu-operator"][0]
    assert any("leases" in r["resources"] and "coordination.k8s.io" in r["apiGroups"] for r in role["rules"])
    off = render_chart(set_flags=["operator.leaderElection=false"])
    dep = [o for o in off if o["kind"] == "Deployment" and o["metadata"]["name"] == "amd-gpu-operator"][0]
    assert "--leader-elect" not in dep["spec"]["template"]["spec"]["containers"][0]["args"]


# ------------------------------------------------------------------ events

def test_event_recorder_aggregates_repeats(client):
    from amdgpu_operator.kube.events import WARNING, EventRecorder, events_for

    clock = Clock()
    node = client.create(R.new("v1", "Node", "gpu-0"))
    rec = EventRecorder(client, "amd-gpu-operator", clock=clock)
    rec.record(node, WARNING, "ValidationFailed", "boom")
    clock.t += 5
    rec.record(node, WARNING, "ValidationFailed", "boom")
    rec.record(node, WARNING, "ValidationFailed", "other")
    evs = events_for(client, "Node", "gpu-0")
    assert sorted((e["message"], e["count"]) for e in evs) == [("boom", 2), ("other", 1)]
    assert all(e["metadata"]["namespace"] == "default" and e["involvedObject"]["uid"] == node["metadata"]["uid"]
               and e["source"]["component"] == "amd-gpu-operator" for e in evs)
    clock.t += 601  # outside the aggregation window: a new Event
    rec.record(node, WARNING, "ValidationFailed", "boom")
    assert len(events_for(client, "Node", "gpu-0")) == 3
    EventRecorder(None, "x").record(node, WARNING, "r", "m")  # no API: silently nothing


def test_bring_up_and_upgrade_leave_events(tmp_path):
    """kubectl describe parity (README.md:179): the ClusterPolicy reports Ready,
    the node reports its validation and each driver-upgrade step."""
    from amdgpu_operator.api.clusterpolicy import REFERENCE_SET_FLAGS, parse_set_flags
    from amdgpu_operator.controller import upgrade as U
    from amdgpu_operator.kube.events import events_for
    from amdgpu_operator.testing.simcluster import NodeSpec, SimCluster

    ref = parse_set_flags(REFERENCE_SET_FLAGS)
    c = SimCluster(str(tmp_path / "c"), [NodeSpec("gpu-0", 1)], fake_gpu=True).start()
    try:
        c.install_operator(ref)
        c.wait_ready(60, {"gpu-0": 1})
        deadline = time.time() + 10
        while time.time() < deadline and not events_for(c.client, "ClusterPolicy", "cluster-policy"):
            time.sleep(0.05)
        cp_events = events_for(c.client, "ClusterPolicy", "cluster-policy")
        assert [e["reason"] for e in cp_events] == ["Ready"] and "time-to-Ready" in cp_events[0]["message"]
        node_events = events_for(c.client, "Node", "gpu-0")
        assert any(e["reason"] == "GPUValidated" and e["type"] == "Normal" for e in node_events)
        cp = c.policy()
        cp["spec"]["driver"]["driverVersion"] = "6.14.0"
        c.client.update(cp)
        deadline = time.time() + 60
        while time.time() < deadline:
            reasons = [e["message"] for e in events_for(c.client, "Node", "gpu-0") if e["reason"] == "DriverUpgrade"]
            if f"driver upgrade: {U.DONE}" in reasons:
                break
            time.sleep(0.05)
        assert f"driver upgrade: {U.CORDON}" in reasons and f"driver upgrade: {U.DONE}" in reasons
    finally:
        c.stop()


def test_operator_process_releases_the_lease_on_sigterm(tmp_path):
    """``amdgpu-operator operator --leader-elect`` (the chart default) stops on
    SIGTERM and releases its Lease, so a standby does not wait out 15 s."""
    import os
    import signal
    import subprocess
    import sys

    from amdgpu_operator.kube.httpapi import HttpApiServer

    api = FakeApiServer()
    LocalClient(api).create(R.new("v1", "Namespace", NS))
    srv = HttpApiServer(api).start()
    try:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        p = subprocess.Popen([sys.executable, "-m", "amdgpu_operator", "operator", "--server", srv.url,
                              "--namespace", NS, "--leader-elect", "--health-port", "0"],
                             cwd=root, env={**os.environ, "POD_NAME": "op-0"},
                             stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        c = LocalClient(api)
        deadline = time.time() + 60
        holder = None
        while time.time() < deadline and holder != "op-0":
            try:
                holder = c.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)["spec"]["holderIdentity"]
            except Exception:  # noqa: BLE001 - not created yet
                pass
            time.sleep(0.05)
        assert holder == "op-0", p.stdout.read() if p.poll() is not None else "no lease"
        p.send_signal(signal.SIGTERM)
        rc = p.wait(timeout=20)
        assert rc == 0
        assert c.get(LEASE_API, "Lease", "amd-gpu-operator-leader", NS)["spec"]["holderIdentity"] == ""
    finally:
        srv.stop()
