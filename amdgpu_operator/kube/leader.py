"""Leader election on a ``coordination.k8s.io/v1`` Lease (operator HA).

The reference's operator is a Deployment installed by ``helm install --wait``
(/root/reference/README.md:101); upstream runs it with leader election so
``replicas > 1`` gives a warm standby instead of two controllers fighting
over the same DaemonSets.  Same protocol as client-go's leaderelection:

* the Lease ``spec`` holds ``holderIdentity``, ``leaseDurationSeconds``,
  ``acquireTime``, ``renewTime`` and ``leaseTransitions``;
* a candidate takes the Lease when it does not exist, when it holds it
  already, when it was released (empty holder), or when the record has not
  changed for ``leaseDurationSeconds`` of the candidate's OWN monotonic
  clock: expiry is measured from the local time at which the candidate last
  saw (holder, renewTime, resourceVersion) change, never by comparing the
  holder's ``renewTime`` - written with the holder's clock - against the
  candidate's wall clock, so skewed node clocks cannot hand a live lease to
  a standby (client-go's observedRecord/observedTime); every write is an
  update on the read ``resourceVersion``, so of two candidates racing for an
  expired Lease exactly one wins (the other gets a Conflict);
* the leader renews every ``retry_period``; if it cannot renew within
  ``renew_deadline`` it stops leading (the caller stops its controller and
  the process exits, so a standby takes over after the lease expires);
* on a clean shutdown the leader releases the Lease (empty holder, duration
  1 s) so a standby does not wait out the full lease.
"""

from __future__ import annotations

import threading
import time
from datetime import datetime, timezone

from .errors import AlreadyExists, Conflict, NotFound
from ..utils.logs import get_logger

log = get_logger("amdgpu.leader")
LEASE_API = "coordination.k8s.io/v1"


def micro_time(t: float) -> str:
    """Kubernetes MicroTime (RFC 3339 with microseconds, UTC)."""
    return datetime.fromtimestamp(t, tz=timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def parse_micro_time(s: str | None) -> float | None:
    if not s:
        return None
    for fmt in ("%Y-%m-%dT%H:%M:%S.%fZ", "%Y-%m-%dT%H:%M:%SZ"):
        try:
            return datetime.strptime(s, fmt).replace(tzinfo=timezone.utc).timestamp()
        except ValueError:
            continue
    return None


class LeaderElector:
    def __init__(self, client, name: str, namespace: str, identity: str, lease_s: float = 15.0,
                 renew_deadline_s: float = 10.0, retry_period_s: float = 2.0, clock=time.time,
                 mono=time.monotonic):
        if not retry_period_s < renew_deadline_s < lease_s:
            raise ValueError("need retry_period < renew_deadline < lease duration")
        self.client = client
        self.name = name
        self.namespace = namespace
        self.identity = identity
        self.lease_s = lease_s
        self.renew_deadline_s = renew_deadline_s
        self.retry_period_s = retry_period_s
        self.clock = clock  # wall time: only what this candidate writes into the Lease
        self.mono = mono    # local monotonic time: all expiry decisions
        self.leading = threading.Event()
        self.transitions_seen = 0
        self._observed: tuple | None = None  # (holder, renewTime, resourceVersion) last seen
        self._observed_at = 0.0               # self.mono() when it last changed

    # -------------------------------------------------------------- one try
    def try_acquire_or_renew(self) -> bool:
        """One attempt; True when this identity holds the Lease afterwards."""
        now = self.clock()
        try:
            lease = self.client.get(LEASE_API, "Lease", self.name, self.namespace)
        except NotFound:
            lease = {"apiVersion": LEASE_API, "kind": "Lease",
                     "metadata": {"name": self.name, "namespace": self.namespace},
                     "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": int(self.lease_s),
                              "acquireTime": micro_time(now), "renewTime": micro_time(now), "leaseTransitions": 0}}
            try:
                self.client.create(lease)
                return True
            except (AlreadyExists, Conflict):
                return False
        spec = lease.setdefault("spec", {})
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_s)
        self.transitions_seen = int(spec.get("leaseTransitions") or 0)
        record = (holder, spec.get("renewTime"), (lease.get("metadata") or {}).get("resourceVersion"))
        if record != self._observed:
            self._observed, self._observed_at = record, self.mono()
        if holder and holder != self.identity and self._observed_at + duration > self.mono():
            return False  # someone else renewed it within the last lease duration (as seen here)
        if holder != self.identity:
            spec["leaseTransitions"] = self.transitions_seen + 1
            spec["acquireTime"] = micro_time(now)
        spec["holderIdentity"] = self.identity
        spec["leaseDurationSeconds"] = int(self.lease_s)
        spec["renewTime"] = micro_time(now)
        try:
            self.client.update(lease)  # carries the read resourceVersion: a racing writer gets a Conflict
            return True
        except (Conflict, NotFound):
            return False

    def release(self) -> None:
        try:
            lease = self.client.get(LEASE_API, "Lease", self.name, self.namespace)
        except NotFound:
            return
        if (lease.get("spec") or {}).get("holderIdentity") != self.identity:
            return
        lease["spec"].update({"holderIdentity": "", "leaseDurationSeconds": 1, "renewTime": micro_time(self.clock())})
        try:
            self.client.update(lease)
        except (Conflict, NotFound):
            pass

    # --------------------------------------------------------------- loops
    def acquire(self, stop: threading.Event) -> bool:
        """Block until leading (True) or ``stop`` (False)."""
        while not stop.is_set():
            try:
                if self.try_acquire_or_renew():
                    self.leading.set()
                    log.info("%s became leader of %s/%s", self.identity, self.namespace, self.name)
                    return True
            except Exception as e:  # noqa: BLE001 - API unavailable: keep trying
                log.warning("leader election: %s", e)
            stop.wait(self.retry_period_s)
        return False

    def renew_loop(self, stop: threading.Event) -> None:
        """Renew until ``stop`` or until renewing failed for ``renew_deadline``;
        clears :attr:`leading` when leadership is lost."""
        last_ok = time.monotonic()
        while not stop.wait(self.retry_period_s):
            try:
                ok = self.try_acquire_or_renew()
            except Exception as e:  # noqa: BLE001
                log.warning("lease renew: %s", e)
                ok = False
            if ok:
                last_ok = time.monotonic()
            elif time.monotonic() - last_ok >= self.renew_deadline_s:
                log.error("%s lost the lease %s/%s", self.identity, self.namespace, self.name)
                self.leading.clear()
                return
        self.leading.clear()

    def run(self, stop: threading.Event, lead) -> bool:
        """Acquire, then run ``lead(lost)`` while renewing; ``lost`` is an Event
        set when leadership ends (renew failure or ``stop``).  Returns True when
        leadership was lost while the process should keep running."""
        if not self.acquire(stop):
            return False
        lost = threading.Event()

        def renew():
            self.renew_loop(stop)
            lost.set()

        th = threading.Thread(target=renew, daemon=True, name="lease-renew")
        th.start()
        try:
            lead(lost)
        finally:
            lost.set()
            if stop.is_set():
                th.join(self.retry_period_s + 5)  # no renew may follow the release
                self.release()
        return not stop.is_set()
