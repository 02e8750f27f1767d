"""ClusterPolicy reconciler: the operator controller.

Reference parity: ``helm install --wait gpu-operator`` starts the operator,
which turns the ClusterPolicy (values at /root/reference/README.md:104-110)
into operand DaemonSets and labels GPU nodes (README.md:119); the reference
then checks that every operand pod is Running/Completed (README.md:199-207).

Behaviour (level-triggered, idempotent, resumable from any point - all state
lives in Kubernetes objects):

1. pick the active ClusterPolicy (oldest; others are marked ``ignored``);
2. validate the spec (pydantic) - an invalid spec sets ``state=error``;
3. label nodes (``amd.com/gpu.present``, ``amd.com/gpu.deploy.<operand>``);
4. walk the ordered states, applying every enabled state's manifests (drift
   is reverted) and deleting disabled states' objects; a state is ready when
   all of its DaemonSets report every scheduled pod ready and updated;
5. write ``status``: ``state`` (ready / notReady / error), per-state readiness,
   conditions, and per-state time-to-ready spans since the policy was created
   (the time-to-Ready breakdown of SURVEY.md §5.1).

Dependencies between operands are enforced on the node by the operands' init
containers, not by the reconciler, so every state is applied on every pass
(same as the upstream controller stepping through all states).
"""

from __future__ import annotations

import os
import queue
import threading
import time
from dataclasses import dataclass, field

from pydantic import ValidationError

from .. import API_GROUP, API_VERSION
from ..api.clusterpolicy import STATES, ClusterPolicySpec, operand_enabled
from ..kube import resources as R
from ..kube.client import NotFound, apply_object
from ..kube.events import NORMAL, WARNING, EventRecorder
from ..utils.logs import get_logger
from .manifests import STATE_BUILDERS, owner_ref
from .nodes import label_nodes, nodes_selected

CP_API = f"{API_GROUP}/{API_VERSION}"
log = get_logger("amdgpu.operator")


@dataclass
class StateResult:
    name: str
    enabled: bool
    ready: bool
    objects: int = 0
    changed: int = 0
    detail: str = ""


# The order a pass applies the states in.  Reported in STATES order; applied
# with the validator right after the driver: on a first pass the operands'
# objects are created one HTTP request at a time (~30 ms on the MI355X box),
# and the validator's pod starts the longest chain of the bring-up (its
# Python start-up, then the HIP runtime behind the start gate), so its
# DaemonSet goes in before the toolkit's, device plugin's and exporters'.
APPLY_ORDER = sorted(STATES, key=lambda sk: {"pre-requisites": 0, "state-node-feature-discovery": 1,
                                              "state-driver": 2, "state-operator-validation": 3}.get(sk[0], 4))


@dataclass
class ReconcileResult:
    policy: str | None
    state: str
    states: list[StateResult] = field(default_factory=list)
    gpu_nodes: int = 0
    seconds: float = 0.0

    @property
    def ready(self) -> bool:
        return self.state == "ready"


def daemonset_ready(ds: dict) -> tuple[bool, str]:
    st = ds.get("status") or {}
    desired = int(st.get("desiredNumberScheduled", 0))
    ready = int(st.get("numberReady", 0))
    updated = int(st.get("updatedNumberScheduled", desired))
    if "observedGeneration" not in st:
        return False, "not yet observed by the DaemonSet controller"
    gen_ok = int(st["observedGeneration"]) >= int(ds["metadata"].get("generation", 1))
    ok = gen_ok and ready >= desired and updated >= desired
    return ok, f"{ready}/{desired} ready"


class ReconcileMetrics:
    """Operator self-metrics: reconcile count/duration, the
    policy state, per-state ready spans and time-to-Ready, in Prometheus text
    format for the operator's ``/metrics`` endpoint."""

    BUCKETS = (0.001, 0.005, 0.01, 0.05, 0.1, 0.5, 1.0, 5.0)

    def __init__(self):
        self._lock = threading.Lock()
        self.count = 0
        self.errors = 0
        self.sum = 0.0
        self.buckets = [0] * len(self.BUCKETS)
        self.state = "absent"
        self.ready_spans: dict[str, float] = {}
        self.time_to_ready: float | None = None
        self.upgrade_nodes: dict[str, int] = {}  # driver-upgrade state -> nodes

    def observe_upgrade(self, upgrade: dict | None) -> None:
        with self._lock:
            if upgrade is not None:
                self.upgrade_nodes = dict(upgrade.get("nodes") or {})

    def observe(self, res: "ReconcileResult", spans: dict[str, float], ttr: float | None) -> None:
        with self._lock:
            self.count += 1
            self.errors += res.state == "error"
            self.sum += res.seconds
            for i, b in enumerate(self.BUCKETS):
                if res.seconds <= b:
                    self.buckets[i] += 1
            self.state = res.state
            self.ready_spans = dict(spans)
            if ttr is not None:
                self.time_to_ready = ttr

    def render(self) -> str:
        p = "amd_gpu_operator_"
        with self._lock:
            out = [f"# TYPE {p}reconcile_total counter", f"{p}reconcile_total {self.count}",
                   f"# TYPE {p}reconcile_errors_total counter", f"{p}reconcile_errors_total {self.errors}",
                   f"# TYPE {p}reconcile_duration_seconds histogram"]
            for b, n in zip(self.BUCKETS, self.buckets):
                out.append(f'{p}reconcile_duration_seconds_bucket{{le="{b}"}} {n}')
            out += [f'{p}reconcile_duration_seconds_bucket{{le="+Inf"}} {self.count}',
                    f"{p}reconcile_duration_seconds_sum {self.sum:.6f}",
                    f"{p}reconcile_duration_seconds_count {self.count}",
                    f"# TYPE {p}policy_ready gauge", f"{p}policy_ready {int(self.state == 'ready')}",
                    f"# TYPE {p}state_ready_seconds gauge"]
            for k, v in sorted(self.ready_spans.items()):
                out.append(f'{p}state_ready_seconds{{state="{k}"}} {v:.4f}')
            if self.time_to_ready is not None:
                out += [f"# TYPE {p}time_to_ready_seconds gauge", f"{p}time_to_ready_seconds {self.time_to_ready:.4f}"]
            if self.upgrade_nodes:
                out.append(f"# TYPE {p}driver_upgrade_nodes gauge")
                for k, v in sorted(self.upgrade_nodes.items()):
                    out.append(f'{p}driver_upgrade_nodes{{state="{k}"}} {v}')
        return "\n".join(out) + "\n"


class ClusterPolicyReconciler:
    def __init__(self, client, namespace: str, clock=time.time):
        self.client = client
        self.namespace = namespace
        self.clock = clock
        self._ready_at: dict[str, dict[str, float]] = {}  # policy uid -> state -> seconds since creation
        self._created_at: dict[str, float] = {}
        self._nodes_changed = False  # a Node event since this pass labelled the nodes (set by the watches)
        self._ttr: dict[str, float] = {}
        self.reconciles = 0
        self.metrics = ReconcileMetrics()
        self._verified: dict = {}  # apply_object fast path: key -> (resourceVersion, desired hash)
        self.events = EventRecorder(client, "amd-gpu-operator")
        self._last_state: dict[str, str] = {}  # policy uid -> state last reported by an Event

    # ------------------------------------------------------------------ helpers
    def _active_policy(self) -> dict | None:
        cps = self.client.list(CP_API, "ClusterPolicy")
        if not cps:
            return None
        cps.sort(key=lambda c: (c["metadata"].get("creationTimestamp", ""), int(c["metadata"].get("resourceVersion", 0))))
        active = cps[0]
        for other in cps[1:]:
            if (other.get("status") or {}).get("state") != "ignored":
                other["status"] = {"state": "ignored", "message": f"only {active['metadata']['name']} is reconciled"}
                try:
                    self.client.update_status(other)
                except Exception as e:  # noqa: BLE001
                    log.warning("status update of ignored policy failed: %s", e)
        return active

    # objects of disabled operands known to be absent (kind, ns, name) -> since:
    # kinds without an informer are not asked again for ABSENT_MEMO_S
    ABSENT_MEMO_S = 30.0

    def _delete_objects(self, objs: list[dict]) -> int:
        """Delete the objects of a disabled operand.  Every pass does this for
        every disabled state (DRA, partition manager, VFIO, sandbox ... ~20
        objects by default), so what is known absent is not asked about: an
        informed kind is looked up in its cache, another kind is remembered
        as absent after its NotFound (for ABSENT_MEMO_S).  Over HTTP the ~20
        DELETEs were ~30 ms of every pass, on the path from the validator's
        Ready to the policy's (profiles/r5_ttr)."""
        n = 0
        now = time.monotonic()
        memo = self.__dict__.setdefault("_absent", {})
        for o in objs:
            t = R.rtype_of(o)
            ns = R.ns_of(o) if t.namespaced else None
            key = (t.api_version, t.kind, ns, R.name_of(o))
            if now - memo.get(key, -1e9) < self.ABSENT_MEMO_S:
                continue
            inf = getattr(self.client, "_informer", None)
            if inf is not None and inf(t.api_version, t.kind, ns) is not None:
                try:
                    self.client.get(t.api_version, t.kind, R.name_of(o), ns)
                except NotFound:
                    continue  # the cache is authoritative for what this operator created
            try:
                self.client.delete(t.api_version, t.kind, R.name_of(o), ns)
                n += 1
            except NotFound:
                if inf is None or inf(t.api_version, t.kind, ns) is None:
                    memo[key] = now
        return n

    def _forget_absent(self, o: dict) -> None:
        """An object this pass applies is no longer known absent."""
        memo = self.__dict__.get("_absent")
        if memo:
            t = R.rtype_of(o)
            memo.pop((t.api_version, t.kind, R.ns_of(o) if t.namespaced else None, R.name_of(o)), None)

    # ---------------------------------------------------------------- reconcile
    def reconcile(self) -> ReconcileResult:
        t0 = time.perf_counter()
        self.reconciles += 1
        cp = self._active_policy()
        if cp is None:
            return ReconcileResult(None, "absent")
        uid = cp["metadata"].get("uid", cp["metadata"]["name"])
        if uid not in self._created_at:
            self._created_at[uid] = self.clock()
        try:
            spec = ClusterPolicySpec.model_validate(cp.get("spec") or {})
        except ValidationError as e:
            msg = str(e).splitlines()[0] if str(e) else "invalid spec"
            self._write_status(cp, "error", [], 0, error=msg)
            self._state_event(cp, "error", msg)
            res = ReconcileResult(cp["metadata"]["name"], "error", seconds=time.perf_counter() - t0)
            self.metrics.observe(res, {}, None)
            return res

        if spec.psa.enabled:
            self._label_namespace_psa()
        self._nodes_changed = False
        gpu_nodes, patched, nfd_scanned, node_labels = label_nodes(self.client, spec)
        owner = owner_ref(cp)
        results: list[StateResult] = []
        driver_live = None
        pool_status = None
        ds_ready: dict[str, bool] = {}
        midpass = not os.environ.get("AMDGPU_EXPERIMENT_NO_MIDPASS_LABELS")  # A/B switch (profiles/r5_ttr)
        for state, key in APPLY_ORDER:
            if self._nodes_changed and midpass:
                # a node changed during this pass (NFD's labels come in during
                # the pass that created NFD, ~30 ms of creates on the box): its
                # GPU-node labels go on now, so the DaemonSets created later in
                # this pass, and those before it, get their pods without
                # waiting for the next pass
                self._nodes_changed = False
                gpu_nodes, again, nfd_scanned, node_labels = label_nodes(self.client, spec)
                patched = patched or again
            enabled = operand_enabled(spec, key)
            objs = STATE_BUILDERS[state](spec, self.namespace, owner)
            unlabelled: list[str] = []
            if state == "state-driver" and enabled and spec.driver.useDriverCRD:
                self._delete_objects([o for o in objs if o["kind"] == "DaemonSet"])  # the policy-wide one
                objs, pool_status = self._driver_pools(spec, owner)
            elif state == "state-driver" and enabled and spec.driver.usePrecompiled:
                from .manifests import state_driver_precompiled

                self._delete_objects([o for o in objs if o["kind"] == "DaemonSet"])  # the policy-wide one
                objs, unlabelled = state_driver_precompiled(spec, self.namespace, owner, self.client.list("v1", "Node"))
            if state == "state-driver":  # per-kernel DaemonSets of kernels no node runs any more
                self._prune_kernel_daemonsets({o["metadata"]["name"] for o in objs if o["kind"] == "DaemonSet"}
                                              if enabled else set())
            if not enabled:
                self._delete_objects(objs)
                results.append(StateResult(state, False, True, 0, 0, "disabled"))
                continue
            changed = 0
            ready = True
            detail = []
            pods_ready = 0
            for o in objs:
                self._forget_absent(o)
                live, action = apply_object(self.client, o, verified=self._verified)
                changed += action != "unchanged"
                if o["kind"] == "DaemonSet" and state == "state-driver":
                    driver_live = live
                if o["kind"] == "DaemonSet":
                    ok, d = daemonset_ready(live)
                    ds_ready[o["metadata"]["name"]] = ok
                    pods_ready += int((live.get("status") or {}).get("numberReady", 0))
                    sel = o["spec"]["template"]["spec"].get("nodeSelector") or {}
                    if ok and sel and int((live.get("status") or {}).get("desiredNumberScheduled", 0)) == 0 \
                            and nodes_selected(node_labels, sel):
                        ok, d = False, "not yet scheduled on the GPU nodes"
                    ready &= ok
                    detail.append(f"{o['metadata']['name']}: {d}")
            if state == "state-node-feature-discovery" and ready:
                # each NFD pod labels its node before it turns Ready; a Node read
                # older than the DaemonSet status would count a GPU node as none
                if nfd_scanned < pods_ready:
                    ready = False
                    detail.append(f"{nfd_scanned}/{pods_ready} nodes labelled")
            if unlabelled:
                ready = False
                detail.append(f"no kernel-version label yet on {unlabelled}")
            if state == "state-driver" and pool_status is not None:
                self._write_pool_status(pool_status, ds_ready)
                ready &= all(st["state"] != "error" for st in pool_status.values())
            results.append(StateResult(state, True, ready, len(objs), changed, "; ".join(detail)))
            if ready and (gpu_nodes == 0 or not patched):
                self._ready_at.setdefault(uid, {}).setdefault(state, self.clock() - self._created_at[uid])

        rank = {st: i for i, (st, _) in enumerate(STATES)}
        results.sort(key=lambda r: rank[r.name])  # reported in the states' order
        upgrade = None
        if spec.driver.enabled and spec.driver.upgradePolicy.autoUpgrade and gpu_nodes and self._upgrade_pending(
                driver_live):
            from .upgrade import DriverUpgradeController

            try:
                upgrade = DriverUpgradeController(self.client, self.namespace, self.clock, self.events).step(spec)
            except Exception as e:  # noqa: BLE001 - next pass retries
                log.warning("driver upgrade pass failed: %s", e)
        overall = "ready" if all(r.ready for r in results) else "notReady"
        if overall == "ready" and patched:
            overall = "notReady"  # node labels just changed: DaemonSet status is stale
        if overall == "ready" and spec.validator.enabled and gpu_nodes:
            from ..validator.validate import VALIDATED_LABEL
            from .nodes import is_gpu_node

            pending = [n["metadata"]["name"] for n in self.client.list("v1", "Node")
                       if is_gpu_node(n) and (n["metadata"].get("labels") or {}).get(VALIDATED_LABEL) != "true"]
            if pending:
                overall = "notReady"
        self._write_status(cp, overall, results, gpu_nodes, upgrade=upgrade)
        self.metrics.observe_upgrade(upgrade)
        if overall == "ready":
            self._ttr.setdefault(uid, self.clock() - self._created_at[uid])
        waiting = [r.name for r in results if r.enabled and not r.ready]
        self._state_event(cp, overall, f"waiting for {', '.join(waiting)}" if waiting else
                          "waiting for GPU node validation" if overall != "ready" else
                          f"all operands ready on {gpu_nodes} GPU node(s) (time-to-Ready {self._ttr.get(uid, 0):.2f} s)")
        res = ReconcileResult(cp["metadata"]["name"], overall, results, gpu_nodes, time.perf_counter() - t0)
        self.metrics.observe(res, self._ready_at.get(uid, {}), self._ttr.get(uid))
        log.debug("reconciled %s: %s (%.3fs)", res.policy, overall, res.seconds)
        return res

    def _state_event(self, cp: dict, state: str, message: str) -> None:
        """One Event per ClusterPolicy state change (``kubectl describe clusterpolicy``)."""
        uid = cp["metadata"].get("uid", cp["metadata"]["name"])
        prev = self._last_state.get(uid)
        if prev == state or (prev is None and state == "notReady"):
            return  # the first notReady of a fresh install is not news
        self._last_state[uid] = state
        if state == "ready":
            self.events.record(cp, NORMAL, "Ready", message)
        elif state == "error":
            self.events.record(cp, WARNING, "ReconcileFailed", message)
        else:
            self.events.record(cp, WARNING, "NotReady", message)

    def _prune_kernel_daemonsets(self, keep: set[str]) -> None:
        from .manifests import KERNEL_DS_LABEL

        stale = [d for d in self.client.list("apps/v1", "DaemonSet", self.namespace, label_selector=KERNEL_DS_LABEL)
                 if d["metadata"]["name"] not in keep]
        self._delete_objects(stale)

    def _driver_pools(self, spec, owner) -> tuple[list[dict], dict]:
        from .manifests import state_driver_pools

        drivers = self.client.list(CP_API, "AMDGPUDriver")
        return state_driver_pools(spec, self.namespace, owner, drivers, self.client.list("v1", "Node"))

    def _write_pool_status(self, statuses: dict[str, dict], ds_ready: dict[str, bool]) -> None:
        """AMDGPUDriver status: ready when its DaemonSet is (readiness from this pass)."""
        for name, st in statuses.items():
            if st["state"] == "pending":
                st["state"] = "ready" if ds_ready.get(f"amd-driver-daemonset-{name}") else "notReady"
            try:
                live = self.client.get(CP_API, "AMDGPUDriver", name)
            except NotFound:
                continue
            if live.get("status") != st:
                live["status"] = st
                try:
                    self.client.update_status(live)
                except Exception as e:  # noqa: BLE001
                    log.warning("AMDGPUDriver %s status: %s", name, e)

    PSA_LABELS = {f"pod-security.kubernetes.io/{mode}": "privileged" for mode in ("enforce", "audit", "warn")}

    def _label_namespace_psa(self) -> None:
        try:
            ns = self.client.get("v1", "Namespace", self.namespace)
        except NotFound:
            return
        labels = ns["metadata"].get("labels") or {}
        if any(labels.get(k) != v for k, v in self.PSA_LABELS.items()):
            self.client.patch("v1", "Namespace", self.namespace, {"metadata": {"labels": self.PSA_LABELS}})

    def _upgrade_pending(self, driver_ds: dict | None) -> bool:
        """Run the upgrade controller only while there is something to do: an
        outdated driver pod (OnDelete leaves it in place) or a node mid-upgrade."""
        from .upgrade import DONE, STATE_LABEL

        st = (driver_ds or {}).get("status") or {}
        if int(st.get("updatedNumberScheduled", 0)) < int(st.get("currentNumberScheduled", 0)):
            return True
        return any((n["metadata"].get("labels") or {}).get(STATE_LABEL, DONE) != DONE
                   for n in self.client.list("v1", "Node"))

    def _write_status(self, cp: dict, state: str, results: list[StateResult], gpu_nodes: int, error: str = "",
                      upgrade: dict | None = None) -> None:
        uid = cp["metadata"].get("uid", cp["metadata"]["name"])
        try:
            live = self.client.get(CP_API, "ClusterPolicy", cp["metadata"]["name"])
        except NotFound:
            return
        status = dict(live.get("status") or {})
        before = R.deep(status)
        status["state"] = state
        status["namespace"] = self.namespace
        status["gpuNodes"] = gpu_nodes
        if upgrade is not None and (upgrade["nodes"] or "driverUpgrade" in status):
            status["driverUpgrade"] = upgrade
        status["states"] = {r.name: ("disabled" if not r.enabled else "ready" if r.ready else "notReady")
                            for r in results}
        spans = self._ready_at.get(uid, {})
        if spans:
            status["stateReadySeconds"] = {k: round(v, 4) for k, v in spans.items()}
        if state == "ready" and "timeToReadySeconds" not in status and uid in self._created_at:
            status["timeToReadySeconds"] = round(self.clock() - self._created_at[uid], 4)
        now = time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())
        not_ready = [r.name for r in results if r.enabled and not r.ready]
        R.set_condition(status, "Ready", state == "ready", "Reconciled" if state == "ready" else
                        ("Error" if state == "error" else "OperandNotReady"),
                        error or (f"waiting for {', '.join(not_ready)}" if not_ready else "all operands ready"), now)
        R.set_condition(status, "Error", state == "error", "ReconcileFailed" if error else "NoError", error, now)
        if status == before:
            return
        live["status"] = status
        try:
            self.client.update_status(live)
        except Exception as e:  # noqa: BLE001 - next pass retries
            log.warning("status update failed: %s", e)

    # ------------------------------------------------------------------- loop
    def cached_kinds(self) -> list[tuple]:
        """What the loop reads through informer caches (kube/informer.py):
        (api_version, kind, namespace, triggers a reconcile)."""
        ns = self.namespace
        return [(CP_API, "ClusterPolicy", None, True), ("v1", "Node", None, True), ("apps/v1", "DaemonSet", ns, True),
                (CP_API, "AMDGPUDriver", None, True), ("v1", "Namespace", None, False),
                ("v1", "ServiceAccount", ns, False), ("v1", "Service", ns, False),
                ("rbac.authorization.k8s.io/v1", "ClusterRole", None, False),
                ("rbac.authorization.k8s.io/v1", "ClusterRoleBinding", None, False),
                ("node.k8s.io/v1", "RuntimeClass", None, False),
                ("monitoring.coreos.com/v1", "ServiceMonitor", ns, False)]

    def run(self, stop: threading.Event, resync_s: float = 30.0, debounce_s: float = 0.02,
            on_result=None, cache: bool = True) -> None:
        """Watch-driven loop: ClusterPolicy, Node, DaemonSet (operand
        namespace) and AMDGPUDriver changes trigger a (debounced) reconcile;
        plus periodic resync.  With ``cache`` the loop reads the objects it
        owns from informer caches kept by the same watches (a pass then makes
        no GETs) and writes through to the server."""
        events: queue.Queue = queue.Queue()
        server = self.client
        if cache:
            from ..kube.informer import CachedClient

            # reads of a kind go to the server until its informer has synced,
            # so the first pass does not wait for the initial lists; the
            # informers end with ``stop`` (e.g. leadership lost), and so does
            # this wrapping: a later run() builds fresh caches
            def on_event(kind):
                if kind == "Node":
                    self._nodes_changed = True
                events.put((kind, time.monotonic()))

            self.client = CachedClient(server, self.cached_kinds(), stop, on_event=on_event)
        else:
            watches = [(CP_API, "ClusterPolicy", None), ("v1", "Node", None), ("apps/v1", "DaemonSet", self.namespace),
                       (CP_API, "AMDGPUDriver", None)]
            for av, kind, ns in watches:
                threading.Thread(target=self._pump, args=(av, kind, ns, events, stop), daemon=True,
                                 name=f"operator-watch-{kind}").start()
        events.put(("start", time.monotonic()))
        try:
            self._loop(stop, events, resync_s, debounce_s, on_result)
        finally:
            self.client = server

    def _loop(self, stop, events, resync_s, debounce_s, on_result) -> None:
        last = 0.0
        # AMDGPU_RECONCILE_TRACE=<file>: one line per pass (wall time at the
        # triggering event and at the pass's start, its duration, the trigger)
        trace = os.environ.get("AMDGPU_RECONCILE_TRACE")
        while not stop.is_set():
            trigger, t_first = "resync", time.monotonic()
            try:
                trigger, t_first = events.get(timeout=min(resync_s, 0.5))
            except queue.Empty:
                if time.monotonic() - last < resync_s:
                    continue
            t_event = time.time()
            # leading edge: the first event after a quiet spell (a new
            # ClusterPolicy, a node NFD just labelled) is handled at once; an
            # event close behind a pass - usually the echo of that pass's own
            # writes - waits out the rest of the debounce window so a burst
            # costs one pass (the rest only: an operand that turns Ready just
            # after a pass, e.g. the validator, is seen at most debounce_s
            # later).  The window runs from the earlier of the pass's end and
            # the event: an event that came in during a long pass (NFD's node
            # labels during the pass that created NFD, ~30 ms over HTTP) has
            # waited already and starts the next pass at once.
            wait = debounce_s - (time.monotonic() - min(last, t_first))
            if wait > 0:
                time.sleep(wait)
            while True:  # coalesce bursts
                try:
                    events.get_nowait()
                except queue.Empty:
                    break
            t_pass = time.time()
            try:
                res = self.reconcile()
            except Exception as e:  # noqa: BLE001 - keep the controller alive
                log.exception("reconcile failed: %s", e)
                stop.wait(0.5)
                continue
            last = time.monotonic()
            if trace:
                with open(trace, "a") as f:
                    f.write(f"{t_event:.4f} {t_pass:.4f} {time.time() - t_pass:.4f} {trigger} {res.state}\n")
            if on_result is not None:
                on_result(res)

    def _pump(self, av, kind, ns, events: queue.Queue, stop: threading.Event) -> None:
        while not stop.is_set():
            try:
                for _etype, _obj in self.client.watch(av, kind, namespace=ns, stop=stop):
                    if kind == "Node":
                        self._nodes_changed = True
                    events.put((kind, time.monotonic()))
            except Exception as e:  # noqa: BLE001 - re-establish the watch
                log.debug("watch %s ended: %s", kind, e)
                stop.wait(0.5)


def cleanup_crd(client, crd_name: str = f"clusterpolicies.{API_GROUP}") -> bool:
    """Helm pre-delete hook (``operator.cleanupCRD``, README.md:110): delete the
    ClusterPolicy objects, then the CRD.  Returns True if the CRD existed."""
    for cp in client.list(CP_API, "ClusterPolicy"):
        try:
            client.delete(CP_API, "ClusterPolicy", cp["metadata"]["name"])
        except NotFound:
            pass
    try:  # AMDGPUDriver objects and their CRD go too (driver.useDriverCRD)
        for d in client.list(CP_API, "AMDGPUDriver"):
            client.delete(CP_API, "AMDGPUDriver", d["metadata"]["name"])
        client.delete("apiextensions.k8s.io/v1", "CustomResourceDefinition", f"amdgpudrivers.{API_GROUP}")
    except NotFound:
        pass
    try:
        client.delete("apiextensions.k8s.io/v1", "CustomResourceDefinition", crd_name)
        return True
    except NotFound:
        return False
