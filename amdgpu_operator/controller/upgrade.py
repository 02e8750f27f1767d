"""Cluster-wide driver upgrade controller (``driver.upgradePolicy``).

Reference parity: the reference installs the operator with the driver
DaemonSet enabled (/root/reference/README.md:104) and its pods run the driver
container (README.md:132-143,212).  Changing the driver version on a running
cluster must not take every GPU node down at once, so with
``driver.upgradePolicy.autoUpgrade`` the driver DaemonSet uses ``OnDelete`` and
this controller walks GPU nodes through the upgrade one bounded batch at a
time (``maxParallelUpgrades``), tracked in a node label as upstream does::

    upgrade-required -> cordon-required -> pod-deletion-required
      -> pod-restart-required -> validation-required -> uncordon-required
      -> upgrade-done                       (or upgrade-failed on timeout)

* outdated = the node's driver pod carries an older ``amd.com/driver-spec-hash``
  template label than the current driver spec;
* cordon: ``spec.unschedulable`` (only nodes the operator cordoned are
  uncordoned again, recorded in an annotation);
* pod deletion: GPU pods (``amd.com/gpu*`` limits) are evicted when
  ``drainEnabled``; with it off the node waits until they finish.  Either way
  the node moves on only once a fresh list shows no GPU pod left, Terminating
  ones included (they still hold ``/dev/kfd``), bounded by
  ``drainTimeoutSeconds`` (then force-deleted with ``podDeletionForce``, else
  ``upgrade-failed``);
* pod restart: the old driver pod is deleted, the DaemonSet creates the new
  one, whose ``amd-driver-manager`` init container unloads the old module;
* validation: the new driver pod is Ready, it reports the module it loaded for
  this spec (``amd.com/gpu-driver.spec-hash`` node annotation, written by
  ``driver/manager.py`` only after the old module was unloaded and the new one
  came up) and the node carries ``amd.com/gpu.validated=true`` again (the
  validator re-ran on the new driver).

The controller is level-triggered: every reconcile recomputes from the node
labels, so an operator restart resumes mid-upgrade.
"""

from __future__ import annotations

import hashlib
import json
import time

from ..api.clusterpolicy import ClusterPolicySpec
from ..kube import resources as R
from ..kube.errors import NotFound
from ..utils.logs import get_logger

log = get_logger("amdgpu.upgrade")

from ..wellknown import UPGRADE_STATE_LABEL as STATE_LABEL  # noqa: E402
HASH_LABEL = "amd.com/driver-spec-hash"
CORDONED_ANN = "amd.com/gpu-driver-upgrade.cordoned"
# the new driver pod (uid) after whose readiness the node's validator was restarted
VALIDATOR_RESTART_ANN = "amd.com/gpu-driver-upgrade.validator-restarted"
SINCE_ANN = "amd.com/gpu-driver-upgrade.since"
from ..wellknown import LOADED_HASH_ANN, LOADED_VERSION_ANN  # noqa: E402,F401 - written by the driver container
DRIVER_DS = "amd-driver-daemonset"
VALIDATOR_DS = "amd-operator-validator"

from ..wellknown import (ACTIVE, CORDON, DONE, FAILED, POD_DELETION, POD_RESTART,  # noqa: E402,F401 - re-exported
                         REQUIRED, UNCORDON, VALIDATION)


def driver_spec_hash(spec: ClusterPolicySpec) -> str:
    """Identity of what the driver pods install (image, versions, module params)."""
    d = spec.driver
    key = {"ref": d.ref("amd-driver"), "rocm": d.rocmVersion, "driver": d.driverVersion,
           "precompiled": d.usePrecompiled, "params": d.kernelModuleParams, "args": d.args, "env": d.env}
    return hashlib.sha1(json.dumps(key, sort_keys=True).encode()).hexdigest()[:16]


def _uses_gpu(pod: dict, client=None) -> bool:
    """amd.com/gpu or a gpu.amd.com DRA claim (wellknown.uses_gpu): an amdgpu
    unload finds the module busy while either kind runs."""
    from ..wellknown import uses_gpu

    get = (lambda ns, n: client.get("resource.k8s.io/v1beta1", "ResourceClaim", n, ns)) if client is not None else None
    return uses_gpu(pod, get)


class DriverUpgradeController:
    def __init__(self, client, namespace: str, clock=time.time, events=None):
        self.client = client
        self.namespace = namespace
        self.clock = clock
        self.events = events  # kube.events.EventRecorder: one Event per node transition

    def _set(self, node: dict, state: str, extra_ann: dict | None = None, unschedulable: bool | None = None) -> None:
        name = node["metadata"]["name"]
        patch: dict = {"metadata": {"labels": {STATE_LABEL: state},
                                    "annotations": {SINCE_ANN: str(round(self.clock(), 3)), **(extra_ann or {})}}}
        if unschedulable is not None:
            patch["spec"] = {"unschedulable": unschedulable}
        self.client.patch("v1", "Node", name, patch)
        node["metadata"].setdefault("labels", {})[STATE_LABEL] = state
        anns = node["metadata"].setdefault("annotations", {})
        for k, v in patch["metadata"]["annotations"].items():
            if v is None:
                anns.pop(k, None)
            else:
                anns[k] = v
        if unschedulable is not None:
            node.setdefault("spec", {})["unschedulable"] = unschedulable
        log.info("driver upgrade %s -> %s", name, state)
        if self.events is not None:
            from ..kube.events import NORMAL, WARNING

            if state == FAILED:
                self.events.record(node, WARNING, "DriverUpgradeFailed",
                                   "driver upgrade did not complete in time; the node stays cordoned until a retry succeeds")
            else:
                self.events.record(node, NORMAL, "DriverUpgrade", f"driver upgrade: {state}")

    def _gpu_pods(self, node_name: str) -> list[dict]:
        return [p for p in self.client.list("v1", "Pod", field_selector=f"spec.nodeName={node_name}")
                if _uses_gpu(p, self.client)]

    def _delete_pod(self, pod: dict, grace: int | None = None) -> None:
        try:
            self.client.delete("v1", "Pod", pod["metadata"]["name"], pod["metadata"].get("namespace"),
                               grace_period_seconds=grace)
        except NotFound:
            pass

    def _driver_pods(self) -> dict[str, dict]:
        """Driver pod per node; a live pod wins over one still Terminating."""
        out: dict[str, dict] = {}
        from .manifests import KERNEL_DS_LABEL

        pods = self.client.list("v1", "Pod", self.namespace, label_selector={"app": DRIVER_DS})
        # usePrecompiled: one DaemonSet per kernel, the same driver spec (and hash) on all
        pods += self.client.list("v1", "Pod", self.namespace, label_selector=KERNEL_DS_LABEL)
        for p in pods:
            node = p["spec"].get("nodeName")
            if node not in out or out[node]["metadata"].get("deletionTimestamp"):
                out[node] = p
        return out

    def step(self, spec: ClusterPolicySpec) -> dict:
        """One level-triggered pass over every driver node; returns a status summary."""
        from ..validator.validate import VALIDATED_LABEL
        from .manifests import DEPLOY_LABEL, OPERAND_LABELS

        pol = spec.driver.upgradePolicy
        desired = driver_spec_hash(spec)
        deploy = DEPLOY_LABEL.format(OPERAND_LABELS["driver"])
        nodes = [n for n in self.client.list("v1", "Node") if (n["metadata"].get("labels") or {}).get(deploy) == "true"]
        pods = self._driver_pods()
        now = self.clock()
        timeout = max(1.0, float(pol.drainTimeoutSeconds))

        def state(n):
            return (n["metadata"].get("labels") or {}).get(STATE_LABEL, "")

        def since(n):
            try:
                return float((n["metadata"].get("annotations") or {}).get(SINCE_ANN, now))
            except ValueError:
                return now

        # 1. mark outdated nodes
        for n in nodes:
            pod = pods.get(n["metadata"]["name"])
            outdated = pod is not None and (pod["metadata"].get("labels") or {}).get(HASH_LABEL) != desired
            if outdated and state(n) in ("", DONE, FAILED):
                if state(n) == FAILED and now - since(n) < timeout:
                    continue  # back off before retrying a failed node
                self._set(n, REQUIRED)
        # 2. admit a bounded batch
        active = sum(1 for n in nodes if state(n) in ACTIVE)
        budget = (pol.maxParallelUpgrades - active) if pol.maxParallelUpgrades > 0 else len(nodes)
        for n in sorted(nodes, key=lambda x: x["metadata"]["name"]):
            if budget <= 0:
                break
            if state(n) == REQUIRED:
                self._set(n, CORDON)
                budget -= 1
        # 3. advance every active node as far as it can go this pass
        for n in nodes:
            name = n["metadata"]["name"]
            for _ in range(len(ACTIVE)):
                st = state(n)
                if st == CORDON:
                    # a retry after upgrade-failed finds the node cordoned by the
                    # first attempt: keep that attempt's record of who cordoned it
                    ann = {} if CORDONED_ANN in (n["metadata"].get("annotations") or {}) else \
                        {CORDONED_ANN: "false" if (n.get("spec") or {}).get("unschedulable") else "true"}
                    self._set(n, POD_DELETION, ann, unschedulable=True)
                elif st == POD_DELETION:
                    expired = now - since(n) > timeout
                    gpu_pods = self._gpu_pods(name)
                    evict = pol.drainEnabled or (expired and pol.podDeletionForce)
                    if gpu_pods and evict:
                        for p in gpu_pods:
                            # a deleted pod stays Terminating for its grace period and
                            # keeps /dev/kfd open; past the drain timeout it is forced
                            terminating = bool(p["metadata"].get("deletionTimestamp"))
                            if terminating and not (expired and pol.podDeletionForce):
                                continue
                            self._delete_pod(p, 0 if terminating else None)
                        gpu_pods = self._gpu_pods(name)
                    if gpu_pods:
                        if expired and not pol.podDeletionForce:
                            self._set(n, FAILED)
                        break  # wait for the workloads to finish / terminate
                    self._set(n, POD_RESTART)
                elif st == POD_RESTART:
                    pod = pods.get(name)
                    if pod is not None and (pod["metadata"].get("labels") or {}).get(HASH_LABEL) != desired:
                        try:
                            self.client.delete("v1", "Pod", pod["metadata"]["name"], self.namespace)
                        except NotFound:
                            pass
                    # the node is validated again only by a validator run on the new driver
                    self.client.patch("v1", "Node", name, {"metadata": {"labels": {VALIDATED_LABEL: None}}})
                    self._set(n, VALIDATION, {VALIDATOR_RESTART_ANN: None})
                    break  # the DaemonSet controller creates the new driver pod
                elif st == VALIDATION:
                    pod = self._driver_pods().get(name)
                    fresh = pod is not None and (pod["metadata"].get("labels") or {}).get(HASH_LABEL) == desired
                    ready = fresh and (R.condition(pod, "Ready") or {}).get("status") == "True"
                    cur = self.client.get("v1", "Node", name)
                    validated = (cur["metadata"].get("labels") or {}).get(VALIDATED_LABEL) == "true"
                    # the new driver pod reports the spec it actually loaded (driver/manager.py)
                    loaded = (cur["metadata"].get("annotations") or {}).get(LOADED_HASH_ANN) == desired
                    uid = pod["metadata"].get("uid", "") if pod is not None else ""
                    restarted = (cur["metadata"].get("annotations") or {}).get(VALIDATOR_RESTART_ANN) == uid
                    if ready and loaded and not restarted:
                        # only now, with the new module live and its driver-ready
                        # written, does a fresh validator run: one restarted with the
                        # driver pod could pass its driver gate on the old driver's
                        # ready file (the new pod's upgrade check had not cleared it)
                        # and validate the node on the module being replaced
                        self.client.patch("v1", "Node", name, {"metadata": {"labels": {VALIDATED_LABEL: None}}})
                        for vp in self.client.list("v1", "Pod", self.namespace, label_selector={"app": VALIDATOR_DS},
                                                   field_selector=f"spec.nodeName={name}"):
                            try:
                                self.client.delete("v1", "Pod", vp["metadata"]["name"], self.namespace)
                            except NotFound:
                                pass
                        self._set(n, VALIDATION, {VALIDATOR_RESTART_ANN: uid, SINCE_ANN: (n["metadata"].get(
                            "annotations") or {}).get(SINCE_ANN)})
                        break
                    if ready and validated and loaded:
                        self._set(n, UNCORDON, {VALIDATOR_RESTART_ANN: None})
                    elif now - since(n) > max(timeout, spec.driver.startupProbeTimeoutSeconds):
                        self._set(n, FAILED)
                        break
                    else:
                        break
                elif st == UNCORDON:
                    ours = (n["metadata"].get("annotations") or {}).get(CORDONED_ANN) == "true"
                    # the cordon record belongs to this upgrade only; the next one records afresh
                    self._set(n, DONE, {CORDONED_ANN: None}, unschedulable=False if ours else None)
                else:
                    break
        counts: dict[str, int] = {}
        for n in self.client.list("v1", "Node"):
            st = (n["metadata"].get("labels") or {}).get(STATE_LABEL)
            if st:
                counts[st] = counts.get(st, 0) + 1
        return {"desiredHash": desired, "nodes": counts,
                "inProgress": sum(v for k, v in counts.items() if k in ACTIVE + (REQUIRED,))}
