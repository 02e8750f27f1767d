"""Helm chart: reference install flags, generated CRD/values freshness,
template rendering (no helm binary in the environment)."""

import os

import pytest
import yaml

from amdgpu_operator.api.clusterpolicy import (REFERENCE_SET_FLAGS, ClusterPolicySpec, parse_set_flags,
                                               spec_from_values)
from amdgpu_operator.helm import render as H
from amdgpu_operator.helm.crd import crd_yaml
from amdgpu_operator.helm.values import values_yaml


def test_crd_file_is_generated_from_spec():
    with open(os.path.join(H.CHART_DIR, "crds", "amd.com_clusterpolicies.yaml")) as f:
        assert f.read() == crd_yaml(), "run python -m amdgpu_operator.helm.crd > deploy/.../crds/amd.com_clusterpolicies.yaml"


def test_values_file_is_generated_from_spec():
    with open(os.path.join(H.CHART_DIR, "values.yaml")) as f:
        assert f.read() == values_yaml(), "run python -m amdgpu_operator.helm.values > deploy/helm/amd-gpu-operator/values.yaml"


def test_reference_set_flags_render():
    docs = H.render_chart(set_flags=REFERENCE_SET_FLAGS)
    kinds = {(d["kind"], d["metadata"]["name"]) for d in docs}
    assert ("ClusterPolicy", "cluster-policy") in kinds
    assert ("Deployment", "amd-gpu-operator") in kinds
    assert ("Job", "amd-gpu-operator-cleanup-crd") in kinds  # operator.cleanupCRD=true
    cp = next(d for d in docs if d["kind"] == "ClusterPolicy")
    spec = ClusterPolicySpec.model_validate(cp["spec"])
    want = spec_from_values(H.chart_values(set_flags=REFERENCE_SET_FLAGS))
    assert spec == want
    assert spec.driver.enabled and spec.toolkit.enabled and spec.devicePlugin.enabled
    assert spec.nodeStatusExporter.enabled and spec.gfd.enabled and not spec.migManager.enabled
    assert spec.operator.cleanupCRD
    job = next(d for d in docs if d["metadata"]["name"] == "amd-gpu-operator-cleanup-crd")
    assert job["metadata"]["annotations"]["helm.sh/hook"] == "pre-delete"
    assert job["spec"]["template"]["spec"]["containers"][0]["args"] == ["cleanup-crd"]


def test_cleanup_hook_absent_by_default():
    docs = H.render_chart()
    assert not any(d["metadata"]["name"] == "amd-gpu-operator-cleanup-crd" for d in docs)


def test_namespace_and_release_flow_into_objects():
    docs = H.render_chart(release_name="rel", namespace="gpu-operator-resources")
    dep = next(d for d in docs if d["kind"] == "Deployment")
    assert dep["metadata"]["namespace"] == "gpu-operator-resources"
    assert dep["metadata"]["labels"]["app.kubernetes.io/instance"] == "rel"
    assert dep["spec"]["template"]["spec"]["containers"][0]["args"][:3] == ["operator", "--namespace",
                                                                            "gpu-operator-resources"]
    crb = next(d for d in docs if d["kind"] == "ClusterRoleBinding")
    assert crb["subjects"][0]["namespace"] == "gpu-operator-resources"


def test_overrides_reach_the_cluster_policy():
    docs = H.render_chart(set_flags=["devicePlugin.partitionStrategy=mixed", "dcgmExporter.port=9500",
                                     "validator.workload.gemmN=8192", "migManager.enabled=true"])
    cp = next(d for d in docs if d["kind"] == "ClusterPolicy")
    s = ClusterPolicySpec.model_validate(cp["spec"])
    assert s.devicePlugin.partitionStrategy == "mixed" and s.dcgmExporter.port == 9500
    assert s.validator.workload.gemmN == 8192 and s.migManager.enabled


@pytest.mark.parametrize("flags", [
    [],
    ["sandboxWorkloads.enabled=true", "sandboxWorkloads.defaultWorkload=vm-passthrough", "vfioManager.enabled=true"],
    ["draDriver.enabled=true", "devicePlugin.enabled=false", "driver.rdma.enabled=true", "psa.enabled=true"],
])
def test_every_spec_section_reaches_the_cluster_policy(flags):
    """The chart's ClusterPolicy carries every section of the spec: what
    `helm install --set ...` sets is what the operator reconciles (the
    simulated cluster builds the CR from the values directly)."""
    from amdgpu_operator.api.clusterpolicy import ClusterPolicySpec as S

    docs = H.render_chart(set_flags=REFERENCE_SET_FLAGS + flags)
    cp = next(d for d in docs if d["kind"] == "ClusterPolicy")
    assert set(cp["spec"]) >= set(S.model_fields), set(S.model_fields) - set(cp["spec"])
    rendered = S.model_validate(cp["spec"]).model_dump()
    assert rendered == spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS + flags)).model_dump()


def test_crd_schema_accepts_rendered_spec_keys():
    crd = H.load_crd()
    props = crd["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"]["properties"]
    for key in ("driver", "toolkit", "devicePlugin", "nodeStatusExporter", "gfd", "migManager", "operator",
                "dcgmExporter", "validator", "nfd", "daemonsets"):
        assert key in props, key
    assert props["driver"]["properties"]["enabled"]["type"] == "boolean"
    assert "$ref" not in yaml.safe_dump(crd)


def test_values_aliases():
    assert spec_from_values({"partitionManager": {"enabled": True}}).migManager.enabled
    assert spec_from_values({"metricsExporter": {"port": 1}}).dcgmExporter.port == 1
    with pytest.raises(Exception):
        spec_from_values({"metricsExporter": {}, "dcgmExporter": {}})
    assert parse_set_flags(["a.b=1", "a.c=true", "d=x", "e=1.5"]) == {"a": {"b": 1, "c": True}, "d": "x", "e": 1.5}


def test_template_engine_subset(tmp_path):
    chart = tmp_path / "c"
    (chart / "templates").mkdir(parents=True)
    (chart / "Chart.yaml").write_text("name: c\nversion: 1.0.0\nappVersion: '2'\n")
    (chart / "templates" / "_h.tpl").write_text('{{- define "n" -}}{{ .Values.x | default "dflt" }}{{- end -}}')
    (chart / "templates" / "a.yaml").write_text(
        "a: {{ include \"n\" . }}\n"
        "{{- if .Values.flag }}\nb: yes\n{{- else if .Values.other }}\nb: other\n{{- else }}\nb: no\n{{- end }}\n"
        "c: {{ .Values.s | quote }}\n"
        "d:{{- toYaml .Values.m | nindent 2 }}\n"
        "{{- range .Values.l }}\n- {{ . }}\n{{- end }}\n"
        "e: {{ not .Values.flag }}\n")
    out = H.Renderer(str(chart), {"flag": False, "other": True, "s": 'q"x', "m": {"k": [1, 2]}, "l": [7, 8]}).render()
    text = out["a.yaml"]
    assert "a: dflt" in text and "b: other" in text and 'c: "q\\"x"' in text
    assert "d:\n  k:\n  - 1\n  - 2" in text and "- 7\n- 8" in text and "e: true" in text


@pytest.mark.parametrize("flags", [
    [],
    ["draDriver.enabled=true", "devicePlugin.enabled=false", "driver.rdma.enabled=true", "migManager.enabled=true",
     "sandboxWorkloads.enabled=true", "dcgmExporter.serviceMonitor.enabled=true", "psa.enabled=true"],
    ["daemonsets.inContainerGates=false", "validator.workload.prespawn=false", "driver.usePrecompiled=true"],
])
def test_every_object_passes_apiserver_validation(flags):
    """What kube-apiserver would reject (kube/validation.py): every object the
    chart renders and every object each operator state builds."""
    from amdgpu_operator.controller import manifests as M
    from amdgpu_operator.kube.validation import validate

    objs = H.render_chart(set_flags=REFERENCE_SET_FLAGS + flags)
    spec = spec_from_values(parse_set_flags(REFERENCE_SET_FLAGS + flags))
    for builder in M.STATE_BUILDERS.values():
        objs += builder(spec, "gpu-operator-resources", None)
    objs += M.state_driver(spec, "gpu-operator-resources", None, kernel="6.8.0-45-generic")
    bad = {f"{o['kind']}/{o['metadata']['name']}": validate(o) for o in objs if validate(o)}
    assert not bad, bad
    assert len(objs) > 30


def test_validation_catches_what_the_apiserver_rejects():
    from amdgpu_operator.kube.fakeapi import ApiError, FakeApiServer
    from amdgpu_operator.kube.validation import install, validate

    ds = {"apiVersion": "apps/v1", "kind": "DaemonSet",
          "metadata": {"name": "x", "namespace": "default", "labels": {"amd.com/gpu.xgmi.hive": "a" * 64}},
          "spec": {"selector": {"matchLabels": {"app": "x"}},
                   "template": {"metadata": {"labels": {"app": "y"}},
                                "spec": {"containers": [{"name": "Main", "image": "i",
                                                         "ports": [{"name": "metrics-exporter-port", "containerPort": 9400}],
                                                         "volumeMounts": [{"name": "gone", "mountPath": "/x"}],
                                                         "env": [{"name": "1BAD", "value": "v"}]}],
                                         "volumes": [{"name": "h", "hostPath": {"path": "/h", "type": "Dir"}}],
                                         "tolerations": [{"key": "k", "operator": "Exists", "value": "v"}]}}}}
    errs = " | ".join(validate(ds))
    for want in ("not a valid label value", "do not match spec.selector", "'Main': not a DNS-1123 label",
                 "not a valid port name", "no volume of that name", "not a valid environment variable name",
                 "hostPath.type 'Dir'", "operator Exists takes no value"):
        assert want in errs, (want, errs)
    api = FakeApiServer()
    install(api)
    with pytest.raises(ApiError) as e:
        api.create(ds)
    assert e.value.code == 422


@pytest.mark.parametrize("flags", [
    [],
    ["draDriver.enabled=true", "devicePlugin.enabled=false", "driver.rdma.enabled=true", "migManager.enabled=true",
     "sandboxWorkloads.enabled=true", "daemonsets.maxUnavailable=25%", "validator.workload.gemmN=8192"],
])
def test_rendered_cluster_policy_matches_the_crd_schema(flags):
    """The CR `helm install` creates passes the CRD's structural schema
    (types, enums, no field the schema would prune)."""
    from amdgpu_operator.kube.validation import schema_errors

    docs = H.render_chart(set_flags=REFERENCE_SET_FLAGS + flags)
    cp = next(d for d in docs if d["kind"] == "ClusterPolicy")
    crd = next(d for d in docs if d["kind"] == "CustomResourceDefinition" and d["spec"]["names"]["kind"] == "ClusterPolicy")
    schema = crd["spec"]["versions"][0]["schema"]["openAPIV3Schema"]
    assert not schema_errors({k: v for k, v in cp.items() if k in ("spec",)}, {
        "type": "object", "properties": {"spec": schema["properties"]["spec"]}}), cp["spec"]
