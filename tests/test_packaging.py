"""Packaging: kustomize manifests, Helm chart, CRDs, ComponentConfigs, console scripts, demo."""
import glob
import json
import importlib
import os
import re
import sys

import pytest
import yaml

from walkai_nos_amd.api.config import (CapacitySchedulingArgs, GpuAgentConfig, GpuPartitionerConfig, MigAgentConfig,
                                       load_config)
from walkai_nos_amd.models.xcp.known_configs import load_known_geometries

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _p(*a):
    return os.path.join(ROOT, *a)


def test_every_plain_yaml_parses():
    files = [f for pat in ("config/**/*.yaml", "demos/**/*.yaml", "hack/**/*.yaml", ".github/**/*.yml",
                           "helm-charts/nos/values.yaml", "helm-charts/nos/Chart.yaml", "helm-charts/nos/crds/*.yaml")
             for f in glob.glob(_p(pat), recursive=True)]
    assert len(files) > 20
    for f in files:
        docs = [d for d in yaml.safe_load_all(open(f)) if d is not None]
        assert docs, f


def test_crds_match_between_kustomize_and_helm():
    for f in glob.glob(_p("config/crd/bases/*.yaml")):
        helm = _p("helm-charts/nos/crds", os.path.basename(f))
        assert open(f).read() == open(helm).read()
    kinds = {yaml.safe_load(open(f))["spec"]["names"]["kind"] for f in glob.glob(_p("config/crd/bases/*.yaml"))}
    assert kinds == {"ElasticQuota", "CompositeElasticQuota"}


def test_crd_schema_covers_quota_model_fields():
    eq = yaml.safe_load(open(_p("config/crd/bases/nos.nebuly.com_elasticquotas.yaml")))
    v = eq["spec"]["versions"][0]
    props = v["schema"]["openAPIV3Schema"]["properties"]
    assert set(props["spec"]["properties"]) == {"min", "max"}
    assert props["spec"]["required"] == ["min"]
    assert "used" in props["status"]["properties"]
    assert v["subresources"] == {"status": {}}
    ceq = yaml.safe_load(open(_p("config/crd/bases/nos.nebuly.com_compositeelasticquotas.yaml")))
    cprops = ceq["spec"]["versions"][0]["schema"]["openAPIV3Schema"]["properties"]["spec"]
    assert set(cprops["required"]) == {"namespaces", "min"}


def test_component_configs_in_manifests_load_and_validate():
    assert isinstance(load_config(open(_p("config/gpupartitioner/gpu_partitioner_config.yaml")).read()),
                      GpuPartitionerConfig)
    assert isinstance(load_config(open(_p("config/partitionagent/partition_agent_config.yaml")).read()),
                      MigAgentConfig)
    assert isinstance(load_config(open(_p("config/sliceagent/slice_agent_config.yaml")).read()), GpuAgentConfig)
    args = load_config(open(_p("config/quota/scheduler_config.yaml")).read())
    assert isinstance(args, CapacitySchedulingArgs) and args.nvidiaGpuResourceMemoryGB == 288
    specs = load_known_geometries(open(_p("config/gpupartitioner/known_geometries.yaml")).read())
    assert specs["MI355X"].allowed_geometries


def test_helm_known_geometries_value_loads():
    values = yaml.safe_load(open(_p("helm-charts/nos/values.yaml")))
    specs = load_known_geometries(yaml.safe_dump(values["gpuPartitioner"]["knownGeometries"]))
    assert {"MI355X", "MI350X", "MI325X", "MI300X"} <= set(specs)
    assert values["nvidiaGpuResourceMemoryGB"] == 288


def _flatten(d, prefix=""):
    out = set()
    for k, v in d.items():
        key = f"{prefix}.{k}" if prefix else k
        out.add(key)
        if isinstance(v, dict):
            out |= _flatten(v, key)
    return out


def test_helm_templates_only_reference_defined_values():
    values = _flatten(yaml.safe_load(open(_p("helm-charts/nos/values.yaml"))))
    missing = []
    for f in glob.glob(_p("helm-charts/nos/templates/**/*.yaml"), recursive=True) + \
            glob.glob(_p("helm-charts/nos/templates/*.tpl")):
        for ref in re.findall(r"\.Values\.([A-Za-z0-9_.]+)", open(f).read()):
            if ref not in values:
                missing.append((os.path.relpath(f, ROOT), ref))
    assert not missing, missing


def test_helm_template_blocks_balanced():
    for f in glob.glob(_p("helm-charts/nos/templates/**/*.yaml"), recursive=True):
        s = open(f).read()
        opens = len(re.findall(r"{{-?\s*(if|with|range|define)\b", s))
        ends = len(re.findall(r"{{-?\s*end\s*-?}}", s))
        assert opens == ends, f


def test_console_scripts_resolve():
    try:
        import tomllib
    except ImportError:  # py3.10
        import tomli as tomllib
    proj = tomllib.load(open(_p("pyproject.toml"), "rb"))
    scripts = proj["project"]["scripts"]
    assert len(scripts) >= 8
    for name, target in scripts.items():
        mod, fn = target.split(":")
        assert callable(getattr(importlib.import_module(mod), fn)), name


def test_manifests_reference_existing_entry_points():
    try:
        import tomllib
    except ImportError:
        import tomli as tomllib
    scripts = set(tomllib.load(open(_p("pyproject.toml"), "rb"))["project"]["scripts"])
    used = set()
    for f in glob.glob(_p("config/**/*.yaml"), recursive=True) + \
            glob.glob(_p("helm-charts/nos/templates/**/*.yaml"), recursive=True):
        used |= set(re.findall(r"command: \[(nos-[a-z]+)\]", open(f).read()))
    assert used and used <= scripts, used - scripts


def test_demo_client_uses_safe_loaders_only():
    src = open(_p("demos/gpu-sharing-comparison/client/main.py")).read()
    assert "allow_pickle=False" in src and "safetensors" in src
    assert "pickle.load" not in src and "weights_only=False" not in src
    compile(src, "main.py", "exec")


@pytest.mark.parametrize("overlay,resource", [("xcp", "amd.com/cpx_nps1"), ("cumask", "amd.com/gpu-32cu.36gb"),
                                              ("time-slicing", "amd.com/gpu")])
def test_demo_overlays_request_valid_resources(overlay, resource):
    from walkai_nos_amd import constant
    k = yaml.safe_load(open(_p("demos/gpu-sharing-comparison/manifests/overlays", overlay, "kustomization.yaml")))
    assert resource in k["patches"][0]["patch"]
    assert (resource == constant.RESOURCE_AMD_GPU or constant.RESOURCE_XCP_REGEX.match(resource)
            or constant.RESOURCE_SLICE_REGEX.match(resource))


def test_every_source_file_has_a_header():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "hack", "check_headers.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout


def test_helm_install_guards_and_telemetry_identity():
    val = open(_p("helm-charts/nos/templates/validation.yaml")).read()
    assert 'eq .Release.Namespace "default"' in val and "fail" in val
    inst = open(_p("helm-charts/nos/templates/telemetry/installation.yaml")).read()
    # the UUID is looked up and reused, kept on uninstall, and nodes are looked up for the payload
    assert 'lookup "v1" "ConfigMap"' in inst and "helm.sh/resource-policy: keep" in inst
    assert 'lookup "v1" "Node"' in inst and "node.kubernetes.io/instance-type" in inst
    for key in ("installationUUID", "nodes:", "chartValues:", "nosGpuPartitioner", "nosScheduler", "nosOperator"):
        assert key in inst
    job = open(_p("helm-charts/nos/templates/telemetry/job.yaml")).read()
    assert "nos-telemetry-metrics" in job and "uuidv4" not in job


def test_metrics_behind_kube_rbac_proxy_and_optional_service_monitor():
    dep = open(_p("helm-charts/nos/templates/gpu-partitioner/deployment.yaml")).read()
    assert "kube-rbac-proxy" in dep and "--upstream=http://127.0.0.1:8080/" in dep
    cm = open(_p("helm-charts/nos/templates/gpu-partitioner/configmap.yaml")).read()
    assert '"127.0.0.1:8080"' in cm
    met = open(_p("helm-charts/nos/templates/gpu-partitioner/metrics.yaml")).read()
    assert "tokenreviews" in met and "subjectaccessreviews" in met and "nonResourceURLs: [/metrics]" in met
    assert "kind: ServiceMonitor" in met and ".Values.gpuPartitioner.metrics.serviceMonitor.enabled" in met
    k = yaml.safe_load(open(_p("config/gpupartitioner/kustomization.yaml")))
    assert "auth_proxy.yaml" in k["resources"] and k["patches"][0]["path"] == "auth_proxy_patch.yaml"
    cfg = yaml.safe_load(open(_p("config/gpupartitioner/gpu_partitioner_config.yaml")))
    assert cfg["metricsBindAddress"] == "127.0.0.1:8080"
    mon = yaml.safe_load(open(_p("config/prometheus/monitor.yaml")))
    assert mon["kind"] == "ServiceMonitor" and mon["spec"]["endpoints"][0]["port"] == "https"


def test_chart_readme_is_generated_from_values():
    """helm-charts/nos/README.md is hack/helm_docs.py's rendering of values.yaml (helm-docs'
    convention, ref Makefile:110-111): every value has a row, and every row is documented."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, _p("hack/helm_docs.py"), "--check"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    sys.path.insert(0, _p("hack"))
    import helm_docs
    text = open(_p("helm-charts/nos/values.yaml")).read()
    import yaml
    rows = helm_docs.rows(yaml.safe_load(text), helm_docs.key_comments(text))
    keys = {r[0] for r in rows}
    assert {"gpuPartitioner.planningPolicy", "partitionAgent.commitBarrier", "scheduler.name",
            "operator.resources", "image.tag"} <= keys
    assert all(r[3] for r in rows), [r[0] for r in rows if not r[3]]


def test_lint_is_clean_and_fails_on_errors(tmp_path):
    import subprocess
    import sys
    r = subprocess.run([sys.executable, _p("hack/lint.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    bad = tmp_path / "bad.py"
    bad.write_text("import os\n\ntry:\n    pass\nexcept:\n    pass\n")
    sys.path.insert(0, _p("hack"))
    import lint
    errs = lint.check_file(str(bad))
    assert any("unused import os" in e for e in errs) and any("bare except" in e for e in errs)


def test_native_libraries_are_stamped_with_their_source_hash():
    from walkai_nos_amd.ops import build as b
    from walkai_nos_amd.ops import native
    for t in b.TARGETS:
        if native.available(t.name):
            assert b.verify(t.name) == t.source_hash()
    t = b.target("libnos_probe.so")
    assert t.source_hash() != b.Target("x", ["probe.hip"], "hipcc", flags=["-DX"]).source_hash()


def test_per_source_flags_build_their_own_object():
    # csrc/attn_wide.hip is compiled alone with its code-generation options and linked first (hipcc
    # marks every .hip source `-x hip`, which would claim an object listed after it); its flags are
    # part of the stamp
    from walkai_nos_amd.ops import build as b
    t = b.target("libnos_kernels.so")
    cmds = t.commands()
    assert len(cmds) == 2
    obj_cmd, link = cmds
    assert "-c" in obj_cmd and obj_cmd[obj_cmd.index("-c") + 1].endswith("attn_wide.hip")
    assert "-amdgpu-mfma-vgpr-form=1" in obj_cmd and "-amdgpu-mfma-vgpr-form=1" not in link
    srcs = [x for x in link if x.endswith((".hip", ".o"))]
    assert srcs[0].endswith("attn_wide.hip.o") and all(x.endswith(".hip") for x in srcs[1:])
    assert "-shared" in link and "-shared" not in obj_cmd
    plain = b.Target(t.name, t.sources, t.compiler)
    assert plain.source_hash() != t.source_hash()


# -- the chart rendered (hack/helmlite.py: a Go-template subset interpreter; no helm binary here) --
def _chart(values=None, namespace="nos-system", lookup=None):
    import sys
    sys.path.insert(0, _p("hack"))
    import helmlite
    return helmlite, helmlite.Chart(_p("helm-charts/nos"), values or {}, namespace=namespace, lookup=lookup)


def test_helm_chart_renders_to_valid_objects():
    from walkai_nos_amd.api.config import load_config
    _, chart = _chart()
    objs = chart.objects()
    kinds = {o["kind"] for o in objs}
    assert {"Deployment", "DaemonSet", "ConfigMap", "ClusterRole", "ClusterRoleBinding", "ServiceAccount",
            "Service", "Job"} <= kinds
    for o in objs:
        assert o.get("apiVersion") and o["metadata"].get("name"), o
        if o["kind"] not in ("ClusterRole", "ClusterRoleBinding"):
            assert o["metadata"]["namespace"] == "nos-system", o["metadata"]
    deps = {o["metadata"]["name"]: o for o in objs if o["kind"] in ("Deployment", "DaemonSet")}
    gp = deps["nos-gpu-partitioner"]["spec"]["template"]["spec"]
    assert [c["name"] for c in gp["containers"]] == ["gpu-partitioner", "kube-rbac-proxy"]
    for d in deps.values():
        for c in d["spec"]["template"]["spec"]["containers"]:
            assert c["image"] and "<no value>" not in json.dumps(c)
    cms = {o["metadata"]["name"]: o for o in objs if o["kind"] == "ConfigMap"}
    cfg = load_config(cms["nos-gpu-partitioner-config"]["data"]["gpu_partitioner_config.yaml"])
    assert cfg.planningPolicy == "pack" and cfg.metricsBindAddress == "127.0.0.1:8080"
    assert cfg.defaultXcpLayout == "slices" and cfg.sharedSliceSkipCounts == [5, 7]
    assert "known_geometries.yaml" in cms["nos-gpu-partitioner-config"]["data"]


def test_helm_chart_passes_pack_knobs_to_the_partitioner_config():
    from walkai_nos_amd.api.config import load_config
    _, chart = _chart({"gpuPartitioner": {"packing": {"minFill": 0.25, "drainGainAfterSeconds": 120}}})
    cms = {o["metadata"]["name"]: o for o in chart.objects() if o["kind"] == "ConfigMap"}
    cfg = load_config(cms["nos-gpu-partitioner-config"]["data"]["gpu_partitioner_config.yaml"])
    p = cfg.pack_params()
    assert (p.min_fill, p.drain_gain_after) == (0.25, 120.0)


def test_helm_chart_refuses_the_default_namespace():
    helmlite, chart = _chart(namespace="default")
    with pytest.raises(helmlite.Fail):
        chart.render()


def test_helm_telemetry_reuses_the_installation_uuid_and_reports_nodes():
    from walkai_nos_amd.exporters.telemetry import Metrics
    node = {"metadata": {"name": "gpu-1", "labels": {"amd.com/gpu.product-name": "MI355X", "kubernetes.io/os": "linux",
                                                     "node.kubernetes.io/instance-type": "mi355x-8"}},
            "status": {"capacity": {"amd.com/gpu": "8"}, "nodeInfo": {"kubeletVersion": "v1.30.0"}}}

    def lookup(api, kind, ns, name):
        if kind == "ConfigMap" and name == "nos-installation-info":
            return {"data": {"installationUUID": "11111111-2222-3333-4444-555555555555"}}
        if kind == "Node":
            return {"items": [node]}
        return {}
    _, chart = _chart(lookup=lookup)
    cms = {o["metadata"]["name"]: o for o in chart.objects() if o["kind"] == "ConfigMap"}
    assert cms["nos-installation-info"]["data"]["installationUUID"] == "11111111-2222-3333-4444-555555555555"
    assert cms["nos-installation-info"]["metadata"]["annotations"]["helm.sh/resource-policy"] == "keep"
    m = Metrics.from_yaml(cms["nos-telemetry-metrics"]["data"]["metrics.yaml"])
    assert m.installationUUID == "11111111-2222-3333-4444-555555555555"
    assert m.nodes[0].name == "gpu-1" and "kubernetes.io/os" not in m.nodes[0].labels
    assert m.nodes[0].labels["node.kubernetes.io/instance-type"] == "mi355x-8"
    assert m.components.nosGpuPartitioner is True
    # a first install generates a fresh UUID
    _, fresh = _chart()
    u = {o["metadata"]["name"]: o for o in fresh.objects()}["nos-installation-info"]["data"]["installationUUID"]
    assert len(u) == 36 and u != "11111111-2222-3333-4444-555555555555"


def test_helm_metrics_exposure_toggles():
    _, plain = _chart({"gpuPartitioner": {"metrics": {"authProxy": {"enabled": False},
                                                      "serviceMonitor": {"enabled": True}}}})
    objs = plain.objects()
    dep = next(o for o in objs if o["kind"] == "Deployment" and o["metadata"]["name"] == "nos-gpu-partitioner")
    assert [c["name"] for c in dep["spec"]["template"]["spec"]["containers"]] == ["gpu-partitioner"]
    svc = next(o for o in objs if o["kind"] == "Service" and o["metadata"]["name"] == "nos-gpu-partitioner-metrics")
    assert svc["spec"]["ports"][0]["port"] == 8080
    sm = next(o for o in objs if o["kind"] == "ServiceMonitor")
    assert sm["spec"]["endpoints"][0]["port"] == "metrics"
    assert not any(o["kind"] == "ClusterRole" and o["metadata"]["name"] == "nos-metrics-reader" for o in objs)
    _, off = _chart({"shareTelemetry": False, "operator": {"enabled": False}})
    names = {o["metadata"]["name"] for o in off.objects()}
    assert "nos-telemetry" not in names and "nos-installation-info" not in names
