"""Annotation protocol: exact reference grammar (pkg/gpu/annotation_test.go:316-449 behaviour)."""
import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.models import annotation as ann
from walkai_nos_amd.models.device import DeviceList, GpuDevice


@pytest.mark.parametrize("key,value", [
    ("", ""),
    ("nos.nebuly.com/foo", "1"),
    (api.ANNOTATION_GPU_STATUS_PREFIX + "foo", "1"),
    ("nos.nebuly.com/status-gpu-0-cpx_nps1-free", "foo"),
    ("nos.nebuly.com/status-gpu-foo-cpx_nps1-free", "1"),
    ("nos.nebuly.com/status-gpu-0-cpx_nps1-foo", "1"),
    ("nos.nebuly.com/status-gpu-0-cpx-nps1-free", "1"),  # a '-' inside a profile breaks the 5-part split
])
def test_parse_status_annotation_errors(key, value):
    with pytest.raises(ValueError):
        ann.parse_status_annotation(key, value)


def test_parse_status_annotation_valid_and_case_insensitive_status():
    a = ann.parse_status_annotation("nos.nebuly.com/status-gpu-1-cpx_nps1-used", "3")
    assert a == ann.StatusAnnotation(profile="cpx_nps1", index=1, status="used", quantity=3)
    b = ann.parse_status_annotation("nos.nebuly.com/status-gpu-2-1g.10gb-FREE", "1")
    assert b.status == "free" and b.profile == "1g.10gb"
    assert a.key == "nos.nebuly.com/status-gpu-1-cpx_nps1-used" and a.value() == "3"


@pytest.mark.parametrize("key,value", [
    ("", ""),
    ("nos.nebuly.com/foo", "1"),
    (api.ANNOTATION_GPU_SPEC_PREFIX + "foo", "1"),
    ("nos.nebuly.com/spec-gpu-0-spx_nps1", "foo"),
    ("nos.nebuly.com/spec-gpu-x-spx_nps1", "1"),
])
def test_parse_spec_annotation_errors(key, value):
    with pytest.raises(ValueError):
        ann.parse_spec_annotation(key, value)


def test_parse_spec_annotation_valid():
    a = ann.parse_spec_annotation("nos.nebuly.com/spec-gpu-1-cpx_nps1", "8")
    assert a == ann.SpecAnnotation(profile="cpx_nps1", index=1, quantity=8)
    assert a.key == "nos.nebuly.com/spec-gpu-1-cpx_nps1"


def test_parse_node_annotations_ignores_garbage():
    status, spec = ann.parse_node_annotations({
        "nos.nebuly.com/spec-gpu-0-cpx_nps1": "8",
        "nos.nebuly.com/spec-gpu-1-spx_nps1": "1",
        "nos.nebuly.com/status-gpu-0-cpx_nps1-used": "3",
        "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "5",
        "nos.nebuly.com/status-gpu-0-bad": "1",
        "nos.nebuly.com/spec-partitioning-plan": "123",
        "other/annotation": "x",
    })
    assert [a.index for a in spec] == [0, 1]
    assert {(a.profile, a.status, a.quantity) for a in status} == {("cpx_nps1", "used", 3), ("cpx_nps1", "free", 5)}


def test_spec_matches_status():
    spec = [ann.SpecAnnotation("cpx_nps1", 0, 8)]
    status = [ann.StatusAnnotation("cpx_nps1", 0, "used", 3), ann.StatusAnnotation("cpx_nps1", 0, "free", 5)]
    assert ann.spec_matches_status(spec, status)
    assert not ann.spec_matches_status(spec, status[:1])
    assert not ann.spec_matches_status(spec + [ann.SpecAnnotation("spx_nps1", 1, 1)], status)
    assert ann.spec_matches_status([], [])


def test_status_annotation_list_equality_is_unordered():
    a = [ann.StatusAnnotation("cpx_nps1", 0, "used", 3), ann.StatusAnnotation("cpx_nps1", 0, "free", 5)]
    assert ann.annotations_equal(a, list(reversed(a)))
    assert not ann.annotations_equal(a, a[:1])


def test_devices_as_status_annotation_groups_and_filters():
    from walkai_nos_amd.models.xcp.profile import extract_profile_name
    devs = DeviceList([
        GpuDevice("amd.com/cpx_nps1", "a/xcp0", "used", 0),
        GpuDevice("amd.com/cpx_nps1", "a/xcp1", "free", 0),
        GpuDevice("amd.com/cpx_nps1", "a/xcp2", "free", 0),
        GpuDevice("amd.com/spx_nps1", "b/xcp0", "free", 1),
        GpuDevice("amd.com/gpu", "c", "used", 2),  # not a partition resource -> excluded
    ])
    out = devs.as_status_annotation(extract_profile_name)
    got = {(a.index, a.profile, a.status, a.quantity) for a in out}
    assert got == {(0, "cpx_nps1", "used", 1), (0, "cpx_nps1", "free", 2), (1, "spx_nps1", "free", 1)}
