"""Geometry selection (Appendix B.1-B.3) and the MI355X compute-partition table.

The scored search is exercised against the reference's own test vectors
(pkg/gpu/mig/gpu_test.go:297-488, 520-596; node_test.go:415-440) by loading an A100-80GB-like
MIG table into the generic :class:`PartitionedGPU` — behaviour parity of the algorithm itself —
and then against the production MI355X table.
"""
import pytest

from walkai_nos_amd.models.geometry import geometry_id, get_fewest_slices_geometry
from walkai_nos_amd.models.partitioned import PartitionedGPU, PartitionedNode
from walkai_nos_amd.models.xcp import known_configs as kc
from walkai_nos_amd.models.xcp.profile import XcpProfile, extract_profile_name, parse_profile, smaller_than

from walkai_nos_amd.models import mig  # noqa: E402

A100_80_BUILTIN = mig.KNOWN_GEOMETRIES[mig.A100_PCIE_80GB]
# the table TestGPU__UpdateGeometryFor installs with SetKnownGeometries before its cases
# (ref pkg/gpu/mig/gpu_test.go:297-317)
A100_80 = [{"1g.10gb": 7}, {"1g.10gb": 5, "2g.20gb": 1}, {"1g.10gb": 3, "2g.20gb": 2}, {"1g.10gb": 1, "2g.20gb": 3},
           {"1g.10gb": 2, "2g.20gb": 1, "3g.40gb": 1}, {"2g.20gb": 2, "3g.40gb": 1}, {"1g.10gb": 3, "3g.40gb": 1},
           {"1g.10gb": 1, "2g.20gb": 1, "3g.40gb": 1}, {"3g.40gb": 2}, {"1g.10gb": 3, "4g.40gb": 1},
           {"1g.10gb": 1, "2g.20gb": 1, "4g.40gb": 1}, {"7g.79gb": 1}]
A100_40 = mig.KNOWN_GEOMETRIES[mig.A100_SXM4_40GB]
A30 = mig.KNOWN_GEOMETRIES[mig.A30]


def g(table, used=None, free=None, model="m"):
    return PartitionedGPU(model, 0, [dict(x) for x in table], dict(used or {}), dict(free or {}))


@pytest.mark.parametrize("gpu,required,expected,updated", [
    # empty requirement
    (g(A100_40, {"2g.20gb": 1}), {}, {"2g.20gb": 1}, False),
    # no geometry provides the profile
    (g(A100_40, {"2g.20gb": 1}), {"1g.10gb": 1}, {"2g.20gb": 1}, False),
    # the only providing geometry would delete used devices
    (g(A100_80, {"2g.20gb": 1}), {"7g.79gb": 1}, {"2g.20gb": 1}, False),
    # current geometry already provides the profiles
    (g(A100_40, {"2g.20gb": 1}, {"2g.20gb": 2}), {"2g.20gb": 2}, {"2g.20gb": 3}, False),
    # the geometry providing the most required profiles wins
    (g(A100_80, {"1g.10gb": 2}), {"1g.10gb": 6}, {"1g.10gb": 7}, True),
    # more of an already present profile
    (g(A100_80, {"3g.40gb": 1}, {"1g.10gb": 3}), {"3g.40gb": 1}, {"3g.40gb": 2}, True),
    # tie on provided -> more slices wins (minimal change)
    (g(A100_80, {}, {"1g.10gb": 7}), {"2g.20gb": 1}, {"1g.10gb": 5, "2g.20gb": 1}, True),
    # tie on provided and slices -> smallest L1 distance keeps existing profiles
    (g(A100_80, {}, {"1g.10gb": 1, "2g.20gb": 1, "4g.40gb": 1}), {"3g.40gb": 1},
     {"1g.10gb": 2, "2g.20gb": 1, "3g.40gb": 1}, True),
])
def test_update_geometry_for_reference_vectors(gpu, required, expected, updated):
    assert gpu.update_geometry_for(required) is updated
    assert gpu.geometry() == expected


def test_builtin_mig_tables_match_the_reference():
    # pkg/gpu/mig/known_configs.go:26-140: 4 A30 and 12 geometries per A100 model
    assert len(A30) == 4 and len(A100_40) == 12 and len(A100_80_BUILTIN) == 12
    assert {"1g.5gb": 7} in A100_40 and {"2g.10gb": 1, "1g.5gb": 5} in A100_40
    assert {"7g.79gb": 1} in A100_80_BUILTIN and {"4g.40gb": 1, "1g.10gb": 3} in A100_80_BUILTIN
    assert max(sum(geo.values()) for geo in A100_40) == 7  # the 7-pods-per-GPU density anchor


def test_apply_geometry_sets_free_and_drops_missing():
    x = g(A100_80, {"1g.10gb": 1}, {"2g.20gb": 2, "1g.10gb": 1})
    x.apply_geometry({"1g.10gb": 7})
    assert x.free == {"1g.10gb": 6} and x.used == {"1g.10gb": 1}
    with pytest.raises(ValueError):
        x.apply_geometry({"7g.79gb": 1})  # would delete a used device
    with pytest.raises(ValueError):
        x.apply_geometry({"1g.10gb": 6})  # not an allowed geometry


def test_init_geometry_reference_vectors():
    with pytest.raises(ValueError):
        g(A30, {"1g.5gb": 5}).init_geometry()
    x = g(A30)
    x.init_geometry()
    assert x.geometry() == {"4g.24gb": 1}
    y = g(A30, {}, {"1g.6gb": 1})
    y.init_geometry()
    assert y.geometry() == {"4g.24gb": 1}


def test_fewest_slices_first_in_list_wins_ties():
    assert get_fewest_slices_geometry([{"a": 2, "b": 1}, {"c": 3}, {"d": 1}]) == {"c": 3}
    assert get_fewest_slices_geometry([]) is None


def test_geometry_id_is_sorted_and_deterministic():
    assert geometry_id({"b": 1, "a": 2}) == "a:2, b:1, "
    assert geometry_id({"a": 2, "b": 1}) == geometry_id({"b": 1, "a": 2})


def test_node_greedy_reference_vector_two_a30():
    # node_test.go:415-440: two empty A30s, request 1g.6gb:3 -> only GPU 0 becomes 1g.6gb:4
    n = PartitionedNode("n", [PartitionedGPU("A30", 0, A30), PartitionedGPU("A30", 1, A30)])
    assert n.update_geometry_for({"1g.6gb": 3})
    assert n.gpus[0].geometry() == {"1g.6gb": 4}
    assert n.gpus[1].geometry() == {}


# -- MI355X table ----------------------------------------------------------------------------
def test_mi355x_allowed_geometries_are_homogeneous_per_nps():
    nps1 = kc.get_allowed_geometries("AMD_Instinct_MI355X", "nps1")
    assert nps1 == [{"spx_nps1": 1}, {"dpx_nps1": 2}, {"qpx_nps1": 4}, {"cpx_nps1": 8}]
    nps2 = kc.get_allowed_geometries("MI355X", "nps2")
    assert {next(iter(x)) for x in nps2} == {"dpx_nps2", "qpx_nps2", "cpx_nps2"}
    assert kc.get_allowed_geometries("unknown-gpu") is None
    assert kc.normalize_model("AMD Instinct MI355X") == "MI355X"


def test_mi355x_init_is_spx_and_flip_is_blocked_by_used_partitions():
    allowed = kc.get_allowed_geometries("MI355X", "nps1")
    x = PartitionedGPU("MI355X", 0, allowed)
    x.init_geometry()
    assert x.geometry() == {"spx_nps1": 1}
    assert x.update_geometry_for({"cpx_nps1": 3})
    assert x.geometry() == {"cpx_nps1": 8}
    x.add_pod({"cpx_nps1": 1})
    assert not x.update_geometry_for({"spx_nps1": 1})  # one used partition pins CPX
    assert x.geometry() == {"cpx_nps1": 8}


def test_fraction_weighted_scoring_prefers_capacity_over_pod_count():
    from walkai_nos_amd.models.xcp.node import fraction_weight
    allowed = kc.get_allowed_geometries("MI355X", "nps1")
    # pending: one whole-GPU pod and two 1/8 pods on an idle GPU
    a = PartitionedGPU("MI355X", 0, allowed)
    assert a.update_geometry_for({"spx_nps1": 1, "cpx_nps1": 2})  # reference score: 2 pods > 1 pod
    assert a.geometry() == {"cpx_nps1": 8}
    b = PartitionedGPU("MI355X", 0, allowed)
    assert b.update_geometry_for({"spx_nps1": 1, "cpx_nps1": 2}, fraction_weight)
    assert b.geometry() == {"spx_nps1": 1}  # 1.0 GPU of demand beats 0.25


def test_known_geometries_validation_and_yaml_roundtrip():
    with pytest.raises(ValueError):
        kc.validate_geometry({"cpx_nps1": 4})  # CPX always yields 8 partitions
    with pytest.raises(ValueError):
        kc.validate_geometry({"cpx_nps1": 8, "spx_nps1": 1})  # modes are homogeneous
    with pytest.raises(ValueError):
        kc.validate_geometry({"1g.10gb": 7})  # not an MI355X profile
    with pytest.raises(ValueError):
        kc.validate_geometry({})
    text = kc.dump_known_geometries()
    specs = kc.load_known_geometries(text)
    assert specs["MI355X"].memory_gb == 288 and specs["MI355X"].compute_units == 256
    custom = kc.load_known_geometries(
        "- models: [AMD_Instinct_MI355X]\n  allowedGeometries:\n    - spx_nps1: 1\n    - cpx_nps1: 8\n")
    kc.set_known_geometries(custom)
    assert kc.get_allowed_geometries("MI355X", "nps1") == [{"spx_nps1": 1}, {"cpx_nps1": 8}]
    with pytest.raises(ValueError):
        kc.load_known_geometries("- models: [X]\n  allowedGeometries:\n    - cpx_nps1: 3\n")


def test_profiles_total_order_and_resources():
    assert smaller_than("cpx_nps1", "qpx_nps1") and smaller_than("qpx_nps1", "dpx_nps1")
    assert smaller_than("dpx_nps1", "spx_nps1") and not smaller_than("spx_nps1", "spx_nps1")
    p = parse_profile("qpx_nps2")
    assert p == XcpProfile("qpx", "nps2") and p.partitions == 4 and p.cus() == 64 and p.memory_gb() == 72
    assert p.resource_name == "amd.com/qpx_nps2"
    assert extract_profile_name("amd.com/cpx_nps1") == "cpx_nps1"
    assert extract_profile_name("amd.com/gpu") is None
    with pytest.raises(ValueError):
        parse_profile("cpx-nps1")


def test_mig_parity_tables_and_helpers():
    assert mig.parse_profile("1g.10gb") == (1, 10) and mig.parse_profile("x") is None
    assert mig.extract_profile_name("nvidia.com/mig-3g.40gb") == "3g.40gb"
    assert mig.memory_gb("7g.79gb") == 79
    gpu = mig.new_gpu(mig.A100_PCIE_80GB, used={"1g.10gb": 1})
    assert gpu.update_geometry_for({"3g.40gb": 2}) and gpu.free.get("3g.40gb") == 1
