"""The bench's cluster-time model on CPU (no GPU, ``control_only``): the window in quanta, pod
start-up charged inside a pod's lifetime, and idle GPU time accounted to exactly one cause."""
from __future__ import annotations

import pytest

from walkai_nos_amd.bench_core import IDLE_CAUSES, BenchConfig, control_only, pod_start_sensitivity


def _cfg(**kw):
    base = dict(gpus=1, steps=10, warmup=2, preroll=20, seed=7, data_plane=False, layout="slices")
    base.update(kw)
    return BenchConfig(**base)


def test_a_driver_step_spans_quanta_per_step_quanta():
    c = BenchConfig(steps=20, warmup=5)
    assert (c.quanta_per_step, c.window_quanta, c.warmup_quanta) == (2, 40, 10)
    assert c.window_quanta / c.mean_lifetime_quanta == 10.0
    c1 = BenchConfig(steps=20, warmup=5, quanta_per_step=1)
    assert (c1.window_quanta, c1.warmup_quanta) == (20, 5)


@pytest.mark.parametrize("layout", ["slices", "partitions"])
def test_idle_time_is_accounted_to_one_cause(layout):
    c = _cfg(layout=layout)
    r = control_only(c, c.warmup_quanta + c.window_quanta, skip=c.warmup_quanta)
    idle = r["idle"]
    assert set(idle["by_cause_pct"]) == set(IDLE_CAUSES)
    assert idle["gpu_quanta"] == c.window_quanta * c.gpus
    # allocated (incl. flip darkness) + every idle cause = the window's GPU time
    total = r["util_incl_outage_pct"] + sum(v for k, v in idle["by_cause_pct"].items() if k != "flip_outage")
    assert total == pytest.approx(100.0, abs=0.5)
    if layout == "slices":
        assert idle["by_cause_pct"]["flip_outage"] == 0.0 and r["flips"] == 0


def test_pod_start_is_charged_inside_the_lifetime():
    """A bound pod holds its slice and serves nothing while it starts: allocation is the same with or
    without start-up (pods leave when their lifetime, start-up included, is over), the modelled
    inferences drop as the start-up grows."""
    rows = {}
    for ps in (0.0, 6.0, 30.0):
        c = _cfg(pod_start_s=ps)
        rows[ps] = control_only(c, c.warmup_quanta + c.window_quanta, skip=c.warmup_quanta)
    assert rows[0.0]["util_pct"] == rows[6.0]["util_pct"] == rows[30.0]["util_pct"]
    assert rows[0.0]["inf_per_s_model"] > rows[6.0]["inf_per_s_model"] > rows[30.0]["inf_per_s_model"]


def test_pod_start_sensitivity_rows():
    c = _cfg(pod_start_s=3.0)
    s = pod_start_sensitivity(c)
    assert list(s) == ["0s", "3s", "6s", "12s"]
    v = [row["inf_per_s_model"] for row in s.values()]
    assert v == sorted(v, reverse=True) and len({row["util_pct"] for row in s.values()}) == 1
