"""Infrastructure: kubelet PodResources gRPC (real unix socket), commit barriers (threads, and a
2-rank gloo process group), batcher, utilities, metrics, workload parity."""
import os
import tempfile
import threading

import pytest

from walkai_nos_amd.device.amdsmi import FakeAmdSmi
from walkai_nos_amd.device.partition_client import PartitionClient
from walkai_nos_amd.device.podresources import PodResourcesClient, PodResourcesServer
from walkai_nos_amd.parallel.barrier import LocalBarrier
from walkai_nos_amd.utils.batcher import Batcher
from walkai_nos_amd.utils.util import hash_fnv32a, local_endpoint, unordered_equal


def test_podresources_grpc_roundtrip_and_partition_client():
    smi = FakeAmdSmi(n_gpus=2)
    smi.set_compute_partition(1, "QPX")
    alloc = [(f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}", d.device_id) for d in smi.logical_devices()]
    used_id = alloc[2][1]  # first QPX partition of GPU 1
    with tempfile.TemporaryDirectory() as d:
        sock = os.path.join(d, "kubelet.sock")
        srv = PodResourcesServer(sock, used=lambda: [("w", "ns", [(alloc[2][0], [used_id])])],
                                 allocatable=lambda: [(r, [i]) for r, i in alloc]).start()
        try:
            c = PodResourcesClient(sock, timeout=5)
            used = c.get_used_devices()
            assert [(x.resource_name, x.device_id, x.status) for x in used] == [("amd.com/qpx_nps1", used_id, "used")]
            assert len(c.get_allocatable_devices()) == 5  # 1 SPX + 4 QPX
            devs = PartitionClient(c, smi).get_partition_devices()
            by = {(x.gpu_index, x.status) for x in devs}
            assert by == {(0, "free"), (1, "used"), (1, "free")}
            assert sum(1 for x in devs if x.gpu_index == 1 and x.is_free()) == 3
            c.close()
        finally:
            srv.stop()


def test_local_barrier_threads_all_or_nothing():
    b = LocalBarrier(3, timeout=5)
    results = []

    def voter(ok):
        results.append(b.vote(ok))

    ts = [threading.Thread(target=voter, args=(v,)) for v in (True, True, True)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert results == [True, True, True]
    results.clear()
    ts = [threading.Thread(target=voter, args=(v,)) for v in (True, False, True)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert results == [False, False, False]


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist

    from walkai_nos_amd.parallel.barrier import TorchBarrier
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        b = TorchBarrier()
        ok_all = b.vote(True)
        veto = b.vote(rank != 1)
        q.put((rank, ok_all, veto))
    finally:
        dist.destroy_process_group()


def test_torch_barrier_two_ranks_gloo():
    import multiprocessing as mp
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    [p.join(120) for p in ps]
    out = sorted(q.get(timeout=10) for _ in range(2))
    assert out == [(0, True, False), (1, True, False)]


def test_batcher_timeout_and_idle_windows():
    t = [0.0]
    b = Batcher(timeout_s=10, idle_s=3, clock=lambda: t[0])
    assert not b.add(1)  # not started -> dropped
    b.start()
    assert b.add(1)
    t[0] = 2
    b.add(2)
    t[0] = 4.9
    assert b.ready() is None
    t[0] = 5.0  # idle window (3 s after the last add) expired
    assert b.ready() == [1, 2]
    b.add(3)
    for k in range(1, 11):  # keep adding within the idle window; the 10 s timeout still fires
        t[0] = 5.0 + k
        b.add(k)
    assert b.ready() is not None
    assert b.flush() == []


def test_utils():
    assert unordered_equal([1, 2, 2], [2, 1, 2]) and not unordered_equal([1, 2], [1, 2, 2])
    assert unordered_equal([{"a": 1}, {"b": 2}], [{"b": 2}, {"a": 1}])
    assert hash_fnv32a("") == 0x811C9DC5 and hash_fnv32a("a") == 0xE40C292C
    assert local_endpoint("/tmp/x.sock") == "unix:///tmp/x.sock"


def test_metrics_render():
    from walkai_nos_amd.utils.metrics import Metrics
    m = Metrics()
    m.node_utilization.labels(node="n").set(87.5)
    m.probe_tflops_per_cu.labels(node="n", gpu="0", slice="cpx0", dtype="fp32").set(0.5)
    out = m.render().decode()
    assert 'nos_node_gpu_utilization_percent{node="n"} 87.5' in out
    assert "nos_probe_tflops_per_cu" in out


def test_yolos_matches_transformers_reference():
    torch = pytest.importorskip("torch")
    transformers = pytest.importorskip("transformers")
    from walkai_nos_amd.models.workload.yolos import YolosConfig, YolosSmall, demo_input
    cfg = transformers.YolosConfig(hidden_size=384, num_hidden_layers=2, num_attention_heads=6,
                                   intermediate_size=1536, image_size=[800, 1333], num_labels=91,
                                   use_mid_position_embeddings=False)
    torch.manual_seed(0)
    hf = transformers.YolosForObjectDetection(cfg).eval()
    m = YolosSmall(YolosConfig(num_layers=2)).eval()
    m.load_hf_state_dict(hf.state_dict())
    x = demo_input(1, (160, 224))
    with torch.no_grad():
        ref = hf(pixel_values=x)
        logits, boxes = m(x)
    assert (ref.logits - logits).abs().max().item() < 1e-5
    assert (ref.pred_boxes - boxes).abs().max().item() < 1e-5
    assert YolosSmall().flops_per_inference() == pytest.approx(359.6e9, rel=1e-3)


def test_bench_control_plane_and_slice_masks():
    from walkai_nos_amd.bench_core import BenchConfig, ChurnProcess, NodeBench, slice_cus, slice_pin
    assert slice_cus("spx_nps1", 0) is None and slice_pin("spx_nps1", 0) == 0
    # spread emulation: every CPX slice covers all 8 XCDs (bit i -> XCD i mod 8)
    assert slice_cus("cpx_nps1", 3, emulation="spread") == list(range(96, 128))
    assert len(slice_cus("dpx_nps1", 1, emulation="spread")) == 128
    assert {c % 8 for c in slice_cus("cpx_nps1", 5, emulation="spread")} == set(range(8))
    assert slice_pin("cpx_nps1", 5, "spread") == 0
    # pinned emulation: partition k of CPX / QPX / DPX owns XCD k / 2k..2k+1 / 4k..4k+3 and all their CUs
    assert {c % 8 for c in slice_cus("cpx_nps1", 5, emulation="pinned")} == {5}
    assert len(slice_cus("cpx_nps1", 5, emulation="pinned")) == 32
    assert slice_pin("cpx_nps1", 5, "pinned") == 1 << 5
    assert slice_pin("qpx_nps1", 1, "pinned") == 0b1100 and len(slice_cus("qpx_nps1", 1, emulation="pinned")) == 64
    assert slice_pin("dpx_nps1", 1, "pinned") == 0xF0 and len(slice_cus("dpx_nps1", 1, emulation="pinned")) == 128
    masks = [slice_pin("cpx_nps1", k, "pinned") for k in range(8)]
    assert sum(masks) == 0xFF and len(set(masks)) == 8
    # landing emulation: own XCDs minus the landing CU (index 31 in each XCD), plus the landing CU of
    # every other XCD; no two partitions share a working CU, and no partition works on a landing CU
    from walkai_nos_amd.bench_core import FLIP_COST_COMPONENTS, working_cus
    for prof, n in (("cpx_nps1", 8), ("qpx_nps1", 4), ("dpx_nps1", 2)):
        work = []
        for k in range(n):
            cus, pin = slice_cus(prof, k, emulation="landing"), slice_pin(prof, k, "landing")
            assert pin == slice_pin(prof, k, "pinned")
            own = [c for c in cus if (pin >> (c % 8)) & 1]
            assert working_cus(cus, pin) == len(own) == 31 * (8 // n)
            assert all(c // 8 != 31 for c in own)
            assert sorted(c % 8 for c in cus if not (pin >> (c % 8)) & 1) == [x for x in range(8) if not (pin >> x) & 1]
            assert all(c // 8 == 31 for c in cus if not (pin >> (c % 8)) & 1)
            work += own
        assert len(work) == len(set(work)) == 248
    a, b = ChurnProcess(BenchConfig(seed=7)), ChurnProcess(BenchConfig(seed=7))
    assert [a.arrivals() for _ in range(20)] == [b.arrivals() for _ in range(20)]
    # a flip darkens its GPU for flip_cost_s of cluster time: 90 s = 1.5 quanta of 60 s (one whole
    # dark quantum, then half of the next), and the dark part of a quantum neither serves nor ages
    cfg = BenchConfig(gpus=2, flip_cost_s=90.0, cluster_s=60.0, quantum_s=0.5)
    assert cfg.flip_quanta == 1.5 and BenchConfig(flip_cost_s=30.0).flip_quanta == 0.5
    nb = NodeBench(cfg, gpu_data_plane=False)
    served, seen = 0, set()
    for _ in range(30):
        nb.control_step()
        served += len(nb.my_pods())
        seen.add(nb.dark(0))
        nb.end_step()
    assert served > 0 and max(nb.util_samples) > 0 and nb.flips > 0
    assert seen <= {0.0, 0.5, 1.0} and 1.0 in seen or 0.5 in seen
    assert 0 < nb.outage_gpu_quanta <= 1.5 * nb.flips + 1e-9
    assert BenchConfig().flip_cost_s == round(sum(FLIP_COST_COMPONENTS.values()), 2)


def test_request_lanes_split_a_partition_into_disjoint_xcd_balanced_runs():
    from walkai_nos_amd.bench_core import lane_cu_runs, slice_cus
    runs = lane_cu_runs(None, 128)  # a whole-GPU pod: two lanes of 128 CUs
    assert [len(r) for r in runs] == [128, 128] and set(runs[0]).isdisjoint(runs[1])
    assert sorted(runs[0] + runs[1]) == list(range(256))
    assert all({c % 8 for c in r} == set(range(8)) for r in runs)  # 16 CUs on each XCD
    dpx = slice_cus("dpx_nps1", 1, emulation="spread")
    assert lane_cu_runs(dpx, 64) == [dpx[:64], dpx[64:]]
    # no split: off, a partition not wider than a lane, or a lane that would unbalance the XCDs
    assert lane_cu_runs(None, 0) == [None]
    assert lane_cu_runs(dpx, 128) == [dpx]
    assert lane_cu_runs(None, 100) == [None] and lane_cu_runs(None, 20) == [None]


def test_split3_cpu_reconstructs_exactly():
    import torch

    from walkai_nos_amd.ops import kernels as K
    x = torch.randn(4096, dtype=torch.float32) * torch.logspace(-10, 10, 4096)
    p = K.split3(x)
    assert torch.equal(p[0].double() + p[1].double() + p[2].double(), x.double())


def test_weight_planes_cached_on_tensor_and_invalidated_by_writes():
    import torch

    from walkai_nos_amd.ops import gemm as G
    w = torch.nn.Parameter(torch.randn(8, 3, 2, 2))
    p1 = G.weight_planes(w.reshape(8, -1))
    assert G.weight_planes(w.reshape(8, -1)) is p1        # views of one weight share the cache
    with torch.no_grad():
        w.mul_(2)
    p2 = G.weight_planes(w.reshape(8, -1))
    assert p2 is not p1
    assert torch.equal(p2[0].float() + p2[1].float() + p2[2].float(), w.detach().reshape(8, -1))
    other = torch.randn(8, 12)                             # a different tensor never hits w's cache
    assert torch.equal(G.weight_planes(other)[0], other.to(torch.bfloat16))


def test_attention_x3_grid_trimmed_to_query_group_boundaries(monkeypatch):
    # 84 query groups (T = 3401, 6 heads, 8 query tiles per workgroup): 256 CUs -> 252 = 84 x 3,
    # DPX 128 -> 126 = 84 x 1.5; slices with fewer slots than groups keep every slot
    from walkai_nos_amd.ops import kernels as K
    monkeypatch.setattr(K, "_x3_wg", 1)
    monkeypatch.setattr(K, "attention_x3_group", lambda: 8)
    assert [K.attention_x3_waves(c, 1, 3401, 6) for c in (256, 128, 64, 32)] == [252, 126, 64, 32]
    assert K.attention_x3_waves(256) == 256  # no shape: every slot


def test_x3_tuned_table_lookup(monkeypatch, tmp_path):
    import json
    from walkai_nos_amd.ops import gemm as G
    p = tmp_path / "x3_tuned.json"
    p.write_text(json.dumps({"M3401_N1152_K384_epi1_out2_cus32": {"tile": 102, "concurrent_us": 1.0},
                             "M1_N1_K32_epi0_out1_cus32": {"tile": 999}}))
    monkeypatch.setattr(G, "_TUNED_PATH", str(p))
    monkeypatch.setattr(G, "_tuned", None)
    t = G.tuned_table()
    assert t == {"M3401_N1152_K384_epi1_out2_cus32": 102}  # unknown tile ids are dropped
    monkeypatch.setattr(G, "_tuned", None)
    monkeypatch.setenv("NOS_X3_TUNED", "0")
    assert G.tuned_table() == {}
    monkeypatch.setattr(G, "_tuned", None)


def test_shipped_x3_tuned_table_names_known_tiles():
    import json
    import os
    from walkai_nos_amd.ops import gemm as G
    with open(G._TUNED_PATH) as f:
        table = json.load(f)
    for key, v in table.items():
        assert v["tile"] in G.X3_TILES, key
        n = int(key.split("_")[1][1:])
        assert n % G.X3_TILES[v["tile"]][1] == 0, key
    assert os.path.basename(G._TUNED_PATH) == "x3_tuned.json"


def test_split_candidates_and_partials_contract():
    # split-K partial configs: only LDS-DMA tiles whose width divides N and whose stage depth
    # divides K, each split covering at least two stages
    from walkai_nos_amd.ops import gemm as G
    c = G.split_candidates(384, 1536)
    assert c and all(cfg in G.SPLIT_TILES and sp in G.SPLIT_COUNTS for cfg, sp in c)
    for cfg, sp in c:
        bm, bn, _, kind = G.X3_TILES[cfg]
        bk = 64 if kind.endswith("64") else 32
        assert 384 % bn == 0 and 1536 // bk >= 2 * sp
    assert all(sp == 2 for _, sp in G.split_candidates(384, 128))  # 4 stages of 32: at most 2 splits
    assert G.split_candidates(100, 1536) == []                     # no tile width divides 100


def test_linear_residual_ln_x3_cpu_reference():
    # the CPU path of the fused projection/fc2 step equals linear + residual + LayerNorm
    import torch
    import torch.nn.functional as F
    from walkai_nos_amd.ops import kernels as K
    torch.manual_seed(2)
    a = torch.randn(2, 5, 64)
    w, b = torch.randn(32, 64) * 0.1, torch.randn(32)
    r, r2 = torch.randn(2, 5, 32), torch.randn(1, 5, 32)
    lw, lb = torch.randn(32), torch.randn(32)
    x, h3 = K.linear_residual_ln_x3(K.split3(a), w, b, r, residual2=r2, ln=(lw, lb, 1e-6))
    ref = F.linear(a, w, b) + r + r2
    assert torch.allclose(x, ref, atol=1e-5)
    assert torch.allclose(h3.float().sum(0) if h3.dtype != torch.float32 else h3.sum(0),
                          F.layer_norm(ref, (32,), lw, lb, 1e-6), atol=1e-4)
    x2, none = K.linear_residual_ln_x3(K.split3(a), w, b, r)
    assert none is None and torch.allclose(x2, F.linear(a, w, b) + r, atol=1e-5)


def test_detection_token_template_cached_per_parameter_version():
    import torch
    from walkai_nos_amd.models.workload.yolos import YolosConfig, YolosSmall
    m = YolosSmall(YolosConfig(num_layers=1))
    t1 = m.token_template((64, 64))
    assert m.token_template((64, 64)) is t1
    nd = m.c.num_detection_tokens
    pe, _ = m.position_embeddings((64, 64))
    assert torch.equal(t1[:, :1], m.cls_token + pe[:, :1]) and torch.equal(t1[:, -nd:], m.det_tokens + pe[:, -nd:])
    assert t1[:, 1:-nd].abs().max().item() == 0
    with torch.no_grad():
        m.det_tokens.add_(1.0)
    t2 = m.token_template((64, 64))
    assert t2 is not t1 and torch.equal(t2[:, -nd:], m.det_tokens + pe[:, -nd:])


def test_density_phase_control_plane_at_four_gpus():
    # saturation through the real control plane: 8 CPX pods per GPU; CU-mask slices at the chart's
    # cap of 8 per GPU (what a default node schedules), and 16 per GPU only with the cap lifted by
    # label, named so (first-fit may leave the last GPU lighter: the minimum is
    # reported beside the mean)
    from walkai_nos_amd.bench_core import BenchConfig, density_phase
    d = density_phase(BenchConfig(gpus=4), None)
    assert d["xcp"]["pods_per_gpu"] == 8 and d["xcp"]["pending"] == 0 and d["xcp"]["pods_per_node"] == 32
    for v in ("cumask", "cumask_shared"):
        assert d[v]["pending"] == 0 and d[v]["pods_per_node"] == 32 and d[v]["pods_per_gpu"] == 8
        assert d[v]["max_slices_per_gpu"] == 8
    for v in ("cumask_threads_cap_lifted", "cumask_shared_threads_cap_lifted"):
        assert d[v]["pending"] == 0 and d[v]["pods_per_node"] == 64 and d[v]["pods_per_gpu"] == 16
        assert 0 < d[v]["pods_per_gpu_min"] <= 16 and "not what a default node schedules" in d[v]["served_as"]


def test_inference_latency_summary_per_mode():
    from types import SimpleNamespace

    from walkai_nos_amd.bench_core import inference_latency
    slots = {("spx_nps1", 0): SimpleNamespace(latency_ms=[9.0, 9.5, 9.2]),
             ("cpx_nps1", 3): SimpleNamespace(latency_ms=[20.0]),
             ("cpx_nps1", 4): SimpleNamespace(latency_ms=[22.0]),
             ("dpx_nps1", 1): SimpleNamespace(latency_ms=[])}
    out = inference_latency(SimpleNamespace(slots=slots))
    assert set(out) == {"spx", "cpx"}  # modes that completed nothing are left out
    assert out["spx"]["n"] == 3 and out["spx"]["p50"] == 9.2 and abs(out["spx"]["mean"] - 9.233) < 1e-3
    assert out["cpx"] == {"n": 2, "mean": 21.0, "p50": 22.0, "p99": 22.0}
    assert inference_latency(None) == {}


def test_splitk_is_only_timed_on_slices_of_64_cus_or_more(monkeypatch):
    # below SPLITK_MIN_CUS the fused-epilogue path is taken without timing split-K (it loses under
    # sibling partitions, profiles/splitk_slice_ab_r2.json); from 64 CUs both pipelines are timed
    import torch

    from walkai_nos_amd.ops import gemm as G
    from walkai_nos_amd.ops import kernels as K
    timed = []
    monkeypatch.setattr(G, "gemm_x3", lambda a3, w, b, residual=None, residual2=None: residual.clone())
    monkeypatch.setattr(K, "layernorm_x3", lambda x, w, b, eps: torch.zeros((3,) + tuple(x.shape)))
    monkeypatch.setattr(G, "_gpu_time", lambda fn, stream: timed.append(fn) or 1.0)
    monkeypatch.setattr(G, "split_candidates", lambda N, Kd: [])
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)
    monkeypatch.setattr(torch.cuda, "current_stream", lambda: None)
    G._fused_cache.clear()
    a3, w, b = torch.zeros(3, 8, 64), torch.zeros(32, 64), torch.zeros(32)
    r = torch.zeros(8, 32)
    K.set_slice_cus(32)
    try:
        x, h3 = G.linear_residual_ln_x3(a3, w, b, r, ln=(b, b, 1e-12))
        assert not timed and x.shape == r.shape
        K.set_slice_cus(64)
        G.linear_residual_ln_x3(a3, w, b, r, ln=(b, b, 1e-12))
        assert len(timed) == 1  # the fused path timed (no split candidates offered here)
    finally:
        K.set_slice_cus(None)
        G._fused_cache.clear()


@pytest.mark.parametrize("gpus,load,seed", [(1, 1.3, 101), (3, 0.7, 102), (3, 1.3, 103), (8, 1.0, 104)])
def test_control_plane_soak_no_admission_failures(gpus, load, seed):
    # the whole control plane (pack planner, agents, partition plugin view, kubelet admission,
    # kube-scheduler semantics) under over- and under-load on odd node sizes: no pod is ever bound
    # to a partition kubelet then rejects, and the allocation figures stay physical
    from walkai_nos_amd.bench_core import BenchConfig, control_only
    r = control_only(BenchConfig(gpus=gpus, seed=seed, offered_load=load), 60)
    assert r["admission_failures"] == 0
    assert 0.0 < r["util_pct"] <= 100.0 and r["util_pct"] <= r["util_incl_outage_pct"] + 1e-9
