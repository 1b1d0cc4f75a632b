"""``config.nos.nebuly.com/v1alpha1`` ComponentConfigs and the capacity-scheduling plugin args.

Field names follow the reference (``pkg/api/nos.nebuly.com/config/v1alpha1/*``,
``config/*/manager/*_config.yaml``) so existing config files load unchanged:

* ``GpuPartitionerConfig`` — manager options plus ``batchWindowTimeoutSeconds``,
  ``batchWindowIdleSeconds``, ``knownMigGeometriesFile`` (alias ``knownGeometriesFile``),
  ``schedulerConfigFile``, ``devicePluginConfigMap{name,namespace}``, ``devicePluginDelaySeconds``;
  MI355X additions ``planningPolicy`` (``pack`` = flip-aware packing, default | ``fifo`` | ``batch`` | ``simulate``) and ``scoring`` (``fraction``|``pods``);
* ``MigAgentConfig`` (the partition agent; also accepted as ``PartitionAgentConfig``) and
  ``GpuAgentConfig`` (the CU-mask slice agent; also ``SliceAgentConfig``) with
  ``reportConfigIntervalSeconds``;
* ``CapacitySchedulingArgs`` with ``nvidiaGpuResourceMemoryGB`` (reference name, kept) and its AMD
  alias ``amdGpuResourceMemoryGB``.

Unlike the reference, ``validate()`` is actually called by every entry point and an
omitted report interval means the documented 10 s rather than "no periodic report" (Q5).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field
from typing import Any, Dict, List, Optional, Type, TypeVar

import yaml

from .. import constant

API_VERSION = "config.nos.nebuly.com/v1alpha1"


@dataclass
class LeaderElection:
    leaderElect: bool = False
    resourceName: str = ""
    resourceNamespace: str = "nos-system"
    leaseDurationSeconds: float = 15.0
    renewDeadlineSeconds: float = 10.0
    retryPeriodSeconds: float = 2.0
    leaderElectionReleaseOnCancel: bool = False


@dataclass
class ManagerConfig:
    healthProbeBindAddress: str = ":8081"
    metricsBindAddress: str = "127.0.0.1:8080"
    webhookPort: int = 9443
    leaderElection: LeaderElection = field(default_factory=LeaderElection)

    def validate(self) -> None:
        le = self.leaderElection
        if le.leaderElect and not le.resourceName:
            raise ValueError("leaderElection.resourceName is required when leaderElect is true")
        if le.leaderElect and not (le.leaseDurationSeconds > le.renewDeadlineSeconds > le.retryPeriodSeconds > 0):
            raise ValueError("leaderElection durations must satisfy leaseDuration > renewDeadline > retryPeriod > 0")


@dataclass
class NamespacedObject:
    name: str = ""
    namespace: str = ""


@dataclass
class GpuPartitionerConfig(ManagerConfig):
    schedulerConfigFile: str = ""
    knownMigGeometriesFile: str = ""
    batchWindowTimeoutSeconds: float = 60.0
    batchWindowIdleSeconds: float = 10.0
    devicePluginConfigMap: NamespacedObject = field(default_factory=lambda: NamespacedObject(
        constant.DEFAULT_DEVICE_PLUGIN_CONFIGMAP_NAME, constant.DEFAULT_DEVICE_PLUGIN_CONFIGMAP_NAMESPACE))
    devicePluginDelaySeconds: float = 5.0
    planningPolicy: str = "pack"
    scoring: str = "fraction"
    #: knobs of the ``pack`` policy (``PackParams``); keys: minFill, starveAfterSeconds,
    #: drainAfterSeconds, drainBacklog, spxReserve, reserveDecay, drainGain, drainGainAfterSeconds,
    #: reserveBreakFill, minStintSeconds, unservedAfterSeconds; sliced GPUs (xcp-layout slices /
    #: auto): sliceReserveAfterSeconds, sliceReserveLifetimes (the threshold in median pod run times
    #: once learned; 0 = the constant), sliceReserveBacklog (GPUs of waiting work per sliced GPU
    #: above which the threshold stretches; 0 = never), sliceReserveStretch (its largest factor),
    #: sliceReserveHold, sliceReserveHoldMaxGpus, sliceFreeDrain, sliceFreeDrainAfterLifetimes,
    #: sliceFreeDrainCapLifetimes, sliceStrandWeight, sliceWholeOvertakeSeconds, sliceWholeOvertakeLifetimes,
    #: sliceFill
    packing: Dict[str, Any] = field(default_factory=dict)
    #: xcp layout of a node that carries no nos.nebuly.com/xcp-layout label: slices (SPX GPUs carved
    #: into CU-mask slices, mixed geometries, no flips), partitions (hardware compute partitions
    #: only) or auto (per GPU: a hardware mode for homogeneous demand, else slices)
    defaultXcpLayout: str = "slices"
    #: memory-only slice counts the planner never leaves on a cumask GPU: it carves two at once past
    #: them, or the odd pod waits (models/slicing/profile.py SKIP_SHARED_COUNTS: odd counts from 5
    #: up split the pods into two rate classes by start order); [] disables
    sharedSliceSkipCounts: List[int] = field(default_factory=lambda: [5, 7])

    PACKING_KEYS = {"minFill": "min_fill", "starveAfterSeconds": "starve_after", "drainAfterSeconds": "drain_after",
                    "drainBacklog": "drain_backlog", "spxReserve": "spx_reserve", "reserveDecay": "reserve_decay",
                    "drainGain": "drain_gain", "drainGainAfterSeconds": "drain_gain_after", "minStintSeconds": "min_stint",
                    "unservedAfterSeconds": "unserved_after", "replanEverySeconds": "replan_every",
                    "reserveBreakFill": "reserve_break_fill", "sliceReserveAfterSeconds": "slice_reserve_after",
                    "sliceReserveBacklog": "slice_reserve_backlog", "sliceReserveStretch": "slice_reserve_stretch",
                    "sliceReserveLifetimes": "slice_reserve_lifetimes", "sliceReserveHold": "slice_reserve_hold",
                    "sliceReserveHoldMaxGpus": "slice_reserve_hold_max_gpus",
                    "sliceFreeDrain": "slice_free_drain", "sliceFreeDrainAfterLifetimes": "slice_free_drain_after",
                    "sliceFreeDrainCapLifetimes": "slice_free_drain_cap",
                    "sliceStrandWeight": "slice_strand_weight",
                    "sliceWholeOvertakeSeconds": "slice_whole_overtake",
                    "sliceWholeOvertakeLifetimes": "slice_whole_overtake_lifetimes", "sliceFill": "slice_fill"}
    BOOL_PACKING_KEYS = ("spxReserve", "sliceFill", "sliceReserveHold", "sliceFreeDrain")

    def pack_params(self) -> Any:
        from ..controllers.partitioner.pod_controller import PackParams
        return PackParams(**{self.PACKING_KEYS[k]: (bool(v) if k in self.BOOL_PACKING_KEYS else float(v))
                             for k, v in self.packing.items()})

    def validate(self) -> None:
        super().validate()
        unknown = set(self.packing) - set(self.PACKING_KEYS)
        if unknown:
            raise ValueError(f"packing: unknown keys {sorted(unknown)}")
        for k, v in self.packing.items():
            if k not in self.BOOL_PACKING_KEYS and (not isinstance(v, (int, float)) or v < 0):
                raise ValueError(f"packing.{k} must be a non-negative number")
        if self.batchWindowTimeoutSeconds <= 0:
            raise ValueError("batchWindowTimeoutSeconds must be greater than 0")
        if self.batchWindowIdleSeconds <= 0:
            raise ValueError("batchWindowIdleSeconds must be greater than 0")
        if self.devicePluginDelaySeconds <= 0:
            raise ValueError("devicePluginDelaySeconds must be greater than 0")
        if self.planningPolicy not in ("fifo", "batch", "simulate", "pack"):
            raise ValueError("planningPolicy must be 'fifo', 'batch', 'simulate' or 'pack'")
        if self.defaultXcpLayout not in ("partitions", "slices", "auto"):
            raise ValueError("defaultXcpLayout must be 'partitions', 'slices' or 'auto'")
        if any(not isinstance(c, int) or c < 2 for c in self.sharedSliceSkipCounts):
            raise ValueError("sharedSliceSkipCounts must list integers >= 2")
        if self.scoring not in ("fraction", "pods"):
            raise ValueError("scoring must be 'fraction' or 'pods'")


@dataclass
class AgentConfig(ManagerConfig):
    reportConfigIntervalSeconds: float = 10.0
    amdSmiBackend: str = "native"           # native | fake
    fakeGpus: int = 8                       # GPUs of the fake backend (development clusters, e2e tests)
    fakeStateFile: str = ""                 # fake backend: keep GPU modes in this file across agent restarts
    devicePluginLabel: str = constant.DEFAULT_DEVICE_PLUGIN_LABEL
    devicePluginNamespace: str = ""
    podResourcesSocket: str = constant.DEFAULT_POD_RESOURCES_SOCKET
    commitBarrier: str = "xgmi"             # xgmi (P2P token ring) | rccl (communicator all-reduce) | none
    probeOnCommit: bool = True
    devicePluginDir: str = "/var/lib/kubelet/device-plugins"  # kubelet's plugin dir (kubelet.sock + our sockets)
    #: pods over their slices' HBM budget (amd-smi per-process VRAM, controllers/hbmguard.py):
    #: off | report (metric + log) | evict (delete the pod)
    hbmGuard: str = "report"
    hbmGuardIntervalSeconds: float = 10.0
    #: VRAM each process may map beyond what the budget interposer counts (HIP runtime, code
    #: objects: 490 MiB measured for a PyTorch process)
    hbmGuardSlackBytes: int = 768 << 20
    #: pods running on more CUs than their slices have (HSA_CU_MASK bypassed; amd-smi per-process
    #: CU occupancy, controllers/hbmguard.py): off | report (metric + Warning event) | evict
    cuGuard: str = "report"
    cuGuardStrikes: int = 3

    def validate(self) -> None:
        super().validate()
        if self.hbmGuard not in ("off", "report", "evict"):
            raise ValueError("hbmGuard must be 'off', 'report' or 'evict'")
        if self.cuGuard not in ("off", "report", "evict"):
            raise ValueError("cuGuard must be 'off', 'report' or 'evict'")
        if self.cuGuardStrikes < 1:
            raise ValueError("cuGuardStrikes must be >= 1")
        if self.hbmGuardIntervalSeconds <= 0:
            raise ValueError("hbmGuardIntervalSeconds must be greater than 0")
        if self.hbmGuardSlackBytes < 0:
            raise ValueError("hbmGuardSlackBytes must be >= 0")
        if self.reportConfigIntervalSeconds <= 0:
            raise ValueError("reportConfigIntervalSeconds must be greater than 0")
        if self.amdSmiBackend not in ("native", "fake"):
            raise ValueError("amdSmiBackend must be 'native' or 'fake'")
        if self.fakeGpus <= 0:
            raise ValueError("fakeGpus must be greater than 0")
        if self.commitBarrier not in ("xgmi", "rccl", "none"):
            raise ValueError("commitBarrier must be 'xgmi', 'rccl' or 'none'")


@dataclass
class MigAgentConfig(AgentConfig):
    """Partition agent configuration (kind kept from the reference for config compatibility).

    ``devicePlugin``: ``nos`` (default) — the agent serves the compute partitions itself
    (``deviceplugin/partitions.py``) and enforces drains through device health; ``amd`` — the AMD
    k8s-device-plugin serves them and is restarted after a flip (no drain enforcement: a GPU the
    partitioner drains keeps receiving pods on its free partitions)."""
    devicePlugin: str = "nos"
    publishAllocatable: bool = True         # patch node status.allocatable right after each plugin sync
    # CU-mask slice layout of the node's sliced GPUs (xcp-layout slices/auto): a host path, so an
    # agent restart keeps serving the slices pods run on
    sliceStateFile: str = "/var/lib/nos/xcp-slices.json"
    hbmLimitShimPath: str = "/usr/lib/nos/libnos_hbmlimit.so"
    # probe-on-commit health rule: a partition/slice whose bf16 rate per CU is below this fraction of
    # its model's expected rate is advertised Unhealthy (0 = never)
    probeHealthyFraction: float = 0.7

    def validate(self) -> None:
        super().validate()
        if self.devicePlugin not in ("nos", "amd"):
            raise ValueError("devicePlugin must be 'nos' or 'amd'")
        if not 0.0 <= self.probeHealthyFraction < 1.0:
            raise ValueError("probeHealthyFraction must be in [0, 1)")


@dataclass
class GpuAgentConfig(AgentConfig):
    """CU-mask slice agent configuration (kind kept from the reference).

    ``sharedSliceHwQueues``: hardware queues a memory-only slice's container may create
    (``GPU_MAX_HW_QUEUES`` in ``Allocate``): 1-4 fixed, 0 leaves HIP's default of 4, -1 (default)
    = 2 while at most 3 memory-only slices share the GPU, else 1. Memory-only slices share every
    CU and the command processor arbitrates dispatch per hardware pipe, so a pod's share of the GPU
    follows where its queues land, not the pod count; the auto rule is the measured best per pod
    count (docs/partitioning-modes-comparison.md, ``profiles/fairness_r4_repeat.json``)."""
    hbmLimitShimPath: str = "/usr/lib/nos/libnos_hbmlimit.so"
    sharedSliceHwQueues: int = -1
    #: memory-only containers of one GPU start one after another through the slice plugin's
    #: PreStartContainer (deviceplugin/startgate.py): the longest wait for the previous one's
    #: compute queues, seconds (0 = no gate; kubelet gives the call 30 s)
    sharedSliceStartGateSeconds: float = 20.0

    def validate(self) -> None:
        super().validate()
        if not -1 <= self.sharedSliceHwQueues <= 4:
            raise ValueError("sharedSliceHwQueues must be -1 (auto), 0 (HIP default) or 1..4")
        if not 0 <= self.sharedSliceStartGateSeconds < 30:
            raise ValueError("sharedSliceStartGateSeconds must be in [0, 30) (kubelet's PreStartContainer timeout)")


@dataclass
class CapacitySchedulingArgs:
    nvidiaGpuResourceMemoryGB: int = constant.DEFAULT_GPU_RESOURCE_MEMORY_GB

    def validate(self) -> None:
        if self.nvidiaGpuResourceMemoryGB <= 0:
            raise ValueError("GPU resource memory must be greater than 0")


KINDS: Dict[str, Type[Any]] = {
    "GpuPartitionerConfig": GpuPartitionerConfig,
    "MigAgentConfig": MigAgentConfig,
    "PartitionAgentConfig": MigAgentConfig,
    "GpuAgentConfig": GpuAgentConfig,
    "SliceAgentConfig": GpuAgentConfig,
    "CapacitySchedulingArgs": CapacitySchedulingArgs,
}

T = TypeVar("T")


def _flatten(doc: Dict[str, Any]) -> Dict[str, Any]:
    """controller-runtime nests manager options; flatten them onto the dataclass fields."""
    out = dict(doc)
    health = out.pop("health", None) or {}
    if "healthProbeBindAddress" in health:
        out["healthProbeBindAddress"] = health["healthProbeBindAddress"]
    metrics = out.pop("metrics", None) or {}
    if "bindAddress" in metrics:
        out["metricsBindAddress"] = metrics["bindAddress"]
    webhook = out.pop("webhook", None) or {}
    if "port" in webhook:
        out["webhookPort"] = webhook["port"]
    if "knownGeometriesFile" in out:
        out["knownMigGeometriesFile"] = out.pop("knownGeometriesFile")
    if "amdGpuResourceMemoryGB" in out:
        out["nvidiaGpuResourceMemoryGB"] = out.pop("amdGpuResourceMemoryGB")
    for dur in ("leaseDuration", "renewDeadline", "retryPeriod"):
        le = out.get("leaderElection")
        if isinstance(le, dict) and dur in le:
            v = str(le.pop(dur)).rstrip("s")
            le[dur + "Seconds"] = float(v)
    return out


def _build(cls: Type[T], data: Dict[str, Any]) -> T:
    kwargs = {}
    fields = getattr(cls, "__dataclass_fields__", {})
    for k, v in data.items():
        if k not in fields:
            raise ValueError(f"{cls.__name__}: unknown field {k!r}")
        ftype = fields[k].type
        if k == "leaderElection" and isinstance(v, dict):
            v = _build(LeaderElection, v)
        elif k == "devicePluginConfigMap" and isinstance(v, dict):
            v = _build(NamespacedObject, v)
        kwargs[k] = v
        del ftype
    return cls(**kwargs)


def load_config(text: str, expected_kind: Optional[str] = None, validate: bool = True) -> Any:
    doc = yaml.safe_load(text) or {}
    kind = doc.pop("kind", expected_kind)
    api_version = doc.pop("apiVersion", API_VERSION)
    if api_version not in (API_VERSION, "kubescheduler.config.k8s.io/v1beta3", "nos.nebuly.com/v1alpha1"):
        raise ValueError(f"unsupported apiVersion {api_version!r}")
    if kind not in KINDS:
        raise ValueError(f"unknown config kind {kind!r}")
    if expected_kind and KINDS[kind] is not KINDS[expected_kind]:
        raise ValueError(f"expected kind {expected_kind}, got {kind}")
    cfg = _build(KINDS[kind], _flatten(doc))
    if validate:
        cfg.validate()
    return cfg


def load_config_file(path: str, expected_kind: Optional[str] = None) -> Any:
    with open(path) as f:
        return load_config(f.read(), expected_kind)


def dump_config(cfg: Any, kind: str) -> str:
    d = asdict(cfg)
    return yaml.safe_dump({"apiVersion": API_VERSION, "kind": kind, **d}, sort_keys=False)
