"""``nos.nebuly.com/v1alpha1`` protocol surface: labels, annotations, resources.

Wire-compatible with the reference (``pkg/api/nos.nebuly.com/v1alpha1/{labels,annotations,
constants}.go``): the same label key opts a node in, the same annotation grammar carries desired
(``spec-gpu-*``) and observed (``status-gpu-*``) partition state, and the same plan-ID pair acts as
the commit marker.

MI355X additions (new keys, never re-purposed old ones):

* partitioning kinds ``xcp`` (compute partitions, the MIG analogue) and ``cumask`` (CU-mask
  slicing, the MPS analogue) instead of ``mig``/``mps``;
* the node-wide memory-partition (NPS) desired/observed annotations, because an NPS change
  reloads the driver on every GPU of the node (``amdsmi.h:6600-6615``).
"""
from __future__ import annotations

GROUP = "nos.nebuly.com"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"

# -- labels (reference labels.go:21) --------------------------------------------------
LABEL_GPU_PARTITIONING = "nos.nebuly.com/gpu-partitioning"
LABEL_CAPACITY_INFO = "nos.nebuly.com/capacity"
# MI355X: how an xcp node's GPUs may be laid out — "partitions" (hardware compute partitions only,
# the default), "slices" (every GPU in SPX carved into CU-mask slices of the partition sizes: mixed
# geometries, re-carved without a drain), "auto" (the planner chooses per GPU); models/xcp/slices.py
LABEL_XCP_LAYOUT = "nos.nebuly.com/xcp-layout"
# cumask nodes: slices per GPU the planner may carve (default models/slicing/profile.MAX_SLICES_PER_GPU)
LABEL_MAX_SLICES_PER_GPU = "nos.nebuly.com/max-slices-per-gpu"
CAPACITY_IN_QUOTA = "in-quota"
CAPACITY_OVER_QUOTA = "over-quota"

# -- annotations (reference annotations.go:21-58) ------------------------------------
ANNOTATION_GPU_SPEC_PREFIX = "nos.nebuly.com/spec-gpu"
ANNOTATION_GPU_STATUS_PREFIX = "nos.nebuly.com/status-gpu"
ANNOTATION_GPU_SPEC_FORMAT = "nos.nebuly.com/spec-gpu-{index}-{profile}"
ANNOTATION_GPU_STATUS_FORMAT = "nos.nebuly.com/status-gpu-{index}-{profile}-{status}"
ANNOTATION_PARTITIONING_PLAN = "nos.nebuly.com/spec-partitioning-plan"
ANNOTATION_REPORTED_PARTITIONING_PLAN = "nos.nebuly.com/status-partitioning-plan"

# MI355X: node-wide memory partition mode (NPS1/NPS2/NPS4/NPS8)
ANNOTATION_MEMORY_PARTITION_SPEC = "nos.nebuly.com/spec-memory-partition"
ANNOTATION_MEMORY_PARTITION_STATUS = "nos.nebuly.com/status-memory-partition"
# MI355X: GPUs served as CU-mask slices (comma-separated indexes): the ones the plan wants sliced
# (written with the spec by the partitioner) and the ones the agent serves sliced (status)
ANNOTATION_SLICED_GPUS_SPEC = "nos.nebuly.com/spec-sliced-gpus"
ANNOTATION_SLICED_GPUS_STATUS = "nos.nebuly.com/status-sliced-gpus"
# MI355X: outcome of the node-atomic commit barrier for the last plan ("ok" / "failed:<reason>")
ANNOTATION_COMMIT_STATUS = "nos.nebuly.com/status-partitioning-commit"
# MI355X: write-ahead journal of the plan the agent is applying (JSON {plan, from, to}); written
# before the first mode flip and removed after the commit, so an agent that crashes between two
# flips finds the half-applied plan at start-up (see Actuator.startup)
ANNOTATION_INFLIGHT_PLAN = "nos.nebuly.com/status-partitioning-inflight"
# MI355X: probe-kernel measurement published by the agent (JSON: per slice TFLOP/s per CU)
ANNOTATION_PROBE_RESULT = "nos.nebuly.com/status-probe"
# MI355X: pods per physical GPU as the agent reads them from kubelet's PodResources (JSON
# {"<gpu index>": ["<ns>/<pod>", ...]}): what nos-scheduler must evict to free a whole GPU for a flip
ANNOTATION_GPU_PODS_STATUS = "nos.nebuly.com/status-pods"
# MI355X (pods): set by nos-scheduler on a pod it evicted a whole GPU for (value: the node); the
# pod's request stays held against its quota until it is bound, so borrowers cannot take it back
ANNOTATION_QUOTA_RECLAIM = "nos.nebuly.com/quota-reclaim"

# -- resources (reference constants.go:24-27) ------------------------------------------
RESOURCE_GPU_MEMORY = "nos.nebuly.com/gpu-memory"

# -- partitioning kinds ---------------------------------------------------------------
PARTITIONING_KIND_XCP = "xcp"
PARTITIONING_KIND_CUMASK = "cumask"
PARTITIONING_KINDS = (PARTITIONING_KIND_XCP, PARTITIONING_KIND_CUMASK)

# -- CRD kinds -------------------------------------------------------------------------
KIND_ELASTIC_QUOTA = "ElasticQuota"
KIND_COMPOSITE_ELASTIC_QUOTA = "CompositeElasticQuota"
