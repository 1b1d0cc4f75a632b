"""Framework-wide constants (reference ``pkg/constant/constants.go:25-101``, AMD-native).

NVIDIA GPU Feature Discovery labels become the labels published by the AMD GPU node labeller;
``nvidia.com/*`` resources become the AMD k8s-device-plugin's ``amd.com/*`` resources; the
device-plugin DaemonSet label is configurable with the AMD plugin's default.
"""
from __future__ import annotations

import re

# controller names
CLUSTER_PARTITIONER_CONTROLLER = "gpu-partitioner"
NODE_INITIALIZER_CONTROLLER = "node-initializer"
AGENT_REPORTER_CONTROLLER = "partition-agent-reporter"
AGENT_ACTUATOR_CONTROLLER = "partition-agent-actuator"
SLICE_AGENT_REPORTER_CONTROLLER = "slice-agent-reporter"
SLICE_AGENT_ACTUATOR_CONTROLLER = "slice-agent-actuator"
QUOTA_OPERATOR_CONTROLLER = "elastic-quota-operator"

# resources
AMD_RESOURCE_PREFIX = "amd.com/"
RESOURCE_AMD_GPU = "amd.com/gpu"
# compute partitions as advertised by the AMD device plugin's "mixed" naming strategy
RESOURCE_XCP_REGEX = re.compile(r"^amd\.com/((spx|dpx|qpx|cpx)_(nps[1248]))$")
# CU-mask / memory slices: amd.com/gpu-<n>gb (memory only, CUs shared) or amd.com/gpu-<c>cu.<n>gb
RESOURCE_SLICE_PREFIX = "amd.com/gpu-"
RESOURCE_SLICE_REGEX = re.compile(r"^amd\.com/gpu-((?:(\d+)cu\.)?(\d+)gb)$")

# node labels (AMD GPU node labeller; count/memory/cu published by the agent if absent)
LABEL_AMD_GPU_PRODUCT = "amd.com/gpu.product-name"
LABEL_AMD_GPU_COUNT = "amd.com/gpu.count"
LABEL_AMD_GPU_VRAM = "amd.com/gpu.vram"             # e.g. "288G"
LABEL_AMD_GPU_CU_COUNT = "amd.com/gpu.cu-count"      # e.g. "256"
LABEL_AMD_COMPUTE_PARTITION = "amd.com/compute-partitioning-mode"
LABEL_AMD_MEMORY_PARTITION = "amd.com/memory-partitioning-mode"

# env
ENV_NODE_NAME = "NODE_NAME"
ENV_HSA_CU_MASK = "HSA_CU_MASK"
ENV_HBM_LIMIT = "NOS_HBM_LIMIT_BYTES"
#: HIP's per-process hardware queue count (memory-only slices: sharedSliceHwQueues)
ENV_GPU_MAX_HW_QUEUES = "GPU_MAX_HW_QUEUES"
ENV_SLICE_CU_MASK = "NOS_SLICE_CU_MASK"  # hex CU bitmap (consumed by the stream shim)

# defaults
DEFAULT_GPU_RESOURCE_MEMORY_GB = 288  # one MI355X (the reference's in-code fallback is 16 for nvidia.com/gpu)
DEFAULT_POD_RESOURCES_TIMEOUT_S = 10.0
DEFAULT_POD_RESOURCES_MAX_MSG_SIZE = 16 * 1024 * 1024
DEFAULT_POD_RESOURCES_SOCKET = "/var/lib/kubelet/pod-resources/kubelet.sock"
DEFAULT_DEVICE_PLUGIN_CONFIGMAP_NAME = "nos-device-plugin-config"
DEFAULT_DEVICE_PLUGIN_CONFIGMAP_NAMESPACE = "nos-system"
DEFAULT_DEVICE_PLUGIN_LABEL = "app=amdgpu-device-plugin-daemonset"
DEFAULT_DEVICE_PLUGIN_RESTART_TIMEOUT_S = 60.0

# field index keys
POD_PHASE_KEY = "status.phase"
POD_NODE_NAME_KEY = "spec.nodeName"
