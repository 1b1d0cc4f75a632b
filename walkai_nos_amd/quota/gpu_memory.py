"""GPU-memory calculator for Elastic Resource Quotas (L5; reference ``pkg/gpu/util/resource.go:28-86``).

``nos.nebuly.com/gpu-memory`` (GB) of a pod =
    ``amd.com/gpu`` x ``gpuResourceMemoryGB`` (a whole GPU; 288 on MI355X)
  + sum over compute partitions ``amd.com/<mode>_<nps>`` of the partition's HBM (288 / partitions)
  + sum over CU-mask slices ``amd.com/gpu-[<c>cu.]<m>gb`` of ``m``.

The reference does the same for ``nvidia.com/gpu`` (x 32 by Helm default, 16 in code) plus the
memory encoded in ``nvidia.com/mig-<g>g.<m>gb``; its docs example (``1g.10gb`` + 1 GPU = 42) is
reproduced by the NVIDIA-compatible branch kept for mixed clusters.
"""
from __future__ import annotations

import re
from typing import Dict, Mapping

from .. import constant
from ..api import v1alpha1 as api
from ..models import resource as res
from ..models.slicing.profile import extract_profile_name as slice_profile, parse_profile as parse_slice
from ..models.xcp.known_configs import get_model_spec
from ..models.xcp.profile import extract_profile_name as xcp_profile, parse_profile as parse_xcp

_NVIDIA_MIG = re.compile(r"^nvidia\.com/mig-\d+g\.(\d+)gb$")


class GpuMemoryCalculator:
    def __init__(self, gpu_resource_memory_gb: int = constant.DEFAULT_GPU_RESOURCE_MEMORY_GB, model: str = "MI355X",
                 nvidia_gpu_resource_memory_gb: int = 32):
        self.gpu_gb = gpu_resource_memory_gb
        spec = get_model_spec(model)
        self.model_gb = spec.memory_gb if spec else gpu_resource_memory_gb
        self.nvidia_gpu_gb = nvidia_gpu_resource_memory_gb

    def required_gb(self, requests: Mapping[str, int]) -> int:
        total = 0
        for r, q in requests.items():
            if q <= 0:
                continue
            if r == constant.RESOURCE_AMD_GPU:
                total += self.gpu_gb * q
                continue
            p = xcp_profile(r)
            if p is not None:
                total += parse_xcp(p).memory_gb(self.model_gb) * q
                continue
            sp = slice_profile(r)
            if sp is not None:
                total += parse_slice(sp).memory_gb * q
                continue
            if r == "nvidia.com/gpu":
                total += self.nvidia_gpu_gb * q
                continue
            m = _NVIDIA_MIG.match(r)
            if m:
                total += int(m.group(1)) * q
        return total

    def pod_request(self, pod: Dict) -> Dict[str, int]:
        """``ComputePodRequest`` + the derived ``nos.nebuly.com/gpu-memory`` entry."""
        rl = res.compute_pod_request(pod)
        rl[api.RESOURCE_GPU_MEMORY] = self.required_gb(rl)
        return rl
