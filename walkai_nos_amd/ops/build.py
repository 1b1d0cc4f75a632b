"""Build every native library in-tree for gfx950.

One target per concern: the amd-smi backend (C++), the slice probe (HIP), the
CU-mask/HBM-limit shim (C++, ``LD_PRELOAD``), the RCCL commit barrier (C++), and the fused
workload kernels (HIP).  Outputs land in ``walkai_nos_amd/_native/`` so they travel to the GPU box
with the ``gpurun`` snapshot.  Rebuilds only when a source is newer than its library.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass, field
from typing import List, Sequence

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
OUT = os.path.join(ROOT, "walkai_nos_amd", "_native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


@dataclass
class Target:
    name: str
    sources: List[str]
    compiler: str  # "hipcc" | "g++"
    flags: List[str] = field(default_factory=list)
    libs: List[str] = field(default_factory=list)
    headers: List[str] = field(default_factory=list)

    @property
    def out(self) -> str:
        return os.path.join(OUT, self.name)

    def stale(self) -> bool:
        if not os.path.exists(self.out):
            return True
        t = os.path.getmtime(self.out)
        deps = [os.path.join(CSRC, s) for s in self.sources + self.headers] + [os.path.abspath(__file__)]
        return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))

    def command(self) -> List[str]:
        srcs = [os.path.join(CSRC, s) for s in self.sources]
        common = ["-O3", "-std=c++17", "-fPIC", "-shared", f"-I{ROCM}/include", f"-I{CSRC}"]
        if self.compiler == "hipcc":
            cc = [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-Wno-unused-result",
                  "-Wno-unused-value"]
        else:
            cc = [shutil.which("g++") or "g++", "-Wall"]
        link = [f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib"] + [f"-l{lib}" for lib in self.libs]
        return cc + common + self.flags + srcs + ["-o", self.out] + link


TARGETS: Sequence[Target] = (
    Target("libnos_amdsmi.so", ["amdsmi_backend.cpp"], "g++", libs=["amd_smi"]),
    Target("libnos_probe.so", ["probe.hip"], "hipcc"),
    Target("libnos_hbmlimit.so", ["hbm_limit.cpp"], "g++", flags=["-D__HIP_PLATFORM_AMD__"], libs=["dl"]),
    Target("libnos_barrier.so", ["rccl_barrier.cpp"], "g++", flags=["-D__HIP_PLATFORM_AMD__"],
           libs=["rccl", "amdhip64"]),
    Target("libnos_kernels.so", ["kernels.hip", "gemm.hip", "gemm_x3.hip"], "hipcc"),
)


def build(force: bool = False, verbose: bool = True, jobs: int = 4) -> List[str]:
    os.makedirs(OUT, exist_ok=True)
    todo = [t for t in TARGETS if os.path.exists(os.path.join(CSRC, t.sources[0])) and (force or t.stale())]

    def run(t: Target) -> str:
        cmd = t.command()
        p = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True)
        if p.returncode != 0:
            raise RuntimeError(f"building {t.name} failed:\n{' '.join(cmd)}\n{p.stderr[-4000:]}")
        return t.name

    built: List[str] = []
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for name in ex.map(run, todo):
            built.append(name)
            if verbose:
                print(f"[nos build] {name}", file=sys.stderr)
    return built


if __name__ == "__main__":
    build(force="--force" in sys.argv)
