"""Build every native library in-tree for gfx950.

One target per concern: the amd-smi backend (C++), the slice probe (HIP), the
CU-mask/HBM-limit shim (C++, ``LD_PRELOAD``), the RCCL commit barrier (C++), and the fused
workload kernels (HIP).  Outputs land in ``walkai_nos_amd/_native/`` so they travel to the GPU box
with the ``gpurun`` snapshot.

Every library is **stamped** with a SHA-256 over its sources, headers, compiler command and this
file (``<lib>.stamp``, JSON).  A library is rebuilt when the stamp is missing or differs — never by
mtime, which a copied tree does not preserve — and :func:`walkai_nos_amd.ops.native.load` refuses
a library whose stamp no longer matches the sources next to it, so a GPU run can never execute a
stale build silently; ``__graft_entry__.build()`` prints the stamps it built or verified.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
from dataclasses import dataclass, field
from typing import Dict, List, Sequence

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
    executable: bool = False   # a program (spawned by the agents), not a shared library
    # options of one source only (its own object, linked into the target): code-generation choices
    # that are right for one kernel and wrong for the rest (csrc/attn_wide.hip)
    source_flags: Dict[str, List[str]] = field(default_factory=dict)

    @property
    def out(self) -> str:
        return os.path.join(OUT, self.name)

    @property
    def stamp_path(self) -> str:
        return self.out + ".stamp"

    def source_hash(self) -> str:
        """SHA-256 over sources + headers (+ every csrc header the sources may include) and the
        build recipe (compiler command, this file)."""
        h = hashlib.sha256()
        deps = sorted(set(self.sources + self.headers + [f for f in os.listdir(CSRC) if f.endswith((".h", ".hpp"))]))
        for d in deps:
            path = os.path.join(CSRC, d)
            if os.path.exists(path):
                h.update(d.encode())
                with open(path, "rb") as f:
                    h.update(f.read())
        # the recipe without machine-specific paths: the tree is built here and run from another
        # checkout path on the GPU box
        recipe = " ".join(" ".join(c[1:]) for c in self.commands())
        recipe = recipe.replace(CSRC, "<csrc>").replace(OUT, "<out>").replace(ROOT, "<root>")
        h.update(recipe.encode())
        with open(os.path.abspath(__file__), "rb") as f:
            h.update(f.read())
        return h.hexdigest()

    def read_stamp(self) -> dict:
        try:
            with open(self.stamp_path) as f:
                return json.load(f)
        except (OSError, ValueError):
            return {}

    def stale(self) -> bool:
        return not os.path.exists(self.out) or self.read_stamp().get("sha256") != self.source_hash()

    def _cc(self) -> List[str]:
        if self.compiler == "hipcc":
            return [os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-Wno-unused-result",
                    "-Wno-unused-value"]
        return [shutil.which("g++") or "g++", "-Wall"]

    def _obj(self, src: str) -> str:
        return os.path.join(OUT, f"{self.name}.{src}.o")

    def commands(self) -> List[List[str]]:
        """The compile commands, in order: one object per source with its own options, then the
        target from the other sources and those objects."""
        inc = ["-O3", "-std=c++17", "-fPIC", f"-I{ROCM}/include", f"-I{CSRC}"]
        cmds = [self._cc() + inc + self.flags + self.source_flags[s] + ["-c", os.path.join(CSRC, s), "-o", self._obj(s)]
                for s in self.sources if s in self.source_flags]
        # the objects first: hipcc marks each .hip source `-x hip`, which would claim a later object
        srcs = [self._obj(s) for s in self.sources if s in self.source_flags] + \
            [os.path.join(CSRC, s) for s in self.sources if s not in self.source_flags]
        link = [f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib"] + [f"-l{lib}" for lib in self.libs]
        shared = [] if self.executable else ["-shared"]
        return cmds + [self._cc() + inc + shared + self.flags + srcs + ["-o", self.out] + link]

    def command(self) -> List[str]:
        """The final (link) command."""
        return self.commands()[-1]


TARGETS: Sequence[Target] = (
    Target("libnos_amdsmi.so", ["amdsmi_backend.cpp"], "g++", libs=["amd_smi"]),
    Target("libnos_probe.so", ["probe.hip"], "hipcc"),
    Target("libnos_hbmlimit.so", ["hbm_limit.cpp"], "g++", flags=["-D__HIP_PLATFORM_AMD__"], libs=["dl"]),
    Target("libnos_barrier.so", ["rccl_barrier.cpp"], "g++", flags=["-D__HIP_PLATFORM_AMD__"],
           libs=["rccl", "amdhip64"]),
    Target("libnos_kernels.so", ["kernels.hip", "gemm.hip", "gemm_x3.hip", "head.hip", "attn_proj.hip", "attn_wide.hip"],
           "hipcc", source_flags={"attn_wide.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}),
    # the agent's commit-barrier helper as a native program: no interpreter start-up on the flip path
    Target("nos-gpuhelper", ["gpuhelper.cpp", "rccl_barrier.cpp", "p2p_barrier.hip"], "hipcc",
           libs=["rccl", "amdhip64"], executable=True),
    # the barrier's ring plan (csrc/ring_plan.h) as a host-only library, for its unit tests
    Target("libnos_ringplan.so", ["ring_plan_capi.cpp"], "g++"),
)


def build(force: bool = False, verbose: bool = True, jobs: int = 4) -> List[str]:
    os.makedirs(OUT, exist_ok=True)
    todo = [t for t in TARGETS if os.path.exists(os.path.join(CSRC, t.sources[0])) and (force or t.stale())]

    def run(t: Target) -> str:
        for cmd in t.commands():
            p = subprocess.run(cmd, cwd="/tmp", capture_output=True, text=True)
            if p.returncode != 0:
                raise RuntimeError(f"building {t.name} failed:\n{' '.join(cmd)}\n{p.stderr[-4000:]}")
        for s in t.source_flags:
            if os.path.exists(t._obj(s)):
                os.remove(t._obj(s))
        with open(t.stamp_path, "w") as f:
            json.dump({"library": t.name, "sha256": t.source_hash(), "arch": ARCH, "sources": t.sources}, f)
        return t.name

    built: List[str] = []
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for name in ex.map(run, todo):
            built.append(name)
            if verbose:
                print(f"[nos build] {name}", file=sys.stderr)
    return built


def target(name: str) -> Target:
    return next(t for t in TARGETS if t.name == name)


def verify(name: str) -> str:
    """The stamp hash of a built library; raises if it does not match the current sources."""
    t = target(name)
    want, got = t.source_hash(), t.read_stamp().get("sha256")
    if got != want:
        raise RuntimeError(f"{name} is stale: built from {str(got)[:12]}, sources are {want[:12]} — rebuild with "
                           "`python -c 'import __graft_entry__ as g; g.build()'`")
    return want


if __name__ == "__main__":
    build(force="--force" in sys.argv)
