"""Where a pod process's start-up goes (the ``pod_start`` the bench charges, ``bench_core.measure_pod_start``):
the pod client's boot (``dataplane/client.py``) phase by phase, in a fresh process with the environment
``Allocate`` gives a 1/8-GPU slice. Prints one JSON line of seconds per phase.

    python tools/pod_start_probe.py [--slice 32cu.36gb] [--out gpurun_out/pod_start_probe.json]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHILD = r"""
import json, time
t = [("start", time.perf_counter())]
import torch
t.append(("import_torch", time.perf_counter()))
from walkai_nos_amd.models.workload.yolos import YolosSmall, demo_input
from walkai_nos_amd.ops import kernels as K
K.set_backend("hip")
t.append(("import_nos", time.perf_counter()))
torch.zeros(1, device="cuda:0")
torch.cuda.synchronize()
t.append(("hip_init", time.perf_counter()))
model = YolosSmall()
t.append(("model_init_cpu", time.perf_counter()))
model = model.to("cuda:0").eval()
x = demo_input(1, (800, 1066), "cuda:0", seed=0)
torch.cuda.synchronize()
t.append(("to_device", time.perf_counter()))
s = torch.cuda.Stream()
with torch.no_grad(), torch.cuda.stream(s):
    model(x)
s.synchronize()
t.append(("first_inference", time.perf_counter()))
with torch.no_grad(), torch.cuda.stream(s):
    model(x)
s.synchronize()
t.append(("second_inference", time.perf_counter()))
g = torch.cuda.CUDAGraph()
with torch.no_grad(), torch.cuda.graph(g, stream=s):
    model(x)
s.synchronize()
t.append(("graph_capture", time.perf_counter()))
t0 = time.perf_counter()
g.replay(); s.synchronize()
t.append(("first_replay", time.perf_counter()))
print(json.dumps({k: round(v - t[i][1], 3) for i, (k, v) in enumerate(t[1:])}))
"""


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--slice", default="32cu.36gb")
    ap.add_argument("--runs", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from walkai_nos_amd.dataplane.procs import allocate_envs
    env = dict(os.environ)
    env.update(allocate_envs([a.slice])[0])
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    runs = []
    for _ in range(a.runs):
        t0 = time.perf_counter()
        r = subprocess.run([sys.executable, "-c", CHILD], cwd=ROOT, env=env, capture_output=True, text=True,
                           timeout=300)
        wall = time.perf_counter() - t0
        line = next((x for x in reversed(r.stdout.splitlines()) if x.startswith("{")), None)
        if r.returncode != 0 or line is None:
            print(r.stdout[-2000:], r.stderr[-3000:], file=sys.stderr)
            return 1
        phases = json.loads(line)
        runs.append({"wall_s": round(wall, 3), "phases_s": phases,
                     "interpreter_and_exit_s": round(wall - sum(phases.values()), 3)})
        print(json.dumps(runs[-1]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"slice": a.slice, "runs": runs}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
