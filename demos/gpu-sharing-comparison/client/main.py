"""GPU-sharing comparison client (reference demo ``demos/gpu-sharing-comparison/client/main.py``).

Endless YOLOS-small object-detection inference, batch 1, on whatever slice of an MI355X this pod
was given (a compute partition, a CU-mask slice, or a time-sliced whole GPU). Each call is timed
into the Prometheus Summary ``inference_time_seconds`` served on :8000, which the comparison
dashboards scrape through a PodMonitor.

Weights: if ``YOLOS_WEIGHTS`` points at a local safetensors file of ``hustvl/yolos-small`` they are
loaded (safetensors only, nothing executable); otherwise the architecture runs with random-init
weights, which has identical cost. Input: an 800x1066 image (``YOLOS_IMAGE`` = path to a .npy
float32 CHW array, else a synthetic one of the same shape).
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch
from prometheus_client import Summary, start_http_server

from walkai_nos_amd.models.workload.yolos import DEMO_INPUT_HW, YolosSmall, demo_input

INFERENCE_TIME = Summary("inference_time_seconds", "Time spent running one YOLOS-small inference")


def load_model(device: str) -> YolosSmall:
    m = YolosSmall()
    path = os.environ.get("YOLOS_WEIGHTS", "")
    if path:
        from safetensors.torch import load_file
        m.load_hf_state_dict(load_file(path))
    return m.to(device).eval()


def load_image(device: str) -> torch.Tensor:
    path = os.environ.get("YOLOS_IMAGE", "")
    if path:
        arr = np.load(path, allow_pickle=False).astype(np.float32)
        return torch.from_numpy(arr).unsqueeze(0).to(device)
    return demo_input(1, DEMO_INPUT_HW, device)


def main() -> None:
    device = "cuda" if torch.cuda.is_available() else "cpu"
    start_http_server(int(os.environ.get("METRICS_PORT", "8000")))
    model, x = load_model(device), load_image(device)
    n = 0
    while True:
        t0 = time.perf_counter()
        with torch.no_grad():
            logits, boxes = model(x)
        if device == "cuda":
            torch.cuda.synchronize()
        INFERENCE_TIME.observe(time.perf_counter() - t0)
        n += 1
        if n % 100 == 0:
            print(f"{n} inferences, last {1000 * (time.perf_counter() - t0):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
