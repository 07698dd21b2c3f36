"""Time the drop-in `LeastSquareTracking.forward` on the GPU at the bench's shape
(B = 8, 640x480, C = 32, Cs = 1, ConvRGBD2 / laplacian, remove_tru_sigma; random
encoder weights): the whole forward, its `_preprocess` (encoder, pyramids, depth) and
the solver levels (forward minus preprocess).

python tools/dropin_timing.py [--reps 20]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import recipe  # noqa: E402
from deep_prob_feature_track_amd.models.LeastSquareTracking import LeastSquareTracking, default_options  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--config", default="uic", choices=["uic", "uic8", "deepic"],
                help="uic: ConvRGBD2 + laplacian U_IC tracker, C=32 (uic8: C=8); deepic: RGB features, IC tracker, "
                     "MultiScale2w M-estimator, Direct-ResVol")
ap.add_argument("--down", type=int, default=1, help="image subsampling (1: 640x480)")
ap.add_argument("--compile", default="", help="also time torch.compile(model, backend=...) (comma list, e.g. "
                                               "aot_eager,cudagraphs)")
a = ap.parse_args()
dev = torch.device("cuda:0")
if os.environ.get("DPFT_DROPIN_BENCHMARK"):  # MIOpen algorithm search for the encoder convs
    torch.backends.cudnn.benchmark = True
torch.manual_seed(0)
if a.config in ("uic", "uic8"):
    m = LeastSquareTracking("ConvRGBD2", "laplacian", 3, "None", "Direct-Nodamping",
                            options=default_options(feature_channel=32 if a.config == "uic" else 8,
                                                    uncertainty_channel=1, feature_extract="conv",
                                                    remove_tru_sigma=True)).to(dev).eval()
else:
    m = LeastSquareTracking("RGB", "None", 3, "MultiScale2w", "Direct-ResVol",
                            options=default_options(feature_channel=1)).to(dev).eval()
B = a.batch
pairs = [(i % 5, (i + 1 + i // 5) % 5) for i in range(B)]
img0 = torch.stack([torch.from_numpy(recipe.color_float(i, a.down)) for i, _ in pairs]).to(dev)
img1 = torch.stack([torch.from_numpy(recipe.color_float(j, a.down)) for _, j in pairs]).to(dev)
d0 = torch.stack([torch.from_numpy(recipe.depth_m(i, a.down)) for i, _ in pairs])[:, None].to(dev)
d1 = torch.stack([torch.from_numpy(recipe.depth_m(j, a.down)) for _, j in pairs])[:, None].to(dev)
K = torch.tensor(recipe.K_FULL / a.down, device=dev).view(1, 4).repeat(B, 1)


def timed(fn):
    with torch.no_grad():
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / a.reps * 1e3


full = timed(lambda: m.forward(img0, img1, d0, d1, K))
if os.environ.get("DPFT_DROPIN_GRAPH"):  # the whole forward captured into one HIP graph
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m.forward(img0, img1, d0, d1, K)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            m.forward(img0, img1, d0, d1, K)
    gr = timed(graph.replay)
    print(f"forward as one HIP graph replay: {gr:.2f} ms per call (eager {full:.2f} ms)", flush=True)
if a.compile:  # torch.compile over the dpft:: ops (torch_ops.py): one traced graph, no code generation
    m.requires_grad_(False)  # an inference module: no autograd state for the graph backends to track
    for backend in a.compile.split(","):
        torch._dynamo.reset()
        mc = torch.compile(m, backend=backend)

        def call():
            if backend == "cudagraphs":
                torch.compiler.cudagraph_mark_step_begin()
            return mc(img0, img1, d0, d1, K)
        with torch.no_grad():
            Re, te = m.forward(img0, img1, d0, d1, K)
            for _ in range(3):
                Rc, tc = call()
            diff = max((Re - Rc).abs().max().item(), (te - tc).abs().max().item())
        cm = timed(call)
        print(f"torch.compile(backend={backend}): {cm:.2f} ms per call (eager {full:.2f} ms); "
              f"max |pose - eager pose| {diff:.1e}", flush=True)
pre = timed(lambda: m._preprocess(img0, img1, d0, d1))
H, W = img0.shape[2:]
print(f"drop-in forward ({a.config}) B={B} {W}x{H}: {full:.2f} ms per call; _preprocess {pre:.2f} ms; "
      f"solver levels {full - pre:.2f} ms", flush=True)

if os.environ.get("DPFT_DROPIN_PROFILE"):
    from torch.profiler import ProfilerActivity, profile
    with torch.no_grad(), profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        for _ in range(3):
            m.forward(img0, img1, d0, d1, K)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25), flush=True)
    print(prof.key_averages().table(sort_by="cpu_time_total", row_limit=25), flush=True)
