"""Experiment: two independent 8-pair solves in flight on two streams (each its own
workspace, pose buffers and HIP graph) vs one at a time.

python tools/inflight.py [--steps 100]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402

import bench  # noqa: E402
from deep_prob_feature_track_amd import ic  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--inflight", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda:0")
B = 8
ap2 = os.environ.get("INFLIGHT_SHARED_INPUTS") == "1"
inputs = []
for j in range(a.inflight):
    # distinct pairs per slot (rank j of make_inputs), unless the shared-input A/B is asked for
    _, lv, K = bench.make_inputs(B, 0 if ap2 else j, dev)
    inputs.append(([dict(d, x0=ic.pack_features(d["x0"]), x1=ic.pack_features(d["x1"])) for d in lv], K))
pose_init = torch.cat((torch.eye(3, device=dev).repeat(B, 1, 1).reshape(-1), torch.zeros(B * 3, device=dev)))


def make(j):
    levels, K = inputs[j]
    solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True)
    pose = pose_init.clone()
    R, t = pose[:9 * B].view(B, 3, 3), pose[9 * B:].view(B, 3)

    def solve():
        pose.copy_(pose_init)
        solver.run(R, t)
    solve()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        solve()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        solve()
    torch.cuda.synchronize()
    return g, R, t, solver  # the graph replays into solver.ws: keep the solver alive


slots = [make(j) for j in range(a.inflight)]
streams = [torch.cuda.Stream(dev) for _ in range(a.inflight)]


def run(n, k_inflight):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        j = i % k_inflight
        with torch.cuda.stream(streams[j]):
            slots[j][0].replay()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


# sequential determinism first: slot 0 alone, replayed
with torch.cuda.stream(streams[0]):
    slots[0][0].replay()
torch.cuda.synchronize()
Rs, ts = slots[0][1].clone(), slots[0][2].clone()
nd = 0
for rep in range(30):
    with torch.cuda.stream(streams[0]):
        slots[0][0].replay()
    torch.cuda.synchronize()
    d = max((slots[0][1] - Rs).abs().max().item(), (slots[0][2] - ts).abs().max().item())
    if d != 0:
        nd += 1
        print(f"sequential replay {rep}: max |d| {d:.3e}")
print("sequential nondeterministic replays:", nd)
for k in (1, a.inflight, 1, a.inflight):
    run(10, k)
    el = run(a.steps, k)
    print(f"in flight {k}: {el / a.steps * 1e6:.1f} us per 8-pair solve, {B * 12 * a.steps / el:.0f} IC iterations/s")
# reference: slot 0 alone, then every slot alone, then all in flight again
with torch.cuda.stream(streams[0]):
    slots[0][0].replay()
torch.cuda.synchronize()
ref = []
for j in range(a.inflight):
    with torch.cuda.stream(streams[j]):
        slots[j][0].replay()
    torch.cuda.synchronize()
    ref.append((slots[j][1].clone(), slots[j][2].clone()))
bad = 0
for rep in range(20):
    run(a.inflight * 3, a.inflight)
    for j in range(a.inflight):
        dR = (slots[j][1] - ref[j][0]).abs().max().item()
        dt = (slots[j][2] - ref[j][1]).abs().max().item()
        if dR or dt:
            bad += 1
            print(f"rep {rep} slot {j} in flight: |dR| {dR:.3e} |dt| {dt:.3e}")
print("in-flight mismatches:", bad)
