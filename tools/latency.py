"""Solve latency of one pyramid call at small batches (the keyframe-VO case: kf_vo.py runs
one frame pair per forward), graph-captured, HIP events.

python tools/latency.py [--batches 1,2,4,8] [--reps 50] [--icp]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch  # noqa: E402

if os.environ.get("DPFT_LIB"):
    from deep_prob_feature_track_amd import _native as _N0
    _N0.LIB_PATH = os.path.abspath(os.environ["DPFT_LIB"])
import bench  # noqa: E402
from deep_prob_feature_track_amd import ic  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batches", default="1,2,4,8")
p.add_argument("--reps", type=int, default=50)
p.add_argument("--icp", action="store_true")
a = p.parse_args()
dev = torch.device("cuda:0")
for B in (int(b) for b in a.batches.split(",")):
    sel, levels, K = bench.make_batches(B, 0, 1, dev, a.icp)
    for d in levels:
        d["x0"], d["x1"] = ic.pack_features(d["x0"]), ic.pack_features(d["x1"])
    solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True, combine_icp=a.icp)
    pose_init = torch.cat((torch.eye(3, device=dev).repeat(B, 1, 1).reshape(-1), torch.zeros(B * 3, device=dev)))
    pose = pose_init.clone()
    R, t = pose[:9 * B].view(B, 3, 3), pose[9 * B:].view(B, 3)

    def solve():
        pose.copy_(pose_init)
        solver.run(R, t)
    solve()
    torch.cuda.synchronize()
    ic.check_status(solver.status)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        solve()
    torch.cuda.current_stream(dev).wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        solve()
    for _ in range(10):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(a.reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"B={B:3d}{' icp' if a.icp else ''}: {ms:.3f} ms per solve (graph replay, back to back), "
          f"{B * 12 / ms * 1e3:.0f} IC iterations/s", flush=True)
