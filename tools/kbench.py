"""Kernel micro-bench: time the fused reduce kernel of one level (HIP events).

python tools/kbench.py [--level 0] [--batch 8] [--reps 20]
"""
import argparse, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests", "golden")]
import torch
if os.environ.get("DPFT_LIB"):
    from deep_prob_feature_track_amd import _native as _N0
    _N0.LIB_PATH = os.path.abspath(os.environ["DPFT_LIB"])
import bench
from deep_prob_feature_track_amd import ic

p = argparse.ArgumentParser()
p.add_argument("--level", type=int, default=0)
p.add_argument("--batch", type=int, default=8)
p.add_argument("--groups", type=int, default=1, help="independent --batch-pair batches per launch (DPFT_GROUP)")
p.add_argument("--reps", type=int, default=20)
p.add_argument("--mode", choices=["reduce", "iterate", "level"], default="reduce",  # (reduce with --icp --c4: the
               # ICP pass + the U_IC reduce, two kernels; include/dpft_ic.h dpft_ic_reduce_only)
               help="level: the solve's launches at one level (iterations forward, reverse, forward)")
p.add_argument("--c4", action="store_true", help="channel-quad packed features")
p.add_argument("--schedule", default=None, help="auto | march | split (channel-quad reduce kernel)")
p.add_argument("--warm-ms", type=float, default=300.0, help="warm-up time before timing")
p.add_argument("--width", type=int, default=640,
               help="crop every level to (width >> level) columns (strip-count experiments)")
p.add_argument("--icp", action="store_true", help="cfg5: with the combine_ICP term (bench.py --icp)")
p.add_argument("--from-solve", action="store_true",
               help="start from the poses of one full pyramid solve (the bench's operating point) instead of identity")
p.add_argument("--save-poses", default=None, help="write the start poses (after --from-solve) to this .pt file")
p.add_argument("--load-poses", default=None,
               help="start from poses saved by --save-poses (a variant library whose solve is not valid, e.g. "
                    "tools/mk_loads_variant.py, replays the shipped solve's operating point)")
a = p.parse_args()
dev = torch.device("cuda:0")
sel, levels, K = bench.make_batches(a.batch, 0, a.groups, dev, a.icp)
if a.width != 640:
    levels = [{k: v[..., : a.width >> l].contiguous() for k, v in d.items()} for l, d in enumerate(levels)]
if a.c4:
    for d in levels:
        d["x0"], d["x1"] = ic.pack_features(d["x0"]), ic.pack_features(d["x1"])
solver = ic.PyramidSolver(levels, K, iters=3, remove_tru_sigma=True, combine_icp=a.icp,
                         schedule=a.schedule, group=a.batch)
R = torch.eye(3, device=dev).repeat(a.batch * a.groups, 1, 1).contiguous()
t = torch.zeros(a.batch * a.groups, 3, device=dev)
import ctypes
from deep_prob_feature_track_amd import _native as N
if a.from_solve:
    solver.run(R, t)
    torch.cuda.synchronize()
if a.load_poses:
    saved = torch.load(a.load_poses, weights_only=True)
    R.copy_(saved["R"].to(dev))
    t.copy_(saved["t"].to(dev))
if a.save_poses:
    torch.save({"R": R.cpu(), "t": t.cpu()}, a.save_poses)
solver.prepare_extrema()  # per-level sigma0 extrema slots (the levels run with EXTREMA_READY)
for level in ([a.level] if a.level >= 0 else range(len(solver.calls))):
    c = solver.calls[level]
    rc = N.lib().dpft_ic_iterate(ctypes.byref(c.desc), ctypes.byref(c.tens), ic._ptr(R.clone()), ic._ptr(t.clone()),
                                 None, None, None, 1, ic._ptr(solver.ws), solver.ws_bytes, ic._stream(dev))
    N.check(rc, "iterate")  # leaves this level's sigma0 extrema in the workspace
    torch.cuda.synchronize()
    def run_level():
        for rev in (False, True, False):
            solver.iterate(level, R, t, reverse=rev)
    run = {"reduce": lambda: solver.reduce_only(level, R, t), "iterate": lambda: solver.iterate(level, R, t),
           "level": run_level}[a.mode]
    per = 3 if a.mode == "level" else 1
    # warm-up by wall time: the GPU clocks ramp over the first tens of milliseconds of load
    # (a 60-launch loop right after start-up times ~20 % slow)
    import time
    torch.cuda.synchronize()
    tw = time.perf_counter()
    while time.perf_counter() - tw < a.warm_ms * 1e-3:
        for _ in range(3):
            run()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / (a.reps * per) * 1e3
    gbs = solver.algorithmic_bytes(level) / (us * 1e-6) / 1e9
    print(f"{os.path.basename(os.environ.get('DPFT_LIB', 'libdpft_ic.so'))}{' c4' if a.c4 else ''}{' icp' if a.icp else ''}{' ' + a.schedule if a.schedule else ''} {a.mode} level {level} B={a.batch}x{a.groups}: "
          f"{us:.1f} us/launch, {gbs:.0f} GB/s algorithmic ({gbs / 80:.1f}% of 8 TB/s)", flush=True)
