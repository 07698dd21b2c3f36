#!/usr/bin/env python
"""Benchmark: IC solver iterations/s, 640x480, C=32, 4-level pyramid (BASELINE.json).

One *step* = one full coarse-to-fine solve (levels 3..0, 3 Gauss-Newton
iterations each = 12 IC iterations per pair) of G independent batches of B frame
pairs per GPU (--groups G, --batch-per-gpu B), replayed from one HIP graph, followed
(N > 1) by the RCCL all-gather of the per-pair poses.  The G batches share every
launch (DPFT_GROUP: each batch keeps its own batch-global truncated-sigma extrema and
is solved exactly as a call of its own), so the per-launch ramp, finish spread and
finalize are paid once per G batches.  An eval stream keeps --inflight such grouped
solves in flight per GPU (distinct pairs each): step k replays slot k % inflight's
graph on that slot's stream, so one solve's latency-bound coarse levels overlap
another's bandwidth-bound level 0.  `latency_ms_per_solve` is one grouped solve with
nothing else in flight.  Workload: cfg3's shard -- B = 8 pairs per GPU per batch,
cycled from the ordered pairs of the five TUM fr1/desk frames, deterministic features
(tests/golden/recipe.py), inputs resident in HBM before the timed region.

`value` = all-level IC iterations/s over the whole job = N * G * B * 12 / step time.
Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one rank per GPU, RCCL).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

H0, W0, C, LEVELS, ITERS = 480, 640, 32, 4, 3
HBM_PEAK_GBS = 8000.0  # MI355X spec, MI355X_MICROARCH.md chip table


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--batch-per-gpu", type=int, default=8)
    p.add_argument("--setup-warm-ms", type=float, default=200.0,
                   help="setup: replay solves for this long before the --warmup steps (the GPU clock ramps over "
                        "the first tens of milliseconds of load; 5 warm-up steps are 3 ms)")
    p.add_argument("--groups", type=int, default=16,
                   help="independent B-pair batches per launch (DPFT_GROUP): each solved as its own call -- its "
                        "own batch-global truncated-sigma extrema -- in launches covering all of them")
    p.add_argument("--inflight", type=int, default=1,
                   help="grouped solves in flight per GPU (one stream, graph, workspace and input set each)")
    p.add_argument("--kernel-reps", type=int, default=50)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--layout", choices=["c4", "nchw"], default="c4",
                   help="resident feature layout the timed solve reads (c4: channel-quad, the solver's native one)")
    p.add_argument("--no-compare", action="store_true", help="skip the secondary timing of the other layout")
    return p.parse_args()


def make_group_inputs(B, G, first, device):
    """G independent B-pair batches (make_inputs `first` .. `first` + G - 1) stacked along
    the pair axis: batch g is pairs [g B, (g + 1) B) of one DPFT_GROUP(B) call."""
    parts = [make_inputs(B, first + g, device) for g in range(G)]
    if G == 1:
        return parts[0]
    sel = [p for part in parts for p in part[0]]
    levels = [{k: torch.cat([part[1][l][k] for part in parts]) for k in parts[0][1][l]} for l in range(LEVELS)]
    return sel, levels, torch.cat([part[2] for part in parts])


def make_inputs(B, rank, device):
    import recipe
    pairs = [(i, j) for i in range(5) for j in range(5) if i != j]
    sel = [pairs[(rank * B + k) % len(pairs)] for k in range(B)]
    feat = {}

    def fs(idx, l):
        if (idx, l) not in feat:
            feat[(idx, l)] = recipe.features(idx, C, l)
        return feat[(idx, l)]

    inv0 = recipe.inv_depth_batch([recipe.depth_m(i) for i, _ in sel])
    inv1 = recipe.inv_depth_batch([recipe.depth_m(j) for _, j in sel])
    levels = []
    for l in range(LEVELS):
        k = 1 << l
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        levels.append(dict(
            x0=dev(np.stack([fs(i, l)[0] for i, _ in sel])), x1=dev(np.stack([fs(j, l)[0] for _, j in sel])),
            sigma0=dev(np.stack([fs(i, l)[1] for i, _ in sel])), sigma1=dev(np.stack([fs(j, l)[1] for _, j in sel])),
            invD0=dev(recipe.max_pool(inv0, k)), invD1=dev(recipe.max_pool(inv1, k))))
    K = torch.from_numpy(np.tile(recipe.K_FULL[None], (B, 1))).to(device)
    return sel, levels, K


def l0_traffic(pairs, group):
    """Per-launch HBM bytes of the level-0 reduce launch from the committed PMC
    measurement (tools/pmc_l0.py: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes,
    gfx950-corrected), used only if it was measured on the machine code of the kernel
    built here (the ISA hash build.py records beside the library; the source file's hash
    for measurements that predate it)."""
    import glob
    import hashlib
    from deep_prob_feature_track_amd import build as B
    src = os.path.join(ROOT, "deep_prob_feature_track_amd", "csrc", "dpft_ic.hip")
    sha = hashlib.sha256(open(src, "rb").read()).hexdigest()
    isa = json.load(open(B.ISA_OUT)).get(B.L0_KERNEL) if os.path.exists(B.ISA_OUT) else None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_l0_traffic.json")), reverse=True):
        d = json.load(open(f))
        if d.get("pairs_per_launch", 8) != pairs or d.get("group", pairs) != group:
            continue  # measured on another launch shape
        if (isa is not None and d.get("isa_sha256") == isa) or d.get("src_sha256") == sha:
            return {"hbm_bytes": d["hbm_bytes"], "source": os.path.relpath(f, ROOT)}
    return None


def copy_peak_gbs(device, nbytes=1 << 30, reps=5):
    """Measured HBM copy rate (torch's copy kernel, read + write bytes / time): the
    practical ceiling SURVEY.md 8(d) asks the roofline to be reported against too."""
    x = torch.empty(nbytes // 4, dtype=torch.float32, device=device)
    y = torch.empty_like(x)
    x.fill_(1.0)
    for _ in range(2):
        y.copy_(x)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    gbs = 2 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del x, y
    return gbs


def read_peak_gbs(device, nbytes, reps=10):
    """Measured HBM read ceiling: the library's diagnostic streaming read
    (dpft_read_probe: 16-byte loads, four in flight per lane, 4096 workgroups) over a
    buffer of the level-0 launch's algorithmic size, plain and non-temporal loads;
    returns the faster, in GB/s."""
    import ctypes
    from deep_prob_feature_track_amd import _native as N, ic
    L = N.lib()
    buf = torch.ones(nbytes // 4, dtype=torch.float32, device=device)
    out = torch.empty(int(L.dpft_read_probe_out_floats()), dtype=torch.float32, device=device)
    st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    best = 0.0
    for nt in (0, 1):
        for _ in range(3):
            N.check(L.dpft_read_probe(ic._ptr(buf), buf.numel() * 4, nt, ic._ptr(out), st), "read probe")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            N.check(L.dpft_read_probe(ic._ptr(buf), buf.numel() * 4, nt, ic._ptr(out), st), "read probe")
        e1.record()
        torch.cuda.synchronize()
        best = max(best, buf.numel() * 4 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9)
    del buf, out
    return best


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_solve_seconds(lv, Kc, threads):
    """One oracle solve of one pair on `threads` host threads (no warm-up)."""
    from oracle import ic_oracle as O
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        with torch.no_grad():
            t_start = time.perf_counter()
            O.solve_pyramid(torch.eye(3)[None], torch.zeros(1, 3, 1), lv, Kc, iters=ITERS, remove_tru_sigma=True)
            return time.perf_counter() - t_start
    finally:
        torch.set_num_threads(old)


def cpu_baseline(levels_gpu, K, R_gpu, t_gpu):
    """Oracle (PyTorch-CPU restatement of the reference solver) on pair 0: 1 warm-up, best of 2."""
    from oracle import ic_oracle as O
    lv = [{k: v[:1].cpu() for k, v in d.items()} for d in levels_gpu]
    lv = [dict(f0=d["x0"], f1=d["x1"], s0=d["sigma0"], s1=d["sigma1"], invD0=d["invD0"], invD1=d["invD1"]) for d in lv]
    Kc = K[:1].cpu()
    R0 = torch.eye(3)[None]
    t0 = torch.zeros(1, 3, 1)
    best = float("inf")
    out = None
    with torch.no_grad():
        for rep in range(3):
            t_start = time.perf_counter()
            out = O.solve_pyramid(R0, t0, lv, Kc, iters=ITERS, remove_tru_sigma=True)
            el = time.perf_counter() - t_start
            if rep > 0:
                best = min(best, el)
    one_thread = cpu_solve_seconds(lv, Kc, 1)
    Ro, to = out
    dR = (R_gpu[:1].cpu() - Ro).abs().max().item()
    dt = (t_gpu[:1].cpu().view(1, 3) - to.view(1, 3)).abs().max().item()
    # 3D end-point error between the two poses over frame-0 points (criterions.py:101-136)
    from deep_prob_feature_track_amd.metrics import epe3d_between, rpe
    d0 = 1.0 / lv[0]["invD0"].clamp(min=1e-6)
    epe = epe3d_between(R_gpu[:1].cpu(), t_gpu[:1].cpu().view(1, 3), Ro, to.view(1, 3), d0,
                        Kc, invalid=(lv[0]["invD0"] <= 0)).item()
    # translational relative pose error between the two estimates (criterions.py
    # compute_RPE_loss; its angle term is floored at acos(1 - 1e-7) = 4.5e-4 rad by the
    # reference's clamp, so the rotation is reported as max |dR| above)
    _, trs = rpe(R_gpu[:1].cpu(), t_gpu[:1].cpu().view(1, 3), Ro, to.view(1, 3))
    return best, dR, dt, epe, one_thread, trs.item()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs (tests of the N > 1 logic on a 1-GPU box): DPFT_BENCH_BACKEND=gloo
    # and DPFT_BENCH_SHARE_GPU=1 put every rank on cuda:0; the driver's runs use neither
    if os.environ.get("DPFT_BENCH_SHARE_GPU"):
        local = 0
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("DPFT_BENCH_BACKEND", "nccl"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if os.environ.get("DPFT_LIB"):  # A/B runs of compile-time variants (tools/build_variants.py)
        from deep_prob_feature_track_amd import _native
        _native.LIB_PATH = os.path.abspath(os.environ["DPFT_LIB"])
    from deep_prob_feature_track_amd import ic, shard

    B = a.batch_per_gpu
    G = max(1, a.groups)
    S = max(1, a.inflight)
    BG = B * G  # pairs per launch
    # batch g of slot j of this rank: the pairs of make_inputs "rank" (rank * S + j) * G + g
    # (distinct pairs per batch, slot and rank, cycled through the 20 ordered pairs of the 5 frames)
    slot_inputs = [make_group_inputs(B, G, (rank * S + j) * G, device) for j in range(S)]
    sel, levels_nchw, K = slot_inputs[0]

    def packed(levels):
        return [dict(d, x0=ic.pack_features(d["x0"]), x1=ic.pack_features(d["x1"])) for d in levels]

    def pack_time_us(levels, reps=10):
        """One-time NCHW -> channel-quad conversion of both feature pyramids (not in the step)."""
        packed(levels)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            packed(levels)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    levels = packed(levels_nchw) if a.layout == "c4" else levels_nchw
    # R [B,3,3] and t [B,3] as two contiguous views of one buffer: one reset copy per step
    pose_init = torch.cat((torch.eye(3, device=device).repeat(BG, 1, 1).reshape(-1), torch.zeros(BG * 3, device=device)))

    def make_step(levels, K=K):
        solver = ic.PyramidSolver(levels, K, iters=ITERS, remove_tru_sigma=True, group=B,
                                  schedule=os.environ.get("DPFT_BENCH_SCHEDULE"))  # A/B only
        pose = pose_init.clone()
        R, t = pose[:9 * BG].view(BG, 3, 3), pose[9 * BG:].view(BG, 3)

        def solve():
            pose.copy_(pose_init)
            solver.run(R, t)

        # eager warm-up (also validates), then capture the whole 4-level solve into one graph
        solve()
        torch.cuda.synchronize()
        ic.check_status(solver.status)
        graph = None
        if not a.no_graph:
            s = torch.cuda.Stream(device)
            s.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(s):
                solve()
            torch.cuda.current_stream(device).wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                solve()
            torch.cuda.synchronize()

        def run():
            if graph is not None:
                graph.replay()
            else:
                solve()
        return solver, R, t, run, graph is not None

    # S in-flight slots: slot j solves its own batch on its own stream from its own HIP
    # graph and workspace; step k runs on slot k % S, so a batch's latency-bound coarse
    # levels and finalizes overlap another batch's bandwidth-bound level 0
    slots = []
    for j in range(S):
        lv = levels if j == 0 else (packed(slot_inputs[j][1]) if a.layout == "c4" else slot_inputs[j][1])
        slots.append(make_step(lv, slot_inputs[j][2]))
    streams = [torch.cuda.Stream(device) for _ in range(S)]
    solver, R, t, run, graphed = slots[0]
    # N > 1: the pose gather of step k runs on the collective stream while step k + 1
    # solves (double-buffered output; poses packed into a fresh buffer first, on the
    # slot's stream); every gather is waited for inside the timed region (drain())
    gathered = [torch.empty(world * BG, 12, device=device) for _ in range(2)] if world > 1 else None
    pending = [None]
    nstep = [0]

    def drain():
        if pending[0] is not None:
            pending[0].wait()
            pending[0] = None

    def step():
        j = nstep[0] % S
        with torch.cuda.stream(streams[j]):
            slots[j][3]()
            if world > 1:
                drain()
                _, pending[0] = shard.gather_poses(slots[j][1], slots[j][2], out=gathered[nstep[0] % 2],
                                                   async_op=True)
        nstep[0] += 1

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    # setup warm-up by wall time (untimed, before the W warm-up steps): a few ms of load
    # leave the chip below its steady clock (MI355X_MICROARCH.md, DVFS) -- measured 141 k
    # vs 150 k IC iterations/s for 20 timed steps after 5 vs 300 warm-up steps.  Solves
    # only, no pose gathers: the ranks run different numbers of these rounds, and a
    # collective issued by one rank and not the other would deadlock.
    torch.cuda.synchronize()
    tw = time.perf_counter()
    while time.perf_counter() - tw < a.setup_warm_ms * 1e-3:
        for j in range(S):
            with torch.cuda.stream(streams[j]):
                slots[j][3]()
        torch.cuda.synchronize()
    for _ in range(a.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch.distributed as dist
        e = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = e.item()
    for sl in slots:
        ic.check_status(sl[0].status)
    ms_per_step = elapsed / a.steps * 1e3
    iters_total = world * BG * LEVELS * ITERS * a.steps
    value = iters_total / elapsed
    # latency of one solve (slot 0 alone, back to back on one stream), rank 0 only
    latency_ms = None
    if rank == 0:
        n_lat = min(a.steps, 50)
        torch.cuda.synchronize()
        tl0 = time.perf_counter()
        for _ in range(n_lat):
            run()
        torch.cuda.synchronize()
        latency_ms = (time.perf_counter() - tl0) / n_lat * 1e3

    # ---- roofline of the dominant kernel: the level-0 fused reduce (+ its in-kernel
    # finalize), i.e. exactly the launches the solve makes at level 0 -- iterations
    # forward, reverse, forward (DPFT_ITER_REVERSE), the group repeated -- continuing
    # from the solved pose; timed with HIP events on the stream they are launched on
    # (the current stream).
    Rk, tk = R.clone(), t.clone()
    solver.iterate(0, Rk, tk, first=True)
    l0_group = [False, True, False]
    for rev in l0_group:
        solver.iterate(0, Rk, tk, reverse=rev)
    groups = max(1, a.kernel_reps // len(l0_group))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(groups):
        for rev in l0_group:
            solver.iterate(0, Rk, tk, reverse=rev)
    ev1.record()
    torch.cuda.synchronize()
    kern_us = ev0.elapsed_time(ev1) / (groups * len(l0_group)) * 1e3
    alg_bytes = solver.algorithmic_bytes(0)
    achieved = alg_bytes / (kern_us * 1e-6) / 1e9
    traffic = l0_traffic(BG, B) if a.layout == "c4" else None
    copy_gbs = copy_peak_gbs(device) if rank == 0 else None
    read_gbs = read_peak_gbs(device, alg_bytes) if rank == 0 else None

    # secondary (rank 0 only, not the headline): the same solve from the other resident
    # layout, and the one-time cost of packing NCHW pyramids into the channel-quad layout
    other = None
    if rank == 0 and not a.no_compare:
        other_layout = "nchw" if a.layout == "c4" else "c4"
        o_solver, o_R, o_t, o_run, _ = make_step(levels_nchw if other_layout == "nchw" else packed(levels_nchw))
        for _ in range(a.warmup):
            o_run()
        torch.cuda.synchronize()
        tt0 = time.perf_counter()
        for _ in range(a.steps):
            o_run()
        torch.cuda.synchronize()
        o_el = time.perf_counter() - tt0
        dpose = max((o_R - R).abs().max().item(), (o_t - t).abs().max().item())
        other = {"layout": other_layout, "ms_per_step": o_el / a.steps * 1e3,
                 "value": BG * LEVELS * ITERS * a.steps / o_el, "max_abs_pose_diff_vs_headline": dpose,
                 "pack_us_all_levels_both_frames": pack_time_us(levels_nchw)}
        del o_solver

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        best, dR, dt, epe, one_thread, rpe_trs = cpu_baseline(levels_nchw, K, R, t)
        cpu = {"value": LEVELS * ITERS / best, "unit": "IC iterations/s",
               "cores": torch.get_num_threads(), "kind": "port", "cpu_model": cpu_model(),
               "value_1_thread": LEVELS * ITERS / one_thread, "seconds_per_pair_1_thread": one_thread,
               "sample": "1 pair, 640x480 C=32, 4 levels x 3 iters, oracle/ic_oracle.py (PyTorch-CPU fp32 "
                         "restatement of algorithms.py:611-723), best of 2 after 1 warm-up",
               "seconds_per_pair": best, "gpu_vs_oracle_max_abs_dR": dR, "gpu_vs_oracle_max_abs_dt": dt,
               "gpu_vs_oracle_3dpe_m": epe, "gpu_vs_oracle_rpe_trans_m": rpe_trs}

    if rank == 0:
        line = {
            "metric": "IC solver iters/sec (640x480, C=32, 4-level)",
            "value": value, "unit": "IC iterations/s (all levels, 12 per pair)",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: deterministic triangle-wave features of the 5 TUM fr1/desk example frames",
            "config": {"workload": "cfg2/cfg3 shard: 640x480, C=32, Cs=1, 4 levels x 3 GN iters, "
                                   "remove_tru_sigma, batches of B pairs per GPU", "pairs_per_gpu": B,
                       "global_batch": world * B, "parallelism": f"pair-sharded x{world}, RCCL all-gather of poses",
                       "graph": graphed, "feature_layout": a.layout,
                       "batches_per_launch": G, "pairs_per_launch": BG, "inflight": S,
                       "setup_warm_ms": a.setup_warm_ms},
            "latency_ms_per_solve": latency_ms,
            "pairs_per_s": world * BG * a.steps / elapsed,
            "l0_iters_per_s": world * BG * ITERS * a.steps / elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic["hbm_bytes"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel": f"ic_reduce_kernel<32,Cs=1,tru,U_IC,{a.layout}> (level 0, + in-kernel finalize)",
                         "kernel_us": kern_us, "algorithmic_bytes_per_launch": alg_bytes,
                         "measured_copy_peak": copy_gbs,
                         "frac_of_measured_copy_peak": achieved / copy_gbs if copy_gbs else None,
                         "measured_read_peak": read_gbs,
                         "frac_of_measured_read_peak": achieved / read_gbs if read_gbs else None},
            "cpu_baseline": cpu,
            "other_layout": other,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
