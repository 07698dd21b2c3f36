#!/usr/bin/env python
"""Benchmark: IC solver iterations/s, 640x480, C=32, 4-level pyramid (BASELINE.json).

Workload (default, cfg3): an eval stream of global batches of 64 frame pairs; one *step* =
one global batch, sharded contiguously over the N ranks (64 / N pairs each, strong
scaling), each rank solving its shard as independent batches of B = 8 pairs (one
reference call each: its own batch-global truncated-sigma extrema) in ONE grouped call
(DPFT_GROUP): levels 3..0, 3 Gauss-Newton iterations each = 12 IC iterations per pair,
replayed from one HIP graph, then (N > 1) the RCCL all-gather of the per-pair poses.
`--inflight S` keeps S consecutive global batches of the stream in flight per GPU (one
stream, graph and input set each), so one batch's latency-bound coarse levels overlap the
next one's bandwidth-bound level 0.  `--pairs-per-gpu P` switches to weak scaling (P
pairs per GPU per step).  `--icp`: cfg5, the same with the combine_ICP term.

Pairs are cycled from the 20 ordered pairs of the five TUM fr1/desk frames, features are
the deterministic recipe of tests/golden/recipe.py (the checkpoints are absent), inputs
are resident in HBM (channel-quad layout) before the timed region.
`value` = all-level IC iterations/s of the whole job = pairs per step * 12 / step time.
Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 under
torch.distributed.run (one rank per GPU, RCCL).
"""
import argparse
import ctypes
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
    p.add_argument("--global-batch", type=int, default=64,
                   help="pairs per step over all ranks (cfg3: 64), sharded contiguously -- strong scaling")
    p.add_argument("--pairs-per-gpu", type=int, default=0,
                   help="> 0: weak scaling instead, this many pairs per GPU per step")
    p.add_argument("--batch", type=int, default=8,
                   help="pairs per independent batch (one reference call: its own batch-global extrema)")
    p.add_argument("--inflight", type=int, default=0,
                   help="calls of the stream in flight per GPU (one stream, graph, workspace each; 0: 2, "
                        "with --icp 4 -- the combine_ICP pass's latency-bound launches overlap the other "
                        "calls' reduce launches, measured +1.5-3.5 %% against 2, DESIGN.md 4.4)")
    p.add_argument("--stream-group", type=int, default=0,
                   help="global batches of the stream per grouped call on each rank (0: enough for "
                        "--min-launch-pairs pairs per call)")
    p.add_argument("--min-launch-pairs", type=int, default=128,
                   help="stream grouping target: pairs per call and rank (at N = 1 a call holds two 64-pair "
                        "global batches; measured +1.5 %% against one batch per call with 4 in flight, DESIGN.md 4.8)")
    p.add_argument("--icp", action="store_true", help="cfg5: with the combine_ICP term (weight 0.01)")
    p.add_argument("--setup-warm-ms", type=float, default=200.0,
                   help="setup: replay solves for this long before the --warmup steps (the GPU clock ramps over "
                        "the first tens of milliseconds of load)")
    p.add_argument("--kernel-reps", type=int, default=30)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--layout", choices=["c4", "nchw"], default="c4",
                   help="resident feature layout the timed solve reads (c4: channel-quad, the solver's native one)")
    p.add_argument("--no-compare", action="store_true", help="skip the secondary timings (other layout, end-to-end)")
    return p.parse_args()


# ---------------------------------------------------------------------------- inputs
def make_batches(B, first, count, device, icp=False):
    """`count` consecutive independent batches of B pairs, batch q (q = first .. first +
    count - 1) holding stream pairs q B .. q B + B - 1, stacked along the pair axis:
    (pairs, per-level NCHW dicts, K [count B, 4]).  Stream pair n is ordered pair n mod 20
    of the five frames with flip code (n div 20) mod 4 (left-right / up-down, both frames
    alike: recipe.flip_case), so the cfg3 batch of 64 holds 64 distinct pairs (SURVEY.md
    8d); pairs 0..19 are unflipped (the reference fixture of batch 0)."""
    import recipe
    n_ord = len(recipe.ORDERED_PAIRS)
    sel, levels = [], [dict() for _ in range(LEVELS)]
    for q in range(first, first + count):
        bsel = [recipe.ORDERED_PAIRS[(q * B + k) % n_ord] for k in range(B)]
        flips = [((q * B + k) // n_ord) % 4 for k in range(B)]
        sel += bsel
        d0 = [recipe.depth_m(i) for i, _ in bsel]
        d1 = [recipe.depth_m(j) for _, j in bsel]
        inv0, inv1 = recipe.inv_depth_batch(d0), recipe.inv_depth_batch(d1)  # per reference call
        for l in range(LEVELS):
            k = 1 << l
            part = dict(x0=np.stack([recipe.features(i, C, l)[0] for i, _ in bsel]),
                        x1=np.stack([recipe.features(j, C, l)[0] for _, j in bsel]),
                        sigma0=np.stack([recipe.features(i, C, l)[1] for i, _ in bsel]),
                        sigma1=np.stack([recipe.features(j, C, l)[1] for _, j in bsel]),
                        invD0=recipe.max_pool(inv0, k), invD1=recipe.max_pool(inv1, k))
            if icp:
                part["depth0"] = recipe.max_pool(np.stack(d0)[:, None], k)
                part["depth1"] = recipe.max_pool(np.stack(d1)[:, None], k)
            for key, v in part.items():
                if any(flips):
                    v = v.copy()  # (level 0's max_pool may return its input, shared by all levels)
                for b, code in enumerate(flips):
                    if code & 1:
                        v[b] = v[b][..., ::-1].copy()
                    if code & 2:
                        v[b] = v[b][..., ::-1, :].copy()
                levels[l].setdefault(key, []).append(v)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(np.concatenate(a))).to(device)
    levels = [{k: dev(v) for k, v in d.items()} for d in levels]
    K = torch.from_numpy(np.tile(recipe.K_FULL[None], (B * count, 1))).to(device)
    return sel, levels, K


def l0_traffic(pairs, group, kernel, icp=False):
    """Per-launch HBM bytes of the level-0 reduce launch from the committed PMC measurement
    (tools/pmc_l0.py: separate FETCH_SIZE / WRITE_SIZE rocprofv3 passes, gfx950-corrected),
    used only if it was measured on the machine code of the kernel built here (the ISA hash
    build.py records beside the library) and on the same launch shape."""
    import glob
    from deep_prob_feature_track_amd import build as Bd
    hashes = json.load(open(Bd.ISA_OUT)) if os.path.exists(Bd.ISA_OUT) else {}
    isa = hashes.get(kernel)
    isa_icp = hashes.get(Bd.ICP_KERNEL) if icp else None  # the cfg5 iteration: the ICP pass too
    if isa is None or (icp and isa_icp is None):
        return None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_l0_traffic.json")), reverse=True):
        d = json.load(open(f))
        if (d.get("level", 0) == 0 and d.get("pairs_per_launch", 8) == pairs and d.get("group", pairs) == group
                and d.get("kbench_mode", "level") == "level"
                and d.get("isa_sha256") == isa
                and bool(d.get("combine_icp", False)) == icp and d.get("isa_sha256_icp") == isa_icp):
            return {"hbm_bytes": d["hbm_bytes"], "source": os.path.relpath(f, ROOT)}
    return None


def _timed(fn, reps, device):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize(device)
    return e0.elapsed_time(e1) * 1e-3 / reps


def copy_peak_gbs(device, nbytes=1 << 30, reps=10):
    """Measured HBM copy ceiling: the library's float4 copies (dpft_copy_probe: one 16-byte
    element per thread, and a grid-stride non-temporal variant), read + write bytes / time of
    the faster."""
    from deep_prob_feature_track_amd import _native as N, ic
    L = N.lib()
    x = torch.ones(nbytes // 4, dtype=torch.float32, device=device)
    y = torch.empty_like(x)
    st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    best = 0.0
    for mode in (0, 1):
        run = lambda: N.check(L.dpft_copy_probe(ic._ptr(x), ic._ptr(y), nbytes, mode, st), "copy probe")
        for _ in range(3):
            run()
        best = max(best, 2 * nbytes / _timed(run, reps, device) / 1e9)
    del x, y
    return best


def read_peak_gbs(device, nbytes, reps=10):
    """Measured HBM read ceiling: dpft_read_probe (16-byte loads, four in flight per lane)
    over a buffer of the level-0 launch's algorithmic size, plain and non-temporal loads;
    the faster, in GB/s."""
    from deep_prob_feature_track_amd import _native as N, ic
    L = N.lib()
    buf = torch.ones(nbytes // 4, dtype=torch.float32, device=device)
    out = torch.empty(int(L.dpft_read_probe_out_floats()), dtype=torch.float32, device=device)
    st = ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    best = 0.0
    for nt in (0, 1):
        run = lambda: N.check(L.dpft_read_probe(ic._ptr(buf), buf.numel() * 4, nt, ic._ptr(out), st), "read probe")
        for _ in range(3):
            run()
        best = max(best, buf.numel() * 4 / _timed(run, reps, device) / 1e9)
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


def host_cpus():
    """CPUs this process may use: its affinity set, capped by the cgroup CPU quota (a GPU box
    grants a share of the host; os.cpu_count() is the whole machine, and that many threads on
    a 16-CPU quota spin far slower than 16)."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------- parity + CPU baseline
def oracle_solve(lv_cpu, Kc, threads, icp):
    """One oracle solve (PyramidSolver's schedule) of the given batch on `threads` host
    threads; (R, t, seconds)."""
    from oracle import ic_oracle as O
    old = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        B = Kc.shape[0]
        with torch.no_grad():
            t_start = time.perf_counter()
            R, t = O.solve_pyramid(torch.eye(3).repeat(B, 1, 1), torch.zeros(B, 3, 1), lv_cpu, Kc, iters=ITERS,
                                   remove_tru_sigma=True, combine_icp=icp)
            return R, t.view(B, 3), time.perf_counter() - t_start
    finally:
        torch.set_num_threads(old)


def cpu_baseline(levels_gpu, K, R_gpu, t_gpu, B, icp, samples=3):
    """The oracle (PyTorch-CPU restatement of algorithms.py:611-723) on batch 0 of slot 0 --
    the same B pairs, one reference call, so the batch-global extrema match the GPU's batch
    -- at every available host CPU, and one pair on one thread: each one warm-up run, then
    the best of `samples` timed runs; the warm-up run of the batch is the
    parity sample.  Parity over all B pairs: max |dR|, |dt|, 3D EPE and translational RPE
    between the GPU and the oracle poses; and the GPU poses against the reference's own run
    of this batch (tests/golden/cfg3_b8_640x480_c32.npz) when the batch is that fixture's."""
    from deep_prob_feature_track_amd.metrics import epe3d_between, rpe
    cpu = lambda d: {k: v[:B].cpu() for k, v in d.items()}
    lv = [dict(f0=d["x0"], f1=d["x1"], s0=d["sigma0"], s1=d["sigma1"], invD0=d["invD0"], invD1=d["invD1"],
               **({"depth0": d["depth0"], "depth1": d["depth1"]} if icp else {})) for d in map(cpu, levels_gpu)]
    Kc = K[:B].cpu()
    threads = host_cpus()
    Ro, to, sec_warm = oracle_solve(lv, Kc, threads, icp)  # warm-up + the parity poses
    secs = [oracle_solve(lv, Kc, threads, icp)[2] for _ in range(samples)]
    sec = min(secs)
    lv1 = [{k: v[:1] for k, v in d.items()} for d in lv]  # timing sample only
    sec1_warm = oracle_solve(lv1, Kc[:1], 1, icp)[2]
    secs1 = [oracle_solve(lv1, Kc[:1], 1, icp)[2] for _ in range(samples)]
    sec1 = min(secs1)
    Rg, tg = R_gpu[:B].cpu(), t_gpu[:B].cpu().view(B, 3)
    d0 = 1.0 / lv[0]["invD0"].clamp(min=1e-6)
    epe = epe3d_between(Rg, tg, Ro, to, d0, Kc, invalid=(lv[0]["invD0"] <= 0))
    _, trs = rpe(Rg, tg, Ro, to)
    out = {"value": B * LEVELS * ITERS / sec, "unit": "IC iterations/s", "cores": threads, "kind": "port",
           "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
           "sample": f"oracle solves of the {B}-pair batch 0 (640x480 C=32, 4 levels x 3 iters, "
                     f"{'combine_ICP, ' if icp else ''}oracle/ic_oracle.py), {threads} threads: the best of "
                     f"{samples} after one warm-up",
           "warmup": 1, "samples": samples,
           "seconds_per_batch": sec, "seconds_per_batch_runs": secs, "seconds_warmup": sec_warm,
           "value_1_thread": LEVELS * ITERS / sec1,
           "sample_1_thread": f"one pair, one thread: the best of {samples} after one warm-up",
           "seconds_per_pair_1_thread": sec1, "seconds_per_pair_1_thread_runs": secs1,
           "seconds_warmup_1_thread": sec1_warm,
           "parity_pairs": B,
           "gpu_vs_oracle_max_abs_dR": (Rg - Ro).abs().max().item(),
           "gpu_vs_oracle_max_abs_dt": (tg - to).abs().max().item(),
           "gpu_vs_oracle_3dpe_m_max": epe.max().item(), "gpu_vs_oracle_3dpe_m_mean": epe.mean().item(),
           "gpu_vs_oracle_rpe_trans_m_max": trs.max().item()}
    golden = os.path.join(ROOT, "tests", "golden", "cfg3_b8_640x480_c32.npz")
    if not icp and B == 8 and os.path.exists(golden):
        import recipe
        z = np.load(golden, allow_pickle=False)
        if [tuple(p) for p in recipe.CASES["cfg3_b8_640x480_c32"]["pairs"]] == \
                [recipe.ORDERED_PAIRS[k] for k in range(8)]:
            for prec in ("f32", "f64"):
                out[f"gpu_vs_reference_{prec}_max_abs_dR"] = float(np.abs(Rg.numpy() - z[f"{prec}_R"][-1]).max())
                out[f"gpu_vs_reference_{prec}_max_abs_dt"] = float(np.abs(tg.numpy() - z[f"{prec}_t"][-1]).max())
            out["reference_fixture"] = "tests/golden/cfg3_b8_640x480_c32.npz (the reference's own run of batch 0)"
    return out


# ---------------------------------------------------------------------------- main
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
    from deep_prob_feature_track_amd import build as Bd, ic, shard

    S = max(1, a.inflight if a.inflight > 0 else (4 if a.icp else 2))
    weak = a.pairs_per_gpu > 0
    if weak:
        n_r = a.pairs_per_gpu
        per_step = world * n_r
        begin = 0
        step_first = lambda k: (rank * 1_000_000 + k) * max(1, n_r // a.batch)  # this rank's own stream
    else:
        per_step = a.global_batch
        begin, end = shard.shard_range(per_step, world, rank)
        n_r = end - begin
        if n_r < 1:
            raise SystemExit(f"global batch {per_step} < {world} ranks")
        step_first = lambda k: k * max(1, per_step // a.batch) + begin // a.batch  # global batch k's shard
    B = a.batch if n_r % a.batch == 0 and (weak or begin % a.batch == 0) else n_r
    G = n_r // B  # independent batches per step (DPFT_GROUP)
    # stream grouping: a rank solves Q consecutive global batches of the stream in ONE grouped
    # call (each batch still its own reference call), so that a call holds >= --min-launch-pairs
    # pairs whatever the shard size -- the N = 8 rank load (8 pairs per global batch) then runs
    # the same 64-pair launches as N = 1 instead of 8-pair launches
    Q = a.stream_group if a.stream_group > 0 else shard.stream_group(n_r, B, a.min_launch_pairs)
    calls_for = lambda steps: shard.stream_calls(steps, Q)

    def inputs_for(call_idx, q):
        """Inputs of call `call_idx` (q global batches: steps call_idx * Q .. + q - 1)."""
        parts = [make_batches(B, step_first(call_idx * Q + k), G, device, a.icp) for k in range(q)]
        if q == 1:
            return parts[0]
        return (sum((p_[0] for p_ in parts), []),
                [{k: torch.cat([p_[1][l][k] for p_ in parts]) for k in parts[0][1][l]} for l in range(LEVELS)],
                torch.cat([p_[2] for p_ in parts]))
    slot_inputs = [inputs_for(j, Q) for j in range(S)]
    sel, levels_nchw, K = slot_inputs[0]

    def packed(levels):
        return [dict(d, x0=ic.pack_features(d["x0"]), x1=ic.pack_features(d["x1"])) for d in levels]

    def capture(fn):
        fn()
        torch.cuda.synchronize()
        if a.no_graph:
            return fn
        s_ = torch.cuda.Stream(device)
        s_.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s_):
            fn()
        torch.cuda.current_stream(device).wait_stream(s_)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            fn()
        torch.cuda.synchronize()
        return graph.replay

    def make_step(levels, K, pre=None):
        """A call's solver, pose buffers and graph-captured solve (every pair from identity)."""
        n = K.shape[0]
        pose_init = torch.cat((torch.eye(3, device=device).repeat(n, 1, 1).reshape(-1),
                               torch.zeros(n * 3, device=device)))
        solver = ic.PyramidSolver(levels, K, iters=ITERS, remove_tru_sigma=True, combine_icp=a.icp,
                                  group=B if n > B else None)
        pose = pose_init.clone()
        R, t = pose[:9 * n].view(n, 3, 3), pose[9 * n:].view(n, 3)

        def solve():
            if pre is not None:
                pre()
            pose.copy_(pose_init)
            solver.run(R, t)
        solve()
        torch.cuda.synchronize()
        ic.check_status(solver.status)
        solver.bench_keep = (pose_init, pose, pre)  # a captured graph reads them (pre: its buffers): keep alive
        return solver, R, t, capture(solve)

    slot_levels = [packed(si[1]) if a.layout == "c4" else si[1] for si in slot_inputs]
    slots = [make_step(slot_levels[j], slot_inputs[j][2]) for j in range(S)]
    # a short last call (K or W not a multiple of Q): q < Q global batches, its own graph
    rems = sorted({c for c in calls_for(a.steps) + calls_for(a.warmup) if c != Q})
    rem_slots, rem_inputs, rem_levels = {}, {}, {}
    for q in rems:
        rem_inputs[q] = ri = inputs_for(S, q)
        rem_levels[q] = packed(ri[1]) if a.layout == "c4" else ri[1]
        rem_slots[q] = make_step(rem_levels[q], ri[2])
    streams = [torch.cuda.Stream(device) for _ in range(S)]
    solver, R, t, run = slots[0]
    gathered = {}
    pending = [None]

    def drain():
        if pending[0] is not None:
            pending[0].wait()
            pending[0] = None

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    def timed_loop(slots, rem_slots, steps, warmup):
        """W warm-up then K timed global batches (call c on slot c % S, Q batches per call, a
        remainder call where Q does not divide), barrier + synchronize on both sides; the
        N > 1 pose gather of call c overlaps call c + 1 (double-buffered)."""
        ncall = [0]

        def call(q):
            j = ncall[0] % len(slots)
            sl = slots[j] if q == Q else rem_slots[q]
            with torch.cuda.stream(streams[j]):
                sl[3]()
                if world > 1:
                    drain()
                    key = (q, ncall[0] % 2)
                    if key not in gathered:
                        gathered[key] = torch.empty(world * q * n_r, 12, device=device)
                    _, pending[0] = shard.gather_poses(sl[1], sl[2], out=gathered[key], async_op=True)
            ncall[0] += 1
        # setup warm-up by wall time, solves only (no collective: ranks run different counts)
        torch.cuda.synchronize()
        tw = time.perf_counter()
        while time.perf_counter() - tw < a.setup_warm_ms * 1e-3:
            for j, sl in enumerate(slots):
                with torch.cuda.stream(streams[j]):
                    sl[3]()
            torch.cuda.synchronize()
        for q in calls_for(warmup):
            call(q)
        drain()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for q in calls_for(steps):
            call(q)
        drain()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        if world > 1:
            import torch.distributed as dist
            e = torch.tensor([el], device=device, dtype=torch.float64)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = e.item()
        return el

    log(f"rank {rank}: {n_r} pairs per global batch in {G} batch(es) of {B}; {Q} global batch(es) per call, "
        f"{S} calls in flight; timing {a.steps} global batches")
    elapsed = timed_loop(slots, rem_slots, a.steps, a.warmup)
    log(f"rank {rank}: {elapsed / a.steps * 1e3:.3f} ms per global batch")
    for sl in slots + list(rem_slots.values()):
        ic.check_status(sl[0].status)
    ms_per_step = elapsed / a.steps * 1e3
    value = per_step * LEVELS * ITERS * a.steps / elapsed
    n_call = n_r * Q  # pairs per call (launch) on this rank

    # Encoder-to-solve: each call also runs the feature heads' epilogue (batchnorm + ELU of the
    # f_conv heads, algorithms.py:1273-1277) of both frames' 4 levels for every pair, which the
    # drop-in's encoder stores straight in the solver's channel-quad layout (dpft_bn_elu_pack)
    # -- the heads' conv outputs stand in as the NCHW features in channels_last with the
    # identity batchnorm (a = 1, b = 0: the features are >= 0, so ELU leaves them unchanged and
    # the solve sees the headline's inputs).  For comparison: the reference's own epilogue
    # alone (in place, its layout, no relayout: dpft_bn_elu -- idempotent here, so it reruns
    # on the same buffers) in front of the same solve, and the previous drop-in's route (that
    # in-place epilogue followed by the relayout dpft_pack_features_nhwc).
    e2e = None
    if a.layout == "c4" and not a.no_compare:
        Lb = ic.N.lib()
        chan = torch.cat((torch.ones(C, device=device), torch.zeros(C, device=device))).contiguous()

        def epilogue(src, dst, how):
            conv = [{k: d[k].contiguous(memory_format=torch.channels_last) for k in ("x0", "x1")} for d in src]

            def run_epilogue():
                for l in range(LEVELS):
                    for key in ("x0", "x1"):
                        c_, d_ = conv[l][key], dst[l][key]
                        Bn, Cn, Hn, Wn = c_.shape
                        if how == "fused_epilogue":
                            ic.N.check(Lb.dpft_bn_elu_pack(ic._ptr(c_), ic._ptr(chan), ic._ptr(d_), Bn, Cn, Hn, Wn,
                                                           ic._stream(device)), "dpft_bn_elu_pack")
                            continue
                        ic.N.check(Lb.dpft_bn_elu(ic._ptr(c_), ic._ptr(chan), c_.numel(), Cn, 1, 1,
                                                  ic._stream(device)), "dpft_bn_elu")
                        if how == "epilogue_then_relayout":
                            ic.N.check(Lb.dpft_pack_features_nhwc(ic._ptr(c_), ic._ptr(d_), Bn, Cn, Hn, Wn,
                                                                  ic._stream(device)), "dpft_pack_features_nhwc")
            run_epilogue.conv = conv
            return run_epilogue
        # HBM bytes per call: the solve's algorithmic bytes; the epilogue reads and writes
        # both frames' features once (4 * 4 * C bytes per pixel and level)
        px = sum(d["x0"].shape[0] * d["x0"].shape[2] * d["x0"].shape[3] for d in levels_nchw)
        solve_bytes = sum(solver.algorithmic_bytes(l) for l in range(LEVELS)) * ITERS
        epi_bytes = 16 * C * px
        e2e = {}
        for how in ("fused_epilogue", "reference_epilogue_in_place", "epilogue_then_relayout"):
            e_slots = [make_step(slot_levels[j], slot_inputs[j][2], pre=epilogue(slot_inputs[j][1], slot_levels[j],
                                                                                  how)) for j in range(S)]
            e_rem = {q: make_step(rem_levels[q], rem_inputs[q][2], pre=epilogue(rem_inputs[q][1], rem_levels[q], how))
                     for q in rem_slots}
            el = timed_loop(e_slots, e_rem, a.steps, a.warmup)
            same = all(torch.equal(es[1], sl[1]) and torch.equal(es[2], sl[2]) for es, sl in zip(e_slots, slots))
            ep_s = _timed(epilogue(slot_inputs[0][1], slot_levels[0], how), 20, device)
            e2e[how] = {"value": per_step * LEVELS * ITERS * a.steps / el, "ms_per_step": el / a.steps * 1e3,
                        "frac_of_headline": (per_step * LEVELS * ITERS * a.steps / el) / value,
                        "poses_equal_headline": same, "epilogue_alone_ms": ep_s * 1e3}
            del e_slots, e_rem
        e2e["epilogue_hbm_gb_per_call"] = epi_bytes / 1e9
        e2e["solve_algorithmic_gb_per_call"] = solve_bytes / 1e9
        e2e["fused_epilogue_tb_s"] = epi_bytes / (e2e["fused_epilogue"]["epilogue_alone_ms"] * 1e-3) / 1e12
        e2e["byte_bound_frac_of_headline"] = solve_bytes / (solve_bytes + epi_bytes)
        e2e["what"] = ("each call also runs the feature heads' batchnorm + ELU epilogue of both frames' 4-level "
                       "feature maps of every pair (conv outputs resident in HBM, channels_last): 'fused_epilogue' "
                       "stores the solver's channel-quad layout directly (dpft_bn_elu_pack, the drop-in's encoder); "
                       "'reference_epilogue_in_place' = the reference's epilogue alone in its own layout "
                       "(dpft_bn_elu in place; the solve still reads the pre-packed features); "
                       "'epilogue_then_relayout' = that in-place epilogue + dpft_pack_features_nhwc (the previous "
                       "drop-in). byte_bound_frac_of_headline = solve bytes / (solve + epilogue bytes): the "
                       "fraction any epilogue pass at the solve's bandwidth allows")
    # latency of one call alone (slot 0, back to back on one stream), rank 0 only
    latency_ms = None
    if rank == 0:
        n_lat = min(a.steps, 50)
        latency_ms = _timed(run, n_lat, device) * 1e3

    # ---- roofline of the dominant kernel: the level-0 fused reduce (+ in-kernel finalize),
    # exactly the launches the solve makes at level 0 (iterations forward, reverse, forward
    # -- DPFT_ITER_REVERSE -- continuing from the solved pose), HIP events on the stream they
    # are launched on (the current stream)
    Rk, tk = R.clone(), t.clone()
    solver.iterate(0, Rk, tk, first=True)
    l0_group = [False, True, False]
    for rev in l0_group:
        solver.iterate(0, Rk, tk, reverse=rev)
    groups = max(1, a.kernel_reps // len(l0_group))

    def l0():
        for rev in l0_group:
            solver.iterate(0, Rk, tk, reverse=rev)
    kern_us = _timed(l0, groups, device) / len(l0_group) * 1e6
    alg_bytes = solver.algorithmic_bytes(0)
    achieved = alg_bytes / (kern_us * 1e-6) / 1e9
    # (combine_ICP on the channel-quad path: the same U_IC reduce kernel plus its own ICP pass,
    # whose bytes the --icp traffic measurement includes)
    kname = "_ZN12_GLOBAL__N_116ic_reduce_kernelILi32ELb1ELb1ELi0ELb1EEEvNS_10IterParamsE"
    traffic = l0_traffic(n_call, B, kname, a.icp) if a.layout == "c4" else None
    copy_gbs = copy_peak_gbs(device) if rank == 0 else None
    read_gbs = read_peak_gbs(device, alg_bytes) if rank == 0 else None

    other = None
    if not a.no_compare:
        # the other feature layout through the same timed loop (S calls in flight, barrier +
        # max over ranks as the headline)
        other_layout = "nchw" if a.layout == "c4" else "c4"
        lay = (lambda lv: lv) if other_layout == "nchw" else packed
        o_slots = [make_step(lay(slot_inputs[j][1]), slot_inputs[j][2]) for j in range(S)]
        o_rem = {q: make_step(lay(rem_inputs[q][1]), rem_inputs[q][2]) for q in rem_slots}
        o_el = timed_loop(o_slots, o_rem, a.steps, a.warmup)
        o_value = per_step * LEVELS * ITERS * a.steps / o_el
        o_solver, o_R, o_t, o_run = o_slots[0]
        sec = _timed(o_run, min(a.steps, 50), device)
        other = {"layout": other_layout, "value": o_value, "ms_per_step": o_el / a.steps * 1e3,
                 "frac_of_headline": o_value / value, "ms_per_call_sequential": sec * 1e3,
                 "what": ("the reference's NCHW features resident in HBM, handed to the same pyramid solve: each level "
                          "packs f0 / f1 to channel quads on entry (pack_c4_x4_kernel, inside the timed graph) and "
                          "runs the channel-quad kernels" if other_layout == "nchw" else
                          "pre-packed channel-quad features"),
                 "value_sequential": n_call * LEVELS * ITERS / sec,
                 "max_abs_pose_diff_vs_headline": max((o_R - R).abs().max().item(), (o_t - t).abs().max().item()),
                 "poses_equal_headline": bool(torch.equal(o_R, R) and torch.equal(o_t, t))}
        del o_slots, o_rem, o_solver

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        log(f"CPU baseline: the oracle on batch 0 ({B} pairs) at {host_cpus()} threads, then one pair on one thread "
            f"(one warm-up and the best of 3 each)")
        cpu = cpu_baseline(levels_nchw, K, R, t, B, a.icp)

    if rank == 0:
        bpa = 280 if a.icp else 272
        line = {
            "metric": "IC solver iters/sec (640x480, C=32, 4-level)" + (" + combine_ICP" if a.icp else ""),
            "value": value, "unit": "IC iterations/s (all levels, 12 per pair)",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms_per_step,
            "higher_is_better": True, "scaling": "weak" if weak else "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: deterministic triangle-wave features of the 5 TUM fr1/desk example frames, "
                    "the 20 ordered pairs cycled with a left-right / up-down flip per round of 20 (distinct pairs) "
                    "(tests/golden/recipe.py; trained checkpoints absent)",
            "config": {"workload": ("cfg5: " if a.icp else "cfg3: ") +
                                   ("eval stream of global batches of %d pairs, " % per_step if not weak else
                                    "weak scaling, %d pairs per GPU per step, " % n_r) +
                                   "640x480, C=32, Cs=1, 4 levels x 3 GN iters, remove_tru_sigma" +
                                   (", combine_ICP (w=0.01)" if a.icp else ""),
                       "global_batch": per_step, "pairs_per_gpu": n_r, "batch": B,
                       "stream_group": Q, "batches_per_launch": G * Q, "pairs_per_launch": n_call, "inflight": S,
                       "parallelism": f"pair-sharded x{world}, RCCL all-gather of poses",
                       "graph": not a.no_graph, "feature_layout": a.layout, "setup_warm_ms": a.setup_warm_ms},
            "latency_ms_per_step": latency_ms,
            "latency_what": f"one call alone on rank 0: its {n_call} pairs ({Q} global batch(es)), 4 levels x 3 "
                            f"iterations, nothing else in flight",
            "pairs_per_s": per_step * a.steps / elapsed,
            "l0_iters_per_s": per_step * ITERS * a.steps / elapsed,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic["hbm_bytes"] if traffic else None,
                         "traffic_source": traffic["source"] if traffic else None,
                         "kernel": (f"icp_records_kernel + ic_reduce_kernel<32,Cs=1,tru,U_IC,{a.layout}> (level 0, "
                                    f"{n_call} pairs per launch: the combine_ICP pass, then the reduce launch with the "
                                    f"in-kernel finalize adding its records)" if a.icp and a.layout == "c4" else
                                    f"ic_reduce_kernel<32,Cs=1,tru,{'U_IC+ICP' if a.icp else 'U_IC'},{a.layout}> "
                                    f"(level 0, {n_call} pairs per launch, + in-kernel finalize)"),
                         "kernel_us": kern_us, "algorithmic_bytes_per_launch": alg_bytes,
                         "algorithmic_bytes_per_pixel": bpa,
                         "measured_copy_peak": copy_gbs,
                         "frac_of_measured_copy_peak": achieved / copy_gbs if copy_gbs else None,
                         "measured_read_peak": read_gbs,
                         "frac_of_measured_read_peak": achieved / read_gbs if read_gbs else None},
            "encoder_epilogue_to_solve": e2e,
            "cpu_baseline": cpu,
            "other_layout": other,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
