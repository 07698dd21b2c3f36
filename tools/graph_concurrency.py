"""Do the two branches of a captured HIP graph run concurrently on this runtime?  Two spin
kernels (torch.cuda._sleep, one workgroup each) forked onto two streams inside one capture:
a replay as long as one spin means the branches overlap, twice as long that they serialise."""
import time
import torch

dev = torch.device("cuda:0")
cyc = 20_000_000
main, s1, s2 = torch.cuda.current_stream(), torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


one = timed(lambda: torch.cuda._sleep(cyc))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(cyc)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(cyc)
    cur.wait_stream(s1)
    cur.wait_stream(s2)
both = timed(g.replay)


def eager():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(cyc)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(cyc)
    cur.wait_stream(s1)
    cur.wait_stream(s2)


eag = timed(eager)
print(f"one spin {one:.2f} ms; two forked spins: graph replay {both:.2f} ms, eager streams {eag:.2f} ms "
      f"({'concurrent' if both < 1.5 * one else 'serialised'} in the graph)")
