"""Do independent branches of a captured hipGraph run concurrently on this
ROCm build?  Two torch.cuda._sleep spin kernels (one wave each) captured on two
forked streams vs on one stream; also the same with 8 spin kernels."""
import torch

torch.cuda.init()
cyc = 2_000_000


def capture(nbranch, parallel):
    g = torch.cuda.CUDAGraph()
    main = torch.cuda.Stream()
    side = [torch.cuda.Stream() for _ in range(nbranch)]
    with torch.cuda.stream(main):
        torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=main):
        if parallel:
            ev = torch.cuda.Event()
            ev.record(main)
            ends = []
            for s in side:
                s.wait_event(ev)
                with torch.cuda.stream(s):
                    torch.cuda._sleep(cyc)
                e = torch.cuda.Event()
                e.record(s)
                ends.append(e)
            for e in ends:
                main.wait_event(e)
        else:
            for _ in range(nbranch):
                torch.cuda._sleep(cyc)
    return g


def timeit(g):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5


e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); torch.cuda._sleep(cyc); e1.record(); torch.cuda.synchronize()
print(f"one spin kernel eager: {e0.elapsed_time(e1):.3f} ms")
for nb in (2, 4, 8):
    ts = timeit(capture(nb, False))
    tp = timeit(capture(nb, True))
    print(f"{nb} branches: serial graph {ts:.3f} ms, forked graph {tp:.3f} ms (ratio {ts / tp:.2f})", flush=True)
