"""Host time per step of the 1-rank exchange loop (bench.py --force-exchange's step: svo_cast_wire on the cast stream,
svo_exchange_wire on a second stream after it, three buffer sets), against the GPU's step time: is the step host-bound?
usage: python tools/xchg_host.py [--steps 50]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    import torch

    import raytracing_test_amd as rt

    tree = rt.Tree.terrain_gpu(6, 4096, 4096, 0)
    cam = rt.normalize((1.0, -0.45, 1.0))
    W, H = 1920, 1080
    desc = rt.Tree.frame_desc((4.0, 90.0, 4.0), cam, W, H, 16384)
    n = rt.Tree.count(desc)
    ex = rt.Exchange(1, 0, rt.Exchange.unique_id(), 0)
    wb = tree.wire_bytes(desc)
    nb = 3
    wires = [torch.empty((n, wb), dtype=torch.uint8, device="cuda") for _ in range(nb)]
    frames = rt.Tree.alloc_hits(n, 0)
    cs, xs = torch.cuda.Stream(), torch.cuda.Stream()
    done = [torch.cuda.Event() for _ in range(nb)]
    xdone = [None] * nb

    def step(k, exchange=True):
        b = k % nb
        t0 = time.perf_counter()
        if xdone[b] is not None:
            cs.wait_event(xdone[b])
        tree.cast_wire(desc, wires[b], None, cs)
        t1 = time.perf_counter()
        if exchange:
            done[b].record(cs)
            xs.wait_event(done[b])
            ex.wire(tree, desc, wires[b], frames, stream=xs)
            e = torch.cuda.Event()
            e.record(xs)
            xdone[b] = e
        return t1 - t0, time.perf_counter() - t1

    for exchange in (False, True):
        for k in range(5):
            step(k, exchange)
        torch.cuda.synchronize()
        hc, hx = [], []
        t0 = time.perf_counter()
        for k in range(a.steps):
            c, x = step(k, exchange)
            hc.append(c)
            hx.append(x)
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tg = time.perf_counter() - t0
        print("exchange %-5s host per step: cast call %.1f us, exchange calls %.1f us, loop %.1f us; wall per step %.1f us"
              % (exchange, 1e6 * sum(hc) / a.steps, 1e6 * sum(hx) / a.steps, 1e6 * th / a.steps, 1e6 * tg / a.steps), flush=True)
    ex.close()


if __name__ == "__main__":
    main()
