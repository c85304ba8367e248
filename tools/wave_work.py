"""Join the STATS build's per-block stamps with its per-ray work (bench.py SVO_STAMPS / SVO_RAY_WORK dumps of one
C3 frame, 16x4 footprints, top tile rows first): per wave the duration against the lanes' iterations and node
loads.  usage: python tools/wave_work.py stamps.npy work.npy [W H]"""
import sys

import numpy as np


def main():
    st = np.load(sys.argv[1]).astype(np.float64) / 100.0
    wk = np.load(sys.argv[2]).astype(np.uint64)
    W, H = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (1920, 1080)
    rows, tiles_x = (H + 7) // 8, W // 16 * 2
    dur = st[:, 1] - st[:, 0]
    f = lambda s: ((wk >> np.uint64(s)) & np.uint64(0xFFFF)).astype(np.int64)
    look, it, br, ld = f(0), f(16), f(32), f(48)
    nb = rows * tiles_x
    b = np.arange(nb)
    trl, tx = rows - 1 - b // tiles_x, b % tiles_x
    lane = np.arange(64)
    py = trl[:, None] * 8 + (tx[:, None] & 1) * 4 + (lane[None, :] >> 4)
    px = (tx[:, None] >> 1) * 16 + (lane[None, :] & 15)
    rec = py * W + px
    ok = (py < H) & (px < W)
    rec = np.where(ok, rec, 0)
    g = lambda a: np.where(ok, a[rec], 0)
    I, L, B, K = g(it), g(ld), g(br), g(look)
    d = dur[:nb]
    order = np.argsort(d)[::-1]
    print("wave  dur_us  iters(max,mean)  loads(max,mean,sum)  brick(max,mean)  lookups(max)")
    for i in list(order[:25]) + list(order[len(order) // 2:len(order) // 2 + 5]):
        print("%5d %7.1f   %4d %6.1f   %4d %6.1f %6d   %4d %6.1f   %4d" % (i, d[i], I[i].max(), I[i].mean(), L[i].max(), L[i].mean(), L[i].sum(),
                                                                  B[i].max(), B[i].mean(), K[i].max()))
    for q in (0.5, 0.9, 0.99, 0.999):
        print("quantile %.3f of wave duration %.1f us" % (q, np.quantile(d, q)))
    c = np.corrcoef(np.vstack([d, I.max(1), L.max(1), L.sum(1), B.max(1)]))
    print("corr(dur, max iters / max loads / sum loads / max brick):", c[0, 1:].round(3))
    top = order[:200]
    print("top-200 waves: mean dur %.1f, max-iters %.1f, max-loads %.1f, sum-loads %.0f; all waves: %.1f, %.1f, %.1f, %.0f" %
          (d[top].mean(), I[top].max(1).mean(), L[top].max(1).mean(), L[top].sum(1).mean(), d.mean(), I.max(1).mean(), L.max(1).mean(), L.sum(1).mean()))


if __name__ == "__main__":
    main()
