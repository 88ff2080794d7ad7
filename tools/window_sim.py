"""Cost of folding a pixel's samples in order ON CHIP, simulated
with the reference's own path lengths (world rays per path of the tests/golden
renders).  A wave owns a pixel and its 64 lanes run the pixel's paths in sample
order; a finished sample can be folded only when every earlier one is.  With an
on-chip window of W samples, a lane may start sample g only while g < frontier + W
(stall), or the samples beyond the window spill to memory (spill).  Reports the
wave-iterations relative to an unbounded window, and the fraction of samples that
would spill.

    python tools/window_sim.py
"""
import os

import numpy as np

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")


def sim(lens, W, n=100000, lanes=64, stall=True, seed=0):
    L = np.random.default_rng(seed).choice(lens, size=n)
    nxt = frontier = spill = it = 0
    remain = np.zeros(lanes, int)
    idx = -np.ones(lanes, int)
    done = np.zeros(n, bool)
    while frontier < n:
        for l in range(lanes):
            if idx[l] < 0 and nxt < n and (not stall or nxt < frontier + W):
                idx[l], remain[l] = nxt, L[nxt]
                nxt += 1
        act = idx >= 0
        remain[act] -= 1
        it += 1
        fin = act & (remain == 0)
        spill += int((idx[fin] >= frontier + W).sum())
        done[idx[fin]] = True
        idx[fin] = -1
        while frontier < n and done[frontier]:
            frontier += 1
    return it, spill / n


def main():
    for name in ["s2", "s3", "s4_d40", "s5_d40"]:
        r = np.fromfile(os.path.join(GOLD, f"{name}.rays.u8"), np.uint8).astype(int).ravel()
        base = sim(r, 10 ** 9)[0]
        stall = [(W, round(sim(r, W)[0] / base, 3)) for W in (64, 128, 256, 512)]
        spill = [(W, round(sim(r, W, stall=False)[1], 3)) for W in (64, 128, 256)]
        print(f"{name}: mean {r.mean():.2f} world rays/path; stall: iterations x {stall}; spill: fraction {spill}")


if __name__ == "__main__":
    main()
