"""Predicted effect of suspendable mesh walks from measured walk lengths.

Model of one wave of k_paths: 64 lanes, each holding one world ray whose mesh walk
takes L node steps (L drawn from the measured per-ray histogram, tools/walk_hist.py).
A wave-iteration costs S (the phases outside the walk) plus c per node step the walk
loop runs (the wave's per-step time is set by its longest-walking lane, not by how
many lanes are in the step).  Without suspension every lane finishes its walk each
iteration, so the walk runs max(L) steps.  With suspension (SRR_WALK_Q = q) the loop
stops, once every lane has taken walk_min steps, at the first step where at most
q/64 of the lanes are still walking; those lanes keep their remaining steps and
resume next iteration alongside fresh rays.  Output: world rays per 1,000 K ticks
with and without, per q.

    python tools/walk_sim.py profiles/r06/walk_hist.txt
"""
import random
import re
import sys


def read_hists(path):
    hists, cur = {}, None
    for line in open(path):
        m = re.match(r"== (\S+)", line)
        if m:
            cur = m.group(1)
        m = re.match(r"steps per ray:(.*)", line)
        if m and cur:
            hists[cur] = {int(a): int(b) for a, b in (kv.split(":") for kv in m.group(1).split())}
    return hists


def sampler(h):
    vals, cum, tot = [], [], 0
    for k in sorted(h):
        tot += h[k]
        vals.append(k)
        cum.append(tot)

    def draw(rng):
        x = rng.random() * tot
        lo, hi = 0, len(cum) - 1
        while lo < hi:
            mid = (lo + hi) // 2
            if cum[mid] > x:
                hi = mid
            else:
                lo = mid + 1
        return max(1, vals[lo])  # (bin 63 holds >= 63; every ray through the mesh takes the root step)
    return draw


def simulate(draw, S, c, q, walk_min=1, iters=20000, seed=1, rho=0.0):
    """rho: lanes of a wave are correlated (k_paths' lanes are samples of the same
    pixels): a refilled lane repeats the wave's current shared draw with probability
    rho, else draws on its own; the shared draw is renewed each iteration."""
    rng = random.Random(seed)
    shared = draw(rng)
    rem = [shared if rng.random() < rho else draw(rng) for _ in range(64)]
    ticks = rays = steps_run = susp = 0
    for _ in range(iters):
        taken = [0] * 64
        s = 0
        while True:
            act = [i for i in range(64) if rem[i] > 0]
            if not act:
                break
            if q and len(act) <= (64 * q) >> 6 and all(taken[i] >= walk_min for i in act):
                susp += len(act)
                break
            for i in act:
                rem[i] -= 1
                taken[i] += 1
            s += 1
        ticks += S + c * s
        steps_run += s
        shared = draw(rng)
        for i in range(64):
            if rem[i] == 0:
                rays += 1
                rem[i] = shared if rng.random() < rho else draw(rng)
    return rays / ticks * 1000, steps_run / iters, susp / iters, rays / iters


def calibrate(draw, S, c, target_max):
    """the rho whose no-suspension walk (the wave's longest lane) averages target_max steps"""
    lo, hi = 0.0, 1.0
    for _ in range(14):
        mid = (lo + hi) / 2
        if simulate(draw, S, c, 0, iters=3000, rho=mid)[1] > target_max:
            lo = mid
        else:
            hi = mid
    return (lo + hi) / 2


# k_paths' measured phase timing (profiles/r05/phases_final.txt): non-walk ticks per
# wave-iteration S (K), ticks per step of the longest walk c (K), longest walk (steps)
MEASURED = {"c2": (88.1, 5.3, 3.8), "c4": (130.0, 5.1, 10.1), "c4r": (93.0, 6.3, 14.5)}


def main():
    hists = read_hists(sys.argv[1])
    for name, h in hists.items():
        n = sum(h.values())
        mean = sum(k * v for k, v in h.items()) / n
        draw = sampler(h)
        S, c, mx = MEASURED.get(name, (93.0, 6.3, None))
        for label, rho in (("independent lanes", 0.0),) + ((("lanes correlated as measured", calibrate(draw, S, c, mx)),) if mx else ()):
            base = simulate(draw, S, c, 0, rho=rho)
            print(f"{name} ({label}, rho {rho:.3f}; S {S} K, c {c} K): {n} walks, mean {mean:.2f} steps; "
                  f"no suspension: walk {base[1]:.1f} steps/it, {base[0]:.1f} rays per 1000 K ticks")
            for q in (4, 8, 12, 16, 24, 32):
                for wm in (1, 4):
                    r = simulate(draw, S, c, q, walk_min=wm, rho=rho)
                    print(f"  q {q:2d} min {wm}: walk {r[1]:.1f} steps/it, {r[2]:.1f} lanes suspended/it, "
                          f"{r[3]:.1f} rays/it, {r[0]:.1f} rays per 1000 K ticks ({100 * (r[0] / base[0] - 1):+.1f} %)")


if __name__ == "__main__":
    main()
