#!/usr/bin/env python3
"""Rejection-trip passes per wave: today every pending lane draws its own
randomUnitVec candidates in stream order (vec.zig:71-80, acceptance pi/6), so a wave pays the
maximum trip count over its lanes; with a counter-based per-(pixel, sample) RNG any lane could draw
candidate j of any pending lane, so a pass of 64 candidate slots spread over the pending lanes
resolves most of them at once (the first accepted candidate of each lane, in stream order, is kept:
the same samples as today for that RNG).  Prints the expected passes per wave for n pending lanes.

    python tools/trip_sim.py
"""
import math
import random

P_ACCEPT = math.pi / 6


def trips():
    k = 1
    while random.random() > P_ACCEPT:
        k += 1
    return k


def passes_now(n):
    return max((trips() for _ in range(n)), default=0)


def passes_lane_parallel(n):
    pend, passes = n, 0
    while pend:
        passes += 1
        base, extra = divmod(64, pend)
        pend -= sum(any(random.random() < P_ACCEPT for _ in range(base + (i < extra))) for i in range(pend))
    return passes


if __name__ == "__main__":
    random.seed(1)
    print("pending lanes | trips today (max over lanes) | passes, lane-parallel candidates")
    for n in (4, 8, 16, 24, 32, 48, 64):
        runs = 4000
        a = sum(passes_now(n) for _ in range(runs)) / runs
        b = sum(passes_lane_parallel(n) for _ in range(runs)) / runs
        print(f"{n:13d} | {a:28.2f} | {b:.2f}")
