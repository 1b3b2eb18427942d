#!/usr/bin/env python3
"""Diagnostics: replay a recorded tile trace (scripts/tile_schedule.py output) through a greedy list
scheduler with P parallel wave slots, to compare tile orders (natural, heavy-first, coarse classes).
Durations are taken as order-independent, which they are only roughly (contention).
Usage: sched_sim.py <trace.npy> [P]"""
import heapq
import sys

import numpy as np


def sim(dur, order, P):
    h = [0.0] * P
    end = 0.0
    for i in order:
        t = heapq.heappop(h)
        t2 = t + dur[i]
        end = max(end, t2)
        heapq.heappush(h, t2)
    return end


def main():
    tr = np.load(sys.argv[1]).astype(np.int64)
    P = int(sys.argv[2]) if len(sys.argv) > 2 else 6300
    dur = (tr[:, 1] - tr[:, 0]) / 100.0
    n = len(dur)
    print("lower bound %.1f  natural %.1f  heavy-first %.1f  random %.1f  (max tile %.1f us)" % (
        dur.sum() / P, sim(dur, range(n), P), sim(dur, np.argsort(-dur, kind="stable"), P),
        sim(dur, np.random.default_rng(1).permutation(n), P), dur.max()))
    # log-spaced buckets (4 per octave), heavy bucket first, natural order inside a bucket
    key = np.floor(4 * np.log2(np.maximum(dur, 1e-3)))
    print("heavy-first by 4/octave buckets: %.1f" % sim(dur, np.lexsort((np.arange(n), -key)), P))
    for q in (2, 4):
        cls = np.digitize(dur, np.quantile(dur, np.linspace(0, 1, q + 1)[1:-1]))
        print("heavy-first by %d quantile classes: %.1f" % (q, sim(dur, np.lexsort((np.arange(n), -cls)), P)))


if __name__ == "__main__":
    main()
