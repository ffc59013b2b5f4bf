#!/usr/bin/env python3
"""Generate and verify the 24-input sorting network used by the daily
peak-shaving target (k_hourly_batt day_target / oracle day_target).

Batcher's odd-even merge sort for 32 inputs, restricted to inputs 0..23 by
treating inputs 24..31 as -inf pads (descending sort: a comparator (i, j),
i < j, leaves max at i and min at j) and dropping every comparator that
touches a pad: a pad is the smallest value, so it never moves out of a
position >= 24 that it starts in -- checked, not assumed, by the 0-1
principle over all 2^24 binary inputs below.

    python scripts/gen_sortnet.py          # verify + print the C table
"""
import numpy as np

N, M = 24, 32


def batcher(n):
    net = []

    def merge(lo, cnt, r):
        step = r * 2
        if step < cnt:
            merge(lo, cnt, step)
            merge(lo + r, cnt, step)
            for i in range(lo + r, lo + cnt - r, step):
                net.append((i, i + r))
        else:
            net.append((lo, lo + r))

    def sort(lo, cnt):
        if cnt > 1:
            h = cnt // 2
            sort(lo, h)
            sort(lo + h, h)
            merge(lo, cnt, 1)

    sort(0, n)
    return net


def network():
    return [(i, j) for i, j in batcher(M) if i < N and j < N]


def verify(net):
    """0-1 principle: every binary 24-vector comes out non-increasing."""
    x = np.arange(1 << N, dtype=np.uint32)
    bits = [((x >> k) & 1).astype(np.uint8) for k in range(N)]
    for i, j in net:
        a, b = bits[i], bits[j]
        bits[i], bits[j] = a | b, a & b          # max to i, min to j
    for k in range(N - 1):
        if np.any(bits[k] < bits[k + 1]):
            return False
    return True


if __name__ == "__main__":
    net = network()
    assert verify(net), "network does not sort"
    print(f"// {len(net)} comparators, verified on all 2^{N} binary inputs (scripts/gen_sortnet.py)")
    print("{" + ", ".join(f"{{{i}, {j}}}" for i, j in net) + "}")
