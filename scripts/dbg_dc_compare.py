#!/usr/bin/env python3
"""Diagnostic: compare two dbg_dc_dump.py npz files (good build vs bad build):
per-agent outputs and the envelope groups (count, max load, lines)."""
import sys

import numpy as np

DCP, NL = 8, 8


def env(buf, n):
    b = buf.reshape(n, -1)
    lines = b[:, :12 * DCP * NL * 16].copy().view(np.float64).reshape(n, 12, DCP, NL, 2)
    o = 12 * DCP * NL * 16
    maxl = b[:, o:o + 12 * DCP * 8].copy().view(np.float64).reshape(n, 12, DCP)
    o += 12 * DCP * 8
    cnt = b[:, o:o + 12 * DCP * 4].copy().view(np.int32).reshape(n, 12, DCP)
    return lines, maxl, cnt


def main():
    a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
    n = a["system_kw"].size
    for k in ("nfev", "system_kw", "x_last", "first_without", "first_with", "price_per_kwh", "payback_raw", "npv", "tariff_final"):
        d = np.nonzero(~np.isclose(a[k], b[k], rtol=1e-12, atol=0))[0]
        print(f"{k}: {d.size} agents differ; first {d[:10].tolist()}")
        for i in d[:3]:
            print(f"    agent {i}: good {a[k][i]!r} bad {b[k][i]!r}")
    la, ma, ca = env(a["dc"], n)
    lb, mb, cb = env(b["dc"], n)
    dc = np.nonzero((ca != cb).any(axis=(1, 2)))[0]
    dm = np.nonzero((ma != mb).any(axis=(1, 2)))[0]
    print("cnt differ:", dc.size, dc[:10].tolist(), " maxl differ:", dm.size, dm[:10].tolist())
    dl = []
    for i in range(n):
        for m in range(12):
            for p in range(DCP):
                k = min(ca[i, m, p], NL)
                if k and not np.array_equal(la[i, m, p, :k], lb[i, m, p, :k]):
                    dl.append((i, m, p))
    print("lines differ:", len(dl), dl[:10])
    for i in dc[:3]:
        print("agent", i, "cnt good", ca[i].tolist(), "\n        bad ", cb[i].tolist())


if __name__ == "__main__":
    main()
