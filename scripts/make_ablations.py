#!/usr/bin/env python3
"""Build kernel variants for A/B timing (diagnostic only; outputs are wrong
by construction).  Each variant is a text edit of a temporary copy of the
source; nothing here is part of the product build."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "dgen_amd", "csrc", "dgen_hip.hip")
OUT = os.path.join(REPO, "dgen_amd", "lib", "ablate")
sys.path.insert(0, REPO)
from dgen_amd.build import FLAGS, hipcc  # noqa: E402

VARIANTS = {
    "base": [],
    "no_target": [("target = day_target(r, ls, cs6, power, avail, dmax, need0, a0, b0);",
                   "target = 0.0; asm volatile(\"\" :: \"v\"(need0), \"v\"(dmax), \"v\"(a0), \"v\"(b0));")],
    "no_hourly_stores": [("if (o_base) o_base[h * n + i] = (float)ld;", "asm volatile(\"\" :: \"v\"(ld));"),
                         ("o_pvo[h * n + i] = (float)(dn > 0.0 ? dn : 0.0);", "asm volatile(\"\" :: \"v\"(dn));"),
                         ("if (o_wb) o_wb[h * n + i] = (float)g2l;", "asm volatile(\"\" :: \"v\"(g2l));")],
    "no_bins": [("acc.at(p) += ld;\n                    acc.hi(p) += sys;",
                 "asm volatile(\"\" :: \"v\"(ld), \"v\"(sys), \"v\"(p));")],
}


def main():
    os.makedirs(OUT, exist_ok=True)
    src = open(SRC).read().replace('#include "../../include/dgen_hip.h"',
                                   f'#include "{REPO}/include/dgen_hip.h"')
    for name, edits in VARIANTS.items():
        s = src
        for a, b in edits:
            assert a in s, (name, a[:40])
            s = s.replace(a, b)
        tmp = f"/tmp/ablate_{name}.hip"
        open(tmp, "w").write(s)
        out = os.path.join(OUT, f"libdgen_{name}.so")
        subprocess.run([hipcc(), *FLAGS, "-o", out, tmp], check=True)
        print("built", out)


if __name__ == "__main__":
    main()
