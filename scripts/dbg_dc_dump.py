#!/usr/bin/env python3
"""Diagnostic (not product): size the demand-charge parity population with the
library named by DGEN_LIB (a debug build exporting dgen_debug_copy_dc) and dump
the outputs plus the per-agent demand-charge envelope buffer to an npz, so two
builds can be compared bit for bit.  Usage: DGEN_LIB=... dbg_dc_dump.py out.npz"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgen_amd import _lib  # noqa: E402
from dgen_amd.config import EngineConfig  # noqa: E402
from dgen_amd.engine import Engine, outputs_to_host  # noqa: E402
from tests.test_gpu_demand import _pop  # noqa: E402

DCW_BYTES = 12 * 8 * (8 * 16 + 8 + 4)


def main():
    pop = _pop(160, net_billing=False)
    eng = Engine(0, EngineConfig(skip_demand_charges=0))
    eng.load_profiles(pop.shapes, pop.cfs, pop.wholesale)
    eng.set_tariffs(pop.tariffs, pop.demand)
    eng.set_switches(pop.switches)
    batch = eng.upload_agents(pop.cols, pop.n_scratch)
    out = eng.alloc_outputs(batch.n, hourly=False)
    eng.size(batch, out)
    torch.cuda.synchronize()
    o = outputs_to_host(out)
    buf = np.zeros(batch.n * DCW_BYTES, np.uint8)
    L = _lib.load()
    L.dgen_debug_copy_dc.restype = ctypes.c_int32
    L.dgen_debug_copy_dc.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    rc = L.dgen_debug_copy_dc(eng.ctx, buf.ctypes.data, buf.size)
    print("copy rc", rc, flush=True)
    np.savez(sys.argv[1], dc=buf, **{k: v for k, v in o.items() if v is not None})


if __name__ == "__main__":
    main()
