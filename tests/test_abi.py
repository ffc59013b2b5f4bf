"""The C-ABI library loads and exports every entry point include/dgen_hip.h
declares; ctypes struct layouts match the header (sizeof / offsetof probe
compiled with gcc).  No compute call is made (no GPU here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from dgen_amd import _lib
from dgen_amd.engine import SWITCH_DTYPE
from dgen_amd.tariff import TARIFF_DTYPE

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dgen_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int32_t|size_t|void)\s+(dgen_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    L = _lib.load(build_if_missing=True)
    names = declared_functions()
    assert len(names) >= 10
    for name in names:
        assert hasattr(L, name), name
    assert set(names) == set(_lib.EXPORTED)
    assert L.dgen_abi_version() == _lib.ABI_VERSION == 14
    m = re.search(r"#define DGEN_DEFAULT_CHUNKS\s+(\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _lib.DEFAULT_CHUNKS
    m = re.search(r"#define DGEN_DEFAULT_HOURLY_MONTHS\s+(\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _lib.DEFAULT_HOURLY_MONTHS
    m = re.search(r"#define DGEN_DEFAULT_HOURLY_SPLIT\s+(\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == _lib.DEFAULT_HOURLY_SPLIT


def test_workspace_bytes_formula():
    L = _lib.load()
    assert L.dgen_workspace_bytes(1000, 0) == 8 * (4 * 144 * 1000 + 1000)
    nb = int(re.search(r"#define DGEN_NB_BYTES\s+(\d+)", open(HEADER).read()).group(1))
    assert L.dgen_workspace_bytes(10, 3) == 8 * (4 * 144 * 10 + 10 + 8760 * 3) + nb * 3
    assert L.dgen_workspace_bytes(-1, 0) == 0


def test_last_error_is_callable():
    buf = ctypes.create_string_buffer(64)
    assert _lib.load().dgen_last_error(buf, 64) == 0


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "dgen_hip.h"
#define S(t) printf(#t " %zu\n", sizeof(t));
#define O(t, f) printf(#t "." #f " %zu\n", offsetof(t, f));
int main(void) {
  S(dgen_cfg) S(dgen_tariff) S(dgen_switch) S(dgen_tables) S(dgen_agents) S(dgen_outputs)
  S(dgen_attach_in) S(dgen_attach_out) S(dgen_diffusion_in) S(dgen_diffusion_out)
  O(dgen_cfg, batt_v_nom) O(dgen_cfg, batt_eta_out) O(dgen_tariff, fixed) O(dgen_tariff, buy)
  O(dgen_tariff, sell) O(dgen_tariff, wkday) O(dgen_tariff, flags) O(dgen_tables, n_shapes)
  O(dgen_tables, n_tariffs) O(dgen_tables, demand) S(dgen_demand) O(dgen_demand, tou_cap)
  O(dgen_demand, flat_price) O(dgen_demand, wkend) O(dgen_agents, vor) O(dgen_outputs, baseline) O(dgen_outputs, net_with_batt)
  return 0;
}
"""


@pytest.fixture(scope="module")
def layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("probe")
    src = d / "probe.c"
    src.write_text(PROBE)
    exe = d / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {k: int(v) for k, v in (line.split() for line in out.strip().splitlines())}


def test_struct_sizes(layout):
    assert layout["dgen_cfg"] == ctypes.sizeof(_lib.Cfg)
    assert layout["dgen_tariff"] == TARIFF_DTYPE.itemsize
    assert layout["dgen_switch"] == SWITCH_DTYPE.itemsize
    assert layout["dgen_tables"] == ctypes.sizeof(_lib.Tables)
    assert layout["dgen_agents"] == ctypes.sizeof(_lib.Agents)
    assert layout["dgen_outputs"] == ctypes.sizeof(_lib.Outputs)
    from dgen_amd import attachment, diffusion
    assert layout["dgen_attach_in"] == ctypes.sizeof(attachment.AttachIn)
    assert layout["dgen_attach_out"] == ctypes.sizeof(attachment.AttachOut)
    assert layout["dgen_diffusion_in"] == ctypes.sizeof(diffusion.DiffIn)
    assert layout["dgen_diffusion_out"] == ctypes.sizeof(diffusion.DiffOut)


def test_struct_offsets(layout):
    assert layout["dgen_cfg.batt_v_nom"] == _lib.Cfg.batt_v_nom.offset
    assert layout["dgen_cfg.batt_eta_out"] == _lib.Cfg.batt_eta_out.offset
    for f in ("fixed", "buy", "sell", "wkday", "flags"):
        assert layout[f"dgen_tariff.{f}"] == TARIFF_DTYPE.fields[f][1], f
    assert layout["dgen_tables.n_shapes"] == _lib.Tables.n_shapes.offset
    assert layout["dgen_tables.n_tariffs"] == _lib.Tables.n_tariffs.offset
    assert layout["dgen_tables.demand"] == _lib.Tables.demand.offset
    from dgen_amd.tariff import DEMAND_DTYPE
    assert layout["dgen_demand"] == DEMAND_DTYPE.itemsize
    for f in ("tou_cap", "flat_price", "wkend"):
        assert layout[f"dgen_demand.{f}"] == DEMAND_DTYPE.fields[f][1], f
    assert layout["dgen_agents.vor"] == _lib.Agents.vor.offset
    assert layout["dgen_outputs.baseline"] == _lib.Outputs.baseline.offset
    assert layout["dgen_outputs.net_with_batt"] == _lib.Outputs.net_with_batt.offset


def test_product_never_imports_oracle():
    """The product package must not import, link or load the oracle."""
    pkg = os.path.join(REPO, "dgen_amd")
    bad = re.compile(r"^\s*(import\s+oracle|from\s+oracle|.*liborc|.*orc_\w+\()", re.M)
    for root, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(root, fn)).read()
                assert not bad.search(text), fn
