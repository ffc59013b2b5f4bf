#!/usr/bin/env python3
"""Build guard for a register-allocator hazard of the gfx950 code generator.

At the join block of a divergent branch the backend restores the wave's exec
mask with ``s_or_b64 exec, exec, s[..]`` (the lowered end of the branch).
When it places a VGPR spill -- a ``v_accvgpr_write`` into an AGPR or a
``scratch_store`` / ``buffer_store`` to the stack -- of a value that is live
across the branch AHEAD of that restore, the spill runs under the branch's
narrower exec mask and copies only the lanes that took the branch.  The reload
after the join returns stale data in every other lane.

This is the root cause of the withdrawn two-agents-per-wave demand-charge
k_size builds: with two agents per wave the agents'
branches diverge, the agent's capex / cost multiplier was spilled to a10-a13
ahead of the exec restore after the envelope build, and the Brent loop's
objective re-read them as 0 (system cost 0, NPV rising with kW, the search
driven to the bracket's top).  A wave-uniform branch (one agent per wave) is
lowered to a scalar branch with no exec restore, so it cannot occur there.

dgen_amd/build.py runs scan() on the device assembly of every build (the
same compile, -save-temps): a flagged 32-lane k_size / k_batt_finance
instantiation is withdrawn (REMEDY: its batches run one agent per wave, whose
branches are wave-uniform) and the library rebuilt; a flagged kernel without
a remedy fails the build.

CLI: python -m dgen_amd.spill_guard file.s  (exit status 1 if any kernel is flagged)
"""
import re
import sys

SPILL = re.compile(r"^\s*(v_accvgpr_write_b32|scratch_store_\w+|buffer_store_\w+)\b")
RESTORE = re.compile(r"^\s*s_or_b64\s+exec,\s*exec,")
LABEL = re.compile(r"^(\.LBB\w+|[A-Za-z_]\w*):")
# instructions that may sit between a join block's label and its exec restore
# without ending the prologue: scalar ops, SGPR lane spills, plain moves
PASS = ("s_", "v_writelane", "v_readlane", "v_mov", "v_accvgpr_read", "v_cndmask")

# 32-lane instantiations with a one-agent-per-wave fallback (compile macro)
REMEDY = {
    "k_size_wILi32ELb0E": "DGEN_NO2_SIZE",
    "k_size_wILi32ELb1E": "DGEN_NO2_SIZE_DC",
    "k_batt_finance_wILi32ELb0E": "DGEN_NO2_FIN",
    "k_batt_finance_wILi32ELb1E": "DGEN_NO2_FIN_DC",
}


def scan(path):
    """{kernel symbol: [(block label, [spill instructions])]} of every join
    block whose prologue spills a VGPR before restoring exec."""
    lines = open(path).read().split("\n")
    hits, fn = {}, None
    for i, l in enumerate(lines):
        m = LABEL.match(l)
        if not m:
            continue
        if m.group(1).startswith("_Z"):
            fn = m.group(1)
            continue
        if not (fn and m.group(1).startswith(".LBB")):
            continue
        spills = []
        for t in lines[i + 1:]:
            s = t.strip()
            if not s or s.startswith(";"):
                continue
            if LABEL.match(t):
                break
            if SPILL.match(t):
                spills.append(s)
            elif RESTORE.match(t):
                if spills:
                    hits.setdefault(fn, []).append((m.group(1), spills))
                break
            elif not s.startswith(PASS):
                break
    return hits


def remedies(hits):
    """(macros to define, kernels without a remedy)"""
    macros, fatal = set(), []
    for fn in hits:
        r = [m for k, m in REMEDY.items() if k in fn]
        if r:
            macros.update(r)
        else:
            fatal.append(fn)
    return sorted(macros), fatal


def report(hits) -> str:
    out = []
    for fn, blocks in hits.items():
        out.append(f"{fn}: {len(blocks)} join block(s) spill before the exec restore")
        for b, sp in blocks[:4]:
            out.append(f"    {b}: {'; '.join(sp[:4])}")
    return "\n".join(out)


if __name__ == "__main__":
    h = scan(sys.argv[1])
    print(report(h) or "no spill ahead of an exec restore")
    sys.exit(1 if h else 0)


def day_dma_wait(path, kernel="k_hourly_battILb1E"):
    """ISA check of k_hourly_batt's next-day LDS DMA:
    the day loop's read-back waits `s_waitcnt vmcnt(K)`; vmcnt retires in issue
    order, so the 12 global_load_lds_dwordx4 of the previous day have landed if
    at least K vector-memory ops are issued after the last of them on every
    path to the wait.  Counts the ops between the last DMA and the loop's back
    edge outside blocks an `s_cbranch_execz` can skip.  Every instantiation
    whose symbol contains `kernel` is checked; returns the (K, issued) pair
    with the smallest margin."""
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"_Z\S*" + kernel + r"\S*:", l)]
    worst = None
    for st in starts:
        en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
        body = [l.strip() for l in lines[st:en]]
        waits = [int(re.search(r"vmcnt\((\d+)\)", body[i]).group(1)) for i in range(len(body) - 1)
                 if body[i].startswith("s_waitcnt") and "vmcnt(" in body[i]
                 and body[i + 1].startswith("ds_read_b128")]
        k = max(waits)
        last = max(i for i, l in enumerate(body) if l.startswith("global_load_lds_dwordx4"))
        issued, cond = 0, False
        for l in body[last + 1:]:
            if l.startswith(".LBB"):
                cond = False
            elif l.startswith("s_cbranch_execz"):
                cond = True
            elif l.startswith("s_branch"):
                break
            elif re.match(r"(global_|buffer_|scratch_)", l) and not cond:
                issued += 1
        if worst is None or issued - k < worst[1] - worst[0]:
            worst = (k, issued)
    return worst
