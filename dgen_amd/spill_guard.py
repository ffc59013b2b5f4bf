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
# register-to-register copies of a live value (live-range splits, AGPR
# reloads, selects) in a join prologue write only the branch's lanes as well:
# the same stale-lane hazard as a spill.  The current build has
# none; phi copies sit at the end of the predecessor blocks, not here.
COPY = re.compile(r"^\s*(v_mov_b(32|64)\w*\s+[va]\S*,\s*[va][\[\d]|v_cndmask_b32\w*|v_accvgpr_read_b32|"
                  r"v_accvgpr_mov_b32)")
RESTORE = re.compile(r"^\s*s_or_b64\s+exec,\s*exec,")
LABEL = re.compile(r"^(\.LBB\w+|[A-Za-z_]\w*):")
# instructions that may sit between a join block's label and its exec restore
# without ending the prologue: scalar ops, SGPR lane spills, moves (a
# VGPR / AGPR-sourced copy or select among them is itself a hit, COPY above)
PASS = ("s_", "v_writelane", "v_readlane", "v_mov", "v_accvgpr_read", "v_accvgpr_mov", "v_cndmask")

# 32-lane instantiations with a one-agent-per-wave fallback (compile macro)
# (symbol prefix: <LPA, DC, NET, PK>; the kWh/kW-peak builds (PK) have their own)
REMEDY = {
    "k_size_wILi32ELb0E": "DGEN_NO2_SIZE",
    "k_size_wILi32ELb1ELb1ELb0E": "DGEN_NO2_SIZE_DC",
    "k_size_wILi32ELb1ELb0ELb0E": "DGEN_NO2_SIZE_DC",
    "k_size_wILi32ELb1ELb1ELb1E": "DGEN_NO2_SIZE_PK",
    "k_batt_finance_wILi32ELb0E": "DGEN_NO2_FIN",
    "k_batt_finance_wILi32ELb1ELb1ELb0E": "DGEN_NO2_FIN_DC",
    "k_batt_finance_wILi32ELb1ELb0ELb0E": "DGEN_NO2_FIN_DC",
    "k_batt_finance_wILi32ELb1ELb1ELb1E": "DGEN_NO2_FIN_PK",
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
            if SPILL.match(t) or COPY.match(t):
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


def _blocks(body):
    """Basic blocks of a function body (stripped lines): split at labels and
    after every branch.  Returns [(label or None, [instructions], [successor
    block indices])]."""
    blocks, cur = [], [None, []]
    for l in body:
        if not l or l.startswith((";", ".")) and not l.startswith(".LBB"):
            continue
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            blocks.append(cur)
            cur = [m.group(1), []]
            continue
        cur[1].append(l)
        if l.startswith(("s_branch", "s_cbranch", "s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur = [None, []]
    blocks.append(cur)
    blocks = [b for b in blocks if b[0] is not None or b[1]]
    index = {b[0]: k for k, b in enumerate(blocks) if b[0]}
    out = []
    for k, (lab, ins) in enumerate(blocks):
        succ = []
        last = ins[-1] if ins else ""
        tgt = last.split()[1] if last.startswith(("s_branch", "s_cbranch")) and len(last.split()) > 1 else None
        if last.startswith("s_branch"):
            succ = [index[tgt]] if tgt in index else []
        elif last.startswith(("s_endpgm", "s_setpc")):
            succ = []
        else:
            if last.startswith("s_cbranch") and tgt in index:
                succ.append(index[tgt])
            if k + 1 < len(blocks):
                succ.append(k + 1)
        out.append((lab, ins, succ))
    return out


VMEM = re.compile(r"^(global_|buffer_|scratch_)")
DMA = "global_load_lds_dwordx4"


def day_dma_wait(path, kernel="k_hourly_battILb1E"):
    """ISA check of k_hourly_batt's next-day LDS DMA:
    the day loop's read-back waits `s_waitcnt vmcnt(K)` (directly ahead of its
    ds_read_b128s); vmcnt retires in issue order, so the previous day's 12
    global_load_lds_dwordx4 have landed if at least K vector-memory ops are
    issued after the last of them on EVERY path to the wait.  The count is the
    shortest path over the control-flow graph from each DMA group's last
    instruction to each wait (a block an s_cbranch_execz skips counts nothing
    on the path that skips it; a path through another DMA group or a full
    drain, s_waitcnt vmcnt(0), ends there).
    Every instantiation whose symbol contains `kernel` is checked; returns the
    (K, issued) pair with the smallest margin, DRAINED when DMA groups and
    counted wait sites exist but every path between them drains (vmcnt(0)), and
    None when no DMA group or no counted wait site was found at all (a symbol
    change or a reordering the check no longer sees: the build fails then)."""
    import heapq
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if re.match(r"_Z\S*" + kernel + r"\S*:", l)]
    worst = None
    seen_src = seen_wait = False
    for st in starts:
        en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
        B = _blocks([l.strip() for l in lines[st + 1:en]])
        # wait sites: (block, position, K)
        waits = [(k, j, int(re.search(r"vmcnt\((\d+)\)", ins[j]).group(1)))
                 for k, (_, ins, _) in enumerate(B) for j in range(len(ins) - 1)
                 if ins[j].startswith("s_waitcnt") and "vmcnt(" in ins[j] and ins[j + 1].startswith("ds_read_b128")]
        srcs = [(k, max(j for j, l in enumerate(ins) if l.startswith(DMA)))
                for k, (_, ins, _) in enumerate(B) if any(l.startswith(DMA) for l in ins)]
        seen_src |= bool(srcs)
        seen_wait |= any(K > 0 for _, _, K in waits)
        for kb, jd in srcs:
            # cost of entering block b from its top, up to a DMA or a full
            # drain s_waitcnt vmcnt(0) (either ends the path) or its end
            def head(b):
                c = 0
                for l in B[b][1]:
                    if l.startswith(DMA) or (l.startswith("s_waitcnt") and "vmcnt(0)" in l):
                        return c, True
                    c += bool(VMEM.match(l))
                return c, False
            tail = sum(bool(VMEM.match(l)) for l in B[kb][1][jd + 1:])
            dist = {}
            pq = [(tail, s) for s in B[kb][2]]
            while pq:
                d, b = heapq.heappop(pq)
                if b in dist:
                    continue
                dist[b] = d
                c, stop = head(b)
                if not stop:
                    for s2 in B[b][2]:
                        if s2 not in dist:
                            heapq.heappush(pq, (d + c, s2))
            for wb, wj, K in waits:
                if wb not in dist or K == 0:
                    continue
                pre = B[wb][1][:wj]
                if any(l.startswith(DMA) or (l.startswith("s_waitcnt") and "vmcnt(0)" in l) for l in pre):
                    continue
                issued = dist[wb] + sum(bool(VMEM.match(l)) for l in pre)
                if worst is None or issued - K < worst[1] - worst[0]:
                    worst = (K, issued)
    if worst is None:
        return DRAINED if (seen_src and seen_wait) else None
    return worst


DRAINED = "drained"


if __name__ == "__main__":
    h = scan(sys.argv[1])
    print(report(h) or "no spill ahead of an exec restore")
    sys.exit(1 if h else 0)
