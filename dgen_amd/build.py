"""Build libdgen_hip.so in-tree (gfx950).

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the resulting .so is git-ignored but travels to the GPU box with
the repository snapshot.
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
SRC = os.path.join(HERE, "csrc", "dgen_hip.hip")
HDR = os.path.join(REPO, "include", "dgen_hip.h")
OUT_DIR = os.path.join(HERE, "lib")
OUT = os.path.join(OUT_DIR, "libdgen_hip.so")
ARCH = os.environ.get("DGEN_OFFLOAD_ARCH", "gfx950")

FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    # keep a*b+c as two roundings: the bracket / Brent path stays bit-identical
    # to scipy and numpy, and the kernels agree with the oracle
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the HIP extension cannot be built")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in (SRC, HDR, __file__, os.path.join(HERE, "spill_guard.py")))


GUARD = os.path.join(OUT_DIR, "build_guard.json")


# The year-lane search kernels (k_size_w, k_dc_env, k_nb_env) build in a
# translation unit of their own under the code generator's iterative
# max-occupancy scheduler: k_size -4 % on C2 and C4 against the default
# scheduler, which the hourly scan keeps (it is 1 % slower under the other;
# DESIGN.md section 6, round 5).
TUS = (("main", []), ("search", ["-mllvm", "-amdgpu-sched-strategy=iterative-maxocc"]))


# Developer cache of compiled units (outside the tree): a unit whose
# preprocessed source (no line markers) and flags are unchanged reuses its
# object and assembly -- an edit to the main unit's kernels does not recompile
# the search unit.  DGEN_BUILD_CACHE=0 turns it off.
CACHE_DIR = os.environ.get("DGEN_BUILD_CACHE_DIR", "/tmp/dgen_build_cache")


def _unit_key(tu_flags):
    import hashlib
    if os.environ.get("DGEN_BUILD_CACHE", "1") == "0":
        return None
    try:
        pp = subprocess.run([hipcc(), *tu_flags, "-E", "-P", SRC], capture_output=True, timeout=300)
    except Exception:
        return None
    if pp.returncode != 0:
        return None
    h = hashlib.sha256(pp.stdout)
    h.update(" ".join(tu_flags).encode())
    return h.hexdigest()


def _cache_get(key, d, obj):
    if not key:
        return False
    src = os.path.join(CACHE_DIR, key)
    o, a = os.path.join(src, "unit.o"), os.path.join(src, "unit.s")
    if not (os.path.exists(o) and os.path.exists(a)):
        return False
    shutil.copyfile(o, obj)
    shutil.copyfile(a, os.path.join(d, f"unit-hip-amdgcn-amd-amdhsa-{ARCH}.s"))
    return True


def _cache_put(key, obj, asm):
    if not key:
        return
    try:
        dst = os.path.join(CACHE_DIR, key)
        os.makedirs(dst, exist_ok=True)
        shutil.copyfile(obj, os.path.join(dst, "unit.o"))
        shutil.copyfile(asm, os.path.join(dst, "unit.s"))
    except OSError:
        pass


def _compile(defines, verbose):
    """hipcc -c of each translation unit in a scratch directory with
    -save-temps, then the link: the library and the gfx950 assembly of both
    units (concatenated) it was assembled from."""
    work = tempfile.mkdtemp(prefix="dgen_build_")
    tmp = os.path.join(work, "libdgen_hip.so")
    cflags = [f for f in FLAGS if f != "-shared"]
    objs, asms = [], []
    try:
        procs = []
        for tu, extra in TUS:                          # the units compile side by side
            d = os.path.join(work, tu)
            os.makedirs(d)
            obj = os.path.join(d, f"{tu}.o")
            tu_flags = [*cflags, *extra, f"-DDGEN_TU_{tu.upper()}=1", *[f"-D{x}=1" for x in defines]]
            key = _unit_key(tu_flags)
            hit = _cache_get(key, d, obj)
            if hit:
                if verbose:
                    print(f"{tu} unit: unchanged (cached object)", flush=True)
                procs.append((tu, d, obj, None, key))
                continue
            cmd = [hipcc(), *tu_flags, "-save-temps", "-c", "-o", obj, SRC]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((tu, d, obj, subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                                                       text=True, cwd=d), key))
        for tu, d, obj, p, key in procs:
            if p is not None:
                _, err = p.communicate()
                if p.returncode != 0:
                    raise RuntimeError(f"hipcc failed on the {tu} unit ({p.returncode}):\n{err[-4000:]}")
            asm = [f for f in os.listdir(d) if f.endswith(f"-hip-amdgcn-amd-amdhsa-{ARCH}.s")]
            if not asm:
                raise RuntimeError(f"hipcc -save-temps left no device assembly of the {tu} unit to check")
            if p is not None:
                _cache_put(key, obj, os.path.join(d, asm[0]))
            objs.append(obj)
            asms.append(os.path.join(d, asm[0]))
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        res = subprocess.run(cmd, capture_output=True, text=True, cwd=work)
        if res.returncode != 0:
            raise RuntimeError(f"link failed ({res.returncode}):\n{res.stderr[-4000:]}")
        both = os.path.join(work, "device.s")
        with open(both, "w") as out:
            for a in asms:
                with open(a) as f:
                    shutil.copyfileobj(f, out)
    except Exception:
        shutil.rmtree(work, ignore_errors=True)
        raise
    return work, tmp, both


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile, then check the device assembly with the spill guard
    (dgen_amd/spill_guard.py): a 32-lane kernel that spills a live value
    ahead of a divergent branch's exec restore is withdrawn (its batches run
    one agent per wave) and the library rebuilt; a flagged kernel without
    that remedy fails the build.  The outcome is written to
    dgen_amd/lib/build_guard.json."""
    from . import spill_guard
    if not force and not needs_build():
        return OUT
    os.makedirs(OUT_DIR, exist_ok=True)
    # start from the previous build's withdrawals (a rebuild of unchanged
    # units then hits the compile cache at once); the guard still scans every
    # build, and DGEN_GUARD_FRESH=1 starts from none
    defines, carried_flags = [], {}
    if os.environ.get("DGEN_GUARD_FRESH", "0") != "1" and os.path.exists(GUARD):
        try:
            with open(GUARD) as f:
                prev = json.load(f)
            defines = sorted(set(prev.get("withdrawn", [])))
            carried_flags = dict(prev.get("flagged_first_build") or {}) if defines else {}
        except (OSError, ValueError):
            defines, carried_flags = [], {}
    first = None
    for attempt in range(2):
        work, lib, asm = _compile(defines, verbose)
        try:
            if os.environ.get("DGEN_KEEP_ASM"):        # a copy of the device assembly to study
                shutil.copyfile(asm, os.environ["DGEN_KEEP_ASM"])
            hits = spill_guard.scan(asm)
            if attempt == 0:
                first = {k: [b for b, _ in v] for k, v in hits.items()}
            # k_hourly_batt's counted next-day DMA wait must cover the DMA
            dma = spill_guard.day_dma_wait(asm)
            if dma is None:
                raise RuntimeError("k_hourly_batt: no next-day DMA group or counted read-back wait found "
                                   "in the device assembly (the DMA-coverage check cannot see the loop)")
            dma_k, dma_issued = (0, 0) if dma == spill_guard.DRAINED else dma
            if dma_issued < dma_k:
                raise RuntimeError(f"k_hourly_batt: the day read-back waits vmcnt({dma_k}) but only "
                                   f"{dma_issued} vector-memory ops follow the next-day DMA on every path")
            if not hits:
                shutil.copyfile(lib, OUT + ".tmp")
                os.replace(OUT + ".tmp", OUT)
                break
            macros, fatal = spill_guard.remedies(hits)
            if fatal or attempt == 1 or set(macros) <= set(defines):
                raise RuntimeError("spill guard: the compiled kernels spill live values ahead of an exec "
                                   "restore (inactive lanes would reload stale data):\n" + spill_guard.report(hits))
            defines = sorted(set(defines) | set(macros))
            if verbose:
                print("spill guard withdrew:", ", ".join(macros), flush=True)
        finally:
            shutil.rmtree(work, ignore_errors=True)
    with open(GUARD, "w") as f:
        # a withdrawal carried over from the previous build keeps that build's
        # evidence (the kernel it flagged)
        json.dump({"flagged_first_build": {**carried_flags, **(first or {})}, "withdrawn": defines,
                   "day_dma_wait_vmcnt": dma_k, "vmem_ops_after_day_dma": dma_issued}, f, indent=1)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
