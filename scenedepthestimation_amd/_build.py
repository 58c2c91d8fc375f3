"""Build libsde.so (all HIP kernels + the C ABI of include/sde.h) for gfx950, in-tree.

    python -m scenedepthestimation_amd._build [--force]

hipcc cross-compiles without a GPU.  The .so lands next to this file so it
travels with the repository snapshot to the GPU box (it is git-ignored).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import re
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OBJ = os.path.join(PKG, "_obj")
LIB = os.path.join(PKG, "libsde.so")
ARCH = os.environ.get("SDE_OFFLOAD_ARCH", "gfx950")

# -ffp-contract=off: the cost volume must reproduce NumPy's separately rounded
# products and sums bit for bit; the SGM recurrence has no products but keep the
# whole library uniform.  No fast-math: IEEE compares, signed zeros and f32
# denormals (gfx950 default mode keeps them) are part of the parity contract.
HIPCC_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-fvisibility=hidden", "-Wall", "-Wno-unused-function", "-I" + INCLUDE, "-I" + CSRC]


# cv_row.hip: the certified row-sweep kernel's per-score max / median / compare run without
# NaN canonicalisation (IEEE mode off).  Its certificate takes every decision that must survive
# non-finite input on integer bit tests, and its exact arithmetic (no NaN, no contraction) is
# unaffected; nothing else is built this way.
PER_FILE_FLAGS = {"cv_row.hip": ["-fno-honor-nans", "-mno-amdgpu-ieee"]}


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm is required to build libsde.so)")


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(INCLUDE, "sde.h"))
    return max(os.path.getmtime(h) for h in hs)


def _compile(src: str, force: bool) -> str:
    obj = os.path.join(OBJ, os.path.basename(src)[:-4] + ".o")
    if not force and os.path.exists(obj) and \
            os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime()):
        return obj
    cmd = [hipcc()] + HIPCC_FLAGS + PER_FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


_EXIT_CALL = re.compile(r"\b(call|jmp)\s+[0-9a-f]+\s+<(atexit|__cxa_atexit|on_exit)(@plt)?>")
_FUNC_HDR = re.compile(r"^[0-9a-f]+ <(.+)>:$")


def exit_hooks(lib: str):
    """Exit-time code registered by `lib` (a rocprofv3 run of a cooperative-launch variant
    crashed inside exit(), in a handler that reached the HIP runtime after the profiler had finalised).
    Returns [(function, instruction)] for every call of atexit / __cxa_atexit / on_exit outside a hipcc
    module constructor (__hip_module_ctor registers __hip_module_dtor, which unregisters the fat binary:
    the one exit-time HIP call every hipcc object carries), plus the .fini_array entries other than the
    C runtime's __do_fini.  Empty = no C++ static destructor, function-local static with a destructor or
    explicit atexit handler of ours runs at exit."""
    objdump = shutil.which("objdump") or "/opt/rocm/lib/llvm/bin/llvm-objdump"
    r = subprocess.run([objdump, "-d", "--no-show-raw-insn", lib], capture_output=True, text=True, check=True)
    bad, func = [], "?"
    for line in r.stdout.splitlines():
        m = _FUNC_HDR.match(line.strip())
        if m:
            func = m.group(1)
            continue
        if _EXIT_CALL.search(line) and func not in ("__hip_module_ctor", "atexit", "__cxa_atexit@plt"):
            bad.append((func, line.strip()))
    nm = subprocess.run(["nm", lib], capture_output=True, text=True, check=True).stdout
    addr = {}
    for ln in nm.splitlines():
        parts = ln.split()
        if len(parts) == 3:
            addr.setdefault(int(parts[0], 16), parts[2])
    # .fini_array entries are R_X86_64_RELATIVE relocations into the section: their addends are the targets
    sec = subprocess.run(["readelf", "-S", "-W", lib], capture_output=True, text=True, check=True).stdout
    lo = hi = 0
    for ln in sec.splitlines():
        if ".fini_array" in ln:
            t = ln.split("]", 1)[1].split()
            lo = int(t[2], 16)
            hi = lo + int(t[4], 16)
    rel = subprocess.run(["readelf", "-r", "-W", lib], capture_output=True, text=True, check=True).stdout
    for ln in rel.splitlines():
        t = ln.split()
        if len(t) >= 4 and t[2] == "R_X86_64_RELATIVE":
            off = int(t[0], 16)
            if lo <= off < hi:
                name = addr.get(int(t[3], 16), t[3])
                if name not in ("__do_fini", "__do_global_dtors_aux"):
                    bad.append((".fini_array", name))
    return bad


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        # ISA lint (store-data overwrite, _isa_lint.py): a schedule that lost values on hardware
        # is a build error, before the library is replaced
        from . import _isa_lint
        _isa_lint.check(objs)
        tmp = LIB + ".tmp"
        cmd = [hipcc(), "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        hooks = exit_hooks(tmp)
        if hooks:
            raise RuntimeError("libsde.so would run code of its own inside exit() (after the HIP runtime or a "
                               "profiler may have finalised): " + "; ".join(f"{f}: {i}" for f, i in hooks[:10]))
        os.replace(tmp, LIB)
    if verbose:
        print(f"built {LIB}", file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
