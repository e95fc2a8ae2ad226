"""Build the native library ``rphedge/_lib/librphedge.so`` for gfx950.

All HIP kernels (``csrc/*.hip``) and the C++ runtime (``csrc/*.cpp``) are
compiled by ``hipcc --offload-arch=gfx950`` into ONE shared object with a C ABI
(bound by ctypes in :mod:`rphedge.ops.native`).  The build is in-tree so the
``.so`` travels with the repository snapshot to the GPU box.

Usage::

    python -m rphedge.build            # incremental (hash of sources)
    python -m rphedge.build --force
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "_lib"
LIB = LIBDIR / "librphedge.so"
STAMP = LIBDIR / "librphedge.sha256"
ARCH = os.environ.get("RPH_OFFLOAD_ARCH", "gfx950")


# per-translation-unit code-generation flags
PER_FILE_FLAGS = {
    # LM solve: keep the fp64 MFMA accumulators of the Cholesky trailing update
    # in VGPRs (the default AGPR form copied them across every panel: ~650
    # v_accvgpr moves per solve)
    "hedge_lm.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"],
}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build rphedge)")


def sources() -> list[Path]:
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _digest(extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for p in sorted(sources() + list(CSRC.glob("*.h"))):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False, debug: bool = False, asan: bool = False,
          defines: tuple = (), name: str | None = None) -> Path:
    """Compile csrc/ for gfx950.  ``asan`` builds a host-AddressSanitizer variant
    (``librphedge_asan.so``; device code is not instrumented — GPU ASan is not
    available on this pool) for host-side race/memory debugging."""
    LIBDIR.mkdir(parents=True, exist_ok=True)
    flags = [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-shared",
        "-Wno-unused-result",
        f"-I{CSRC}",
        "-L/opt/rocm/lib",
        "-lrccl",
    ]
    lib, stamp = LIB, STAMP
    if debug:  # device RPH_DASSERT checks + host debug info: librphedge_debug.so (RPH_NATIVE_LIB=debug)
        flags += ["-g", "-DRPH_DEBUG=1"]
        lib, stamp = LIBDIR / "librphedge_debug.so", LIBDIR / "librphedge_debug.sha256"
    if asan:
        flags += ["-g", "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"]
        lib, stamp = LIBDIR / "librphedge_asan.so", LIBDIR / "librphedge_asan.sha256"
    if name:  # A/B variant: extra -D defines, rphedge/_lib/ab/librphedge_<name>.so (RPH_NATIVE_LIB=<path>)
        flags += [f"-D{x}" for x in defines]
        (LIBDIR / "ab").mkdir(exist_ok=True)
        lib, stamp = LIBDIR / "ab" / f"librphedge_{name}.so", LIBDIR / "ab" / f"librphedge_{name}.sha256"
    digest = _digest(" ".join(flags) + repr(sorted(PER_FILE_FLAGS.items())))
    if not force and lib.exists() and stamp.exists() and stamp.read_text().strip() == digest:
        return lib
    tmp = lib.with_suffix(".so.tmp")
    # one hipcc per translation unit in parallel (the kernels are template-heavy),
    # then one link into the shared object
    objdir = LIBDIR / ("obj_asan" if asan else "obj_debug" if debug else f"obj_{name}" if name else "obj")
    objdir.mkdir(exist_ok=True)
    cflags = [f for f in flags if f not in ("-shared", "-lrccl") and not f.startswith("-L")]
    jobs = []
    for src in sources():
        obj = objdir / (src.name + ".o")
        jobs.append(([_hipcc(), *cflags, *PER_FILE_FLAGS.get(src.name, []), "-c", str(src), "-o", str(obj)], obj))
    from concurrent.futures import ThreadPoolExecutor

    def _run(job):
        cmd, _ = job
        if verbose:
            print(" ".join(cmd), flush=True)
        return subprocess.run(cmd, capture_output=True, text=True)

    with ThreadPoolExecutor(max_workers=min(len(jobs), max(1, (os.cpu_count() or 2)))) as ex:
        results = list(ex.map(_run, jobs))
    for (cmd, _), res in zip(jobs, results):
        if res.returncode != 0:
            raise RuntimeError(f"hipcc failed ({res.returncode}): {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    cmd = [_hipcc(), *flags, *[str(o) for _, o in jobs], "-o", str(tmp)]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc link failed ({res.returncode}):\n{res.stdout}\n{res.stderr}")
    os.replace(tmp, lib)
    stamp.write_text(digest)
    return lib


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host AddressSanitizer variant")
    ap.add_argument("--variant", default=None, help="A/B library name (with --define)")
    ap.add_argument("--define", action="append", default=[], help="extra preprocessor define (A/B variant)")
    ap.add_argument("-v", "--verbose", action="store_true")
    a = ap.parse_args(argv)
    lib = build(force=a.force, verbose=a.verbose, debug=a.debug, asan=a.asan, defines=tuple(a.define),
                name=a.variant)
    print(lib)
    return 0


if __name__ == "__main__":
    sys.exit(main())
