"""In-tree build of the HIP kernel library for gfx950.

The kernels are plain HIP (no torch headers) exposed through a C ABI, so each
translation unit compiles in seconds with ``hipcc --offload-arch=gfx950`` and
the resulting ``_sc_kernels.so`` travels with the repository snapshot.  A sha256
of every source, header and flag is compiled into the library (``sc_source_hash``);
objects are rebuilt when their inputs' digest changes (not only their mtimes), and the
loader refuses a library whose hash does not match the tree (``_lib.lib()``).  The
library is loaded with ctypes *after* ``import torch`` so its NEEDED
``libamdhip64.so.7`` resolves to the HIP runtime torch already mapped (one
runtime per process).

Usage::

    python -m sparse_coding__amd.ops.build          # incremental
    python -m sparse_coding__amd.ops.build --force  # full rebuild
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
LIB = HERE / "_sc_kernels.so"
RUNTIME_LIB = HERE / "_sc_runtime.so"
ARCH = os.environ.get("SC_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found; the MI355X kernels need ROCm's hipcc")


def _kernel_sources():
    return sorted(CSRC.glob("*.hip"))


def _runtime_sources():
    return sorted((CSRC / "runtime").glob("*.cpp"))


def _headers():
    return sorted(CSRC.glob("*.h")) + sorted((CSRC / "runtime").glob("*.h"))


HASH_TAG = b"SC_SOURCE_HASH:"


def _digest(paths, extra: str = "") -> str:
    h = hashlib.sha256(extra.encode())
    for p in paths:
        h.update(p.relative_to(CSRC).as_posix().encode() + b"\0")
        h.update(p.read_bytes())
        h.update(b"\0")
    return h.hexdigest()


def source_hash() -> str:
    """sha256 over every kernel source, header and build flag: the identity of the library
    that ``build()`` produces from this tree.  It is compiled INTO ``_sc_kernels.so``
    (``sc_source_hash()``), and ``_lib.lib()`` refuses a library whose hash differs."""
    return _digest(_kernel_sources() + _headers(), f"{ARCH}|{sorted(EXTRA_FLAGS.items())}")


def embedded_hash(path: Path = None) -> str:
    """The source hash baked into a built library (read from its bytes, without loading it)."""
    data = Path(path or LIB).read_bytes()
    i = data.find(HASH_TAG)
    if i < 0:
        return ""
    return data[i + len(HASH_TAG): i + len(HASH_TAG) + 64].decode("ascii", "replace")


def _stale(target: Path, deps, key: str = None) -> bool:
    """Rebuild when the target is missing, older than a dependency, or (``key``) built from
    different contents (a sidecar ``.hash`` records the digest the object was built from)."""
    if not target.exists():
        return True
    if key is not None:
        side = target.with_suffix(target.suffix + ".hash")
        if not side.exists() or side.read_text() != key:
            return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


# Per-source extra flags.  sae_gemm.hip (128x128 blocks, software-pipelined K loop with two
# MFMA groups per iteration) uses the VGPR form of the MFMA: with AGPR accumulators the
# register allocator rotated them through v_accvgpr copies every iteration.
EXTRA_FLAGS = {"sae_gemm.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"],
               "sae_gemm_256x128.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def _compile_one(src: Path, force: bool) -> Path:
    obj = BUILD / (src.stem + ".o")
    key = _digest([src, *_headers()], f"{ARCH}|{EXTRA_FLAGS.get(src.name, [])}")
    if not force and not _stale(obj, [src, *_headers()], key):
        return obj
    cmd = [
        _hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-munsafe-fp-atomics",
        f"-I{CSRC}",
        *EXTRA_FLAGS.get(src.name, []),
        "-c",
        str(src),
        "-o",
        str(obj),
    ]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{res.stderr}")
    obj.with_suffix(obj.suffix + ".hash").write_text(key)
    return obj


def _provenance_object(digest: str) -> Path:
    """A one-function host object carrying the source hash (``sc_source_hash()``)."""
    src = BUILD / "provenance.cpp"
    src.write_text('extern "C" const char* sc_source_hash() {\n'
                   f'  static const char tag[] = "{HASH_TAG.decode()}{digest}";\n'
                   f'  return tag + {len(HASH_TAG)};\n}}\n')
    obj = BUILD / "provenance.o"
    cxx = shutil.which("g++") or "c++"
    res = subprocess.run([cxx, "-O2", "-fPIC", "-c", str(src), "-o", str(obj)], capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"provenance object failed:\n{res.stderr}")
    return obj


def _compile_host(src: Path, force: bool) -> Path:
    obj = BUILD / (src.stem + ".host.o")
    if not force and not _stale(obj, [src, *_headers()]):
        return obj
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-pthread", f"-I{CSRC}", "-c", str(src), "-o", str(obj)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"g++ failed for {src.name}:\n{res.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> Path:
    BUILD.mkdir(exist_ok=True)
    srcs = _kernel_sources()
    rt_srcs = _runtime_sources()
    workers = max(1, min(8, os.cpu_count() or 1, len(srcs) + len(rt_srcs)))
    with cf.ThreadPoolExecutor(workers) as ex:
        objs = list(ex.map(lambda s: _compile_one(s, force), srcs))
        rt_objs = list(ex.map(lambda s: _compile_host(s, force), rt_srcs))
    digest = source_hash()
    if force or _stale(LIB, objs) or embedded_hash(LIB) != digest:
        objs = objs + [_provenance_object(digest)]
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(LIB)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed:\n{res.stderr}")
        if verbose:
            print(f"[sc-build] linked {LIB.name} from {len(objs)} objects")
    if rt_objs and (force or _stale(RUNTIME_LIB, rt_objs)):
        cxx = shutil.which("g++") or "c++"
        cmd = [cxx, "-shared", "-fPIC", "-pthread", *map(str, rt_objs), "-o", str(RUNTIME_LIB)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"runtime link failed:\n{res.stderr}")
        if verbose:
            print(f"[sc-build] linked {RUNTIME_LIB.name} from {len(rt_objs)} objects")
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    args = ap.parse_args(argv)
    build(force=args.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
