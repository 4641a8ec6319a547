"""Compile csrc/*.hip into libsslmae.so for gfx950 (hipcc, in-tree, no JIT cache).

The objects are rebuilt only when a source or header is newer than the library.
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_PKG = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT_PKG, "csrc")
REPO = os.path.dirname(ROOT_PKG)
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG_DIR, "libsslmae.so")
BUILD = os.path.join(ROOT_PKG, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SM_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC, "-I", INCLUDE,
         "-Wno-unused-result", "-munsafe-fp-atomics"]
# Per-source extra flags.  fed.hip reproduces the reference's separately rounded
# multiply and add bit for bit; hipcc's default -ffp-contract=fast ignores
# `#pragma clang fp contract`, so contraction is switched off for that file.
FILE_FLAGS = {"fed.hip": ["-ffp-contract=off"], "attention.hip": ["-fno-slp-vectorize"], "gemm.hip": ["-fno-slp-vectorize"]}


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _flag_tag(src):
    import zlib
    flags = " ".join([HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []))
    return f"{zlib.crc32(flags.encode()):08x}"


STAMP = LIB + ".flags"   # the flag tags the library was linked from (one line per source)


def _stamp_text():
    return "".join(f"{os.path.basename(s)} {_flag_tag(s)}\n" for s in _sources())


def needs_build():
    lib_t = os.path.getmtime(LIB) if os.path.exists(LIB) else -1.0
    if lib_t < _newest_input():
        return True
    # a compile-flag change leaves the sources older than the library: rebuild when the
    # library was linked from objects built with other flags (stamp written at link time).
    # A library without a stamp cannot show which flags it was built with: stale.
    if not os.path.exists(STAMP):
        return True
    with open(STAMP) as f:
        return f.read() != _stamp_text()


def _newest_input():
    files = _sources() + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max(os.path.getmtime(f) for f in files)


def build(verbose=False, jobs=None):
    if not needs_build():
        return LIB
    os.makedirs(BUILD, exist_ok=True)
    srcs = _sources()
    # the object name carries a hash of its compile flags, so a flag change rebuilds it
    objs = [os.path.join(BUILD, f"{os.path.basename(s)}.{_flag_tag(s)}.o") for s in srcs]

    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    hdr_t = max(os.path.getmtime(f) for f in headers) if headers else 0.0

    def compile_one(pair):
        src, obj = pair
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_t):
            return obj   # object up to date with its source and every header
        cmd = [HIPCC] + FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr[-6000:]}")
        if verbose:
            print("compiled", os.path.basename(src), file=sys.stderr)
        return obj

    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 2) // 2), 8)
    with ThreadPoolExecutor(jobs) as ex:
        list(ex.map(compile_one, zip(srcs, objs)))
    tmp = LIB + ".tmp"
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    os.replace(tmp, LIB)
    with open(STAMP, "w") as f:
        f.write(_stamp_text())
    return LIB


ARENA_SRC = os.path.join(CSRC, "arena.cpp")
ARENA_LIB = os.path.join(PKG_DIR, "libsmarena.so")


def build_arena():
    """Host-only C++ (csrc/arena.cpp, the device-memory arena behind PyTorch's
    pluggable-allocator hook) into libsmarena.so, linked against the HIP runtime."""
    if os.path.exists(ARENA_LIB) and os.path.getmtime(ARENA_LIB) >= os.path.getmtime(ARENA_SRC):
        return ARENA_LIB
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    tmp = ARENA_LIB + ".tmp"
    cmd = [os.environ.get("CXX", "g++"), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(rocm, "include"), ARENA_SRC,
           "-L", os.path.join(rocm, "lib"), "-lamdhip64", f"-Wl,-rpath,{os.path.join(rocm, 'lib')}", "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"arena build failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, ARENA_LIB)
    return ARENA_LIB


if __name__ == "__main__":
    print(build(verbose=True))
    print(build_arena())
