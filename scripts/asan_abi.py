"""Host-side AddressSanitizer + UBSan check of the C ABI's argument handling.

The library is rebuilt with its HOST code (every extern "C" entry point of
include/sm_api.h: argument checks, workspace sizing, launch configuration) instrumented by
-fsanitize=address,undefined (each flag after -Xarch_host; the gfx950 device code is not
instrumented and never runs here) into a throw-away shared library, and every entry point is called through ctypes with invalid
and degenerate arguments (negative / zero / tiny sizes, NULL pointers, zero workspace).
No GPU is needed: an argument error returns before any HIP call, and a call that gets as
far as a launch fails in the HIP runtime (no device / no code object) and returns its
status.  Any sanitizer report fails the run.

    python scripts/asan_abi.py build OUT_DIR     # compile + link OUT_DIR/libsslmae_asan.so
    python scripts/asan_abi.py run LIB           # (child, under LD_PRELOAD=asan) call every entry point
    python scripts/asan_abi.py check OUT_DIR     # both; exit 0 iff no sanitizer report
"""
import ctypes
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ssl-vit-video-analytics_amd", "csrc")
LIBPY = os.path.join(ROOT, "ssl-vit-video-analytics_amd", "ssl_mae_amd", "_lib.py")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SAN = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined", "-Xarch_host",
       "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=all"]


def build(out):
    os.makedirs(out, exist_ok=True)
    objs = []
    for src in sorted(glob.glob(os.path.join(CSRC, "*.hip"))):
        obj = os.path.join(out, os.path.basename(src) + ".o")
        deps = [src, os.path.join(CSRC, "common.h"), os.path.join(ROOT, "include", "sm_api.h")]
        if os.path.exists(obj) and os.path.getmtime(obj) > max(os.path.getmtime(d) for d in deps):
            objs.append(obj)   # up to date (repeated runs in one OUT_DIR)
            continue
        cmd = [HIPCC, "--offload-arch=gfx950", "-g", "-O1", "-std=c++17", "-fPIC", "-I", CSRC,
               "-I", os.path.join(ROOT, "include"), "-Wno-unused-result"] + SAN + ["-c", src, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{' '.join(cmd)}\n{r.stderr[-4000:]}")
        objs.append(obj)
    lib = os.path.join(out, "libsslmae_asan.so")
    r = subprocess.run([HIPCC, "-shared", "--offload-arch=gfx950", "-Xarch_host", "-fsanitize=address",
                        "-Xarch_host", "-fsanitize=undefined", "-o", lib] + objs,
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-4000:])
    return lib


def signatures():
    """_lib._SIGS evaluated without importing torch (name -> (restype, argtypes))."""
    src = open(LIBPY).read()
    m = re.search(r"^_SIGS = (\{.*?^\})", src, re.S | re.M)
    ns = {"_c_i32": ctypes.c_int, "_c_i64": ctypes.c_int64, "_c_f32": ctypes.c_float,
          "_c_u64": ctypes.c_uint64, "_c_p": ctypes.c_void_p}
    return eval(m.group(1), ns)   # noqa: S307 -- our own source file


def run(lib_path):
    lib = ctypes.CDLL(lib_path)
    sigs = signatures()
    patterns = {"negative": (-1, -1, 0.0), "zero": (0, 0, 0.0), "one": (1, 1, 0.5), "odd": (7, 7, 0.1),
                "dtype_bad": (5, 5, -1.0)}
    ncalls = 0
    for name, (res, argt) in sorted(sigs.items()):
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, argt
        for pname, (iv, lv, fv) in patterns.items():
            args = []
            for t in argt:
                if t is ctypes.c_void_p:
                    args.append(None)
                elif t is ctypes.c_float:
                    args.append(fv)
                elif t is ctypes.c_uint64:
                    args.append(0)
                elif t is ctypes.c_int64:
                    args.append(lv)
                else:
                    args.append(iv)
            rc = fn(*args)
            if name.endswith(("_workspace_bytes", "_partial_rows")):
                assert isinstance(rc, int), (name, pname, rc)
            ncalls += 1
    print(f"asan_abi: {len(sigs)} entry points, {ncalls} calls, no sanitizer report", flush=True)


def check(out):
    lib = build(out)
    rt = subprocess.run(["/opt/rocm/llvm/bin/clang++", "-print-file-name=libclang_rt.asan-x86_64.so"],
                        capture_output=True, text=True).stdout.strip()
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "run", lib], capture_output=True, text=True,
                       env=env, timeout=600)
    bad = "AddressSanitizer" in r.stderr or "runtime error:" in r.stderr
    print(r.stdout[-2000:])
    if r.returncode != 0 or bad:
        print(r.stderr[-6000:])
        return 1
    return 0


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "build":
        print(build(sys.argv[2]))
    elif what == "run":
        run(sys.argv[2])
    else:
        sys.exit(check(sys.argv[2]))
