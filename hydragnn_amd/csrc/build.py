"""In-tree builder for the gfx950 native library ``hydragnn_amd/_C.so``.

Every ``*.hip`` / ``*.cpp`` file in this directory is compiled directly with
``hipcc --offload-arch=gfx950`` (no hipify, no CUDA shims) against the PyTorch
headers and linked into one shared object whose ops register themselves under
``torch.ops.hydra.*`` (TORCH_LIBRARY).  Objects are cached in ``csrc/build/``
and rebuilt unless the digest stored with the object matches its source, the local
headers and the flags; the library's digest is derived from the digests of the objects
it was linked from.

Usage:  python -m hydragnn_amd.csrc.build [-j N] [--force]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
OUT = os.path.join(PKG, "_C.so")
BUILD = os.path.join(HERE, "build")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")


def _torch_paths():
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hipcc():
    for c in (os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc"), "hipcc"):
        if os.path.sep not in c or os.path.exists(c):
            return c
    return "hipcc"


def sources():
    return sorted(glob.glob(os.path.join(HERE, "*.hip")) + glob.glob(os.path.join(HERE, "*.cpp")))


def _headers_bytes():
    out = b""
    for h in sorted(glob.glob(os.path.join(HERE, "*.h"))):
        with open(h, "rb") as fh:
            out += os.path.basename(h).encode() + fh.read()
    return out


def object_digest(src, flags=(ARCH, "-O3"), headers=None):
    """sha256 of ONE translation unit's inputs: its bytes, every local header and the
    compile flags.  Stored beside the object (``<obj>.srchash``); an object is reused only
    when this digest matches (not by mtime: a copy that preserves times cannot pass off
    stale objects)."""
    import hashlib

    h = hashlib.sha256()
    h.update(os.path.basename(src).encode())
    with open(src, "rb") as fh:
        h.update(fh.read())
    h.update(_headers_bytes() if headers is None else headers)
    h.update("\0".join(flags).encode())
    return h.hexdigest()


def source_digest():
    """sha256 over the per-object digests of every native source (names + bytes + headers):
    written next to the library at link time FROM THE DIGESTS OF THE OBJECTS LINKED, and
    checked at load time, so a stale ``_C.so`` (sources edited, library not rebuilt) fails
    loudly instead of running old kernels."""
    import hashlib

    hb = _headers_bytes()
    h = hashlib.sha256()
    for f in sources():
        h.update(object_digest(f, headers=hb).encode())
    return h.hexdigest()


def _read(path):
    try:
        with open(path) as fh:
            return fh.read().strip()
    except OSError:
        return None


def _compile(src, inc, abi, force):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    want = object_digest(src)
    if (not force) and os.path.exists(obj) and _read(obj + ".srchash") == want:
        return obj, None, False
    py_inc = sysconfig.get_paths()["include"]
    cmd = [
        _hipcc(),
        f"--offload-arch={ARCH}",
        "-O3",
        "-fPIC",
        "-std=c++17",
        "-ffp-contract=fast-honor-pragmas",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
        f"-I{HERE}",
        f"-I{py_inc}",
    ] + [f"-I{p}" for p in inc] + ["-c", src, "-o", obj]
    if os.path.exists(obj + ".srchash"):
        os.remove(obj + ".srchash")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"FAILED: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}", True
    with open(obj + ".srchash", "w") as fh:
        fh.write(want + "\n")
    return obj, None, True


def build(jobs=None, force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    inc, lib, abi = _torch_paths()
    srcs = sources()
    jobs = jobs or min(8, os.cpu_count() or 4, len(srcs) or 1)
    objs, errs, rebuilt = [], [], False
    with cf.ThreadPoolExecutor(jobs) as ex:
        for obj, err, fresh in ex.map(lambda s: _compile(s, inc, abi, force), srcs):
            objs.append(obj)
            rebuilt |= fresh
            if err:
                errs.append(err)
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    # the library digest is derived from the digests stored with the objects being linked
    import hashlib

    h = hashlib.sha256()
    for o in objs:
        d = _read(o + ".srchash")
        if d is None:
            raise RuntimeError(f"{o} has no source digest")
        h.update(d.encode())
    linked = h.hexdigest()
    if force or rebuilt or not os.path.exists(OUT) or _read(OUT + ".srchash") != linked:
        if os.path.exists(OUT + ".srchash"):
            os.remove(OUT + ".srchash")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT] + objs + [
            f"-L{lib}", "-ltorch", "-ltorch_cpu", "-lc10", "-lc10_hip", "-ltorch_hip", f"-Wl,-rpath,{lib}",
        ]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        with open(OUT + ".srchash", "w") as fh:
            fh.write(linked + "\n")
    if verbose:
        print(f"[hydragnn_amd] built {OUT} from {len(srcs)} sources for {ARCH}")
    return OUT


ASAN_OUT = os.path.join(BUILD, "_C_host_asan.so")  # build dir: host-only, never shipped to the GPU box


def build_asan(verbose=True):
    """Sanitizer flavour of the HOST C++ sources (collate.cpp, shm_store.cpp): g++ with
    -fsanitize=address,undefined into ``_C_host_asan.so``.  GPU code is never
    sanitized (not available on this pool); load this library alone, in a process started
    with ``LD_PRELOAD`` of the ASan/UBSan runtimes (tests/test_host_asan.py)."""
    inc, lib, abi = _torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "*.cpp")))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared", "-fsanitize=address,undefined",
           "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-Wno-deprecated-declarations", f"-I{HERE}", f"-I{sysconfig.get_paths()['include']}"] + \
        [f"-I{p}" for p in inc] + srcs + ["-o", ASAN_OUT, f"-L{lib}", "-ltorch", "-ltorch_cpu", "-lc10",
                                           f"-Wl,-rpath,{lib}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"asan build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[hydragnn_amd] built {ASAN_OUT} (host sources, ASan + UBSan)")
    return ASAN_OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asan", action="store_true", help="build the sanitized host-code library instead")
    a = ap.parse_args()
    try:
        if a.asan:
            build_asan()
            sys.exit(0)
        build(a.j, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
