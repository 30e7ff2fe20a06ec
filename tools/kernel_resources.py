"""Per-kernel register / scratch / occupancy report of the native sources (compile-time,
no GPU): ``python tools/kernel_resources.py [file.hip ...] [--all]``.  Kernels that spill
to scratch (private memory: every access is a global-memory round trip) are listed first;
``--all`` prints every kernel."""
import argparse
import glob
import os
import re
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "hydragnn_amd", "csrc")


def report(src):
    import torch

    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api", "include"),
           sysconfig.get_paths()["include"]]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", os.devnull,
           "--offload-device-only", "-Rpass-analysis=kernel-resource-usage", "-DUSE_ROCM",
           f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"]
    for i in inc:
        cmd += ["-I", i]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=CSRC)
    out, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
            m = re.search(pat, line)
            if m and cur is not None:
                cur[key] = int(m.group(1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="*")
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    files = a.files or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    bad = 0
    for f in files:
        for k in report(os.path.abspath(f)):
            if a.all or k.get("scratch", 0) > 0:
                bad += k.get("scratch", 0) > 0
                print(f"{os.path.basename(f):18s} scratch {k.get('scratch', 0):4d}  vgpr {k.get('vgpr', 0):3d}  "
                      f"agpr {k.get('agpr', 0):3d}  lds {k.get('lds', 0):6d}  occ {k.get('occ', 0)}  {k['name'][:90]}")
    print(f"{bad} kernel(s) with scratch")
    return 0


if __name__ == "__main__":
    sys.exit(main())
