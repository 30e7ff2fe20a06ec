"""Host C++ under AddressSanitizer + UBSan: the native collate and the
shared-memory store (csrc/collate.cpp, csrc/shm_store.cpp) built with
``-fsanitize=address,undefined`` (``python -m hydragnn_amd.csrc.build --asan``) and
exercised in a child process that preloads the sanitizer runtimes.  CPU only."""
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys, torch
    torch.ops.load_library(sys.argv[1])
    ops = torch.ops.hydra
    g = torch.Generator().manual_seed(0)
    # collate: per-sample edge lists (dst-sorted) with node offsets
    counts, eis = [], []
    for n in (5, 1, 9, 3, 7):
        E = int(torch.randint(0, 3 * n, (1,), generator=g))
        src = torch.randint(0, n, (E,), generator=g)
        dst = torch.randint(0, n, (E,), generator=g).sort().values
        eis.append(torch.stack([src, dst]).long())
        counts.append(n)
    ei = ops.collate_edges(eis, torch.tensor(counts))
    off = torch.tensor([0] + counts[:-1]).cumsum(0)
    ref = torch.cat([e + o for e, o in zip(eis, off.tolist())], 1)
    assert torch.equal(ei, ref), "collate_edges mismatch"
    N = sum(counts)
    drp, srp, sperm = ops.csr_from_edges(ei[0].int(), ei[1].int(), N)
    assert torch.equal(drp[1:] - drp[:-1], torch.bincount(ei[1], minlength=N).int())
    assert torch.equal(srp[1:] - srp[:-1], torch.bincount(ei[0], minlength=N).int())
    assert torch.equal(sperm.long(), torch.argsort(ei[0], stable=True))
    # empty graph
    drp, srp, sperm = ops.csr_from_edges(torch.zeros(0, dtype=torch.int32), torch.zeros(0, dtype=torch.int32), 4)
    assert drp.tolist() == [0] * 5 and sperm.numel() == 0
    # shared-memory store round trip
    name = f"hy_asan_{os.getpid()}"
    h = ops.shm_store_create(name, 4096)
    x = torch.arange(256, dtype=torch.float32)
    ops.shm_store_write(h, 128, x)
    y = ops.shm_store_read(h, 128, 1024).view(torch.float32)
    assert torch.equal(x, y)
    v = ops.shm_store_view(h, 128, 1024)
    assert v.numel() == 1024 and ops.shm_store_size(h) == 4096
    h2 = ops.shm_store_attach(name)
    assert torch.equal(ops.shm_store_read(h2, 128, 1024).view(torch.float32), x)
    ops.shm_store_close(h2)
    ops.shm_store_close(h)
    ops.shm_store_unlink(name)
    print("ASAN_OK")
""")


def _runtime(lib):
    out = subprocess.run(["g++", f"-print-file-name={lib}"], capture_output=True, text=True).stdout.strip()
    return out if os.path.isabs(out) and os.path.exists(out) else None


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_code_under_asan_ubsan(tmp_path):
    asan, ubsan = _runtime("libasan.so"), _runtime("libubsan.so")
    if asan is None or ubsan is None:
        pytest.skip("sanitizer runtimes not installed")
    sys.path.insert(0, ROOT)
    from hydragnn_amd.csrc import build

    lib = build.ASAN_OUT
    srcs = [os.path.join(build.HERE, f) for f in ("collate.cpp", "shm_store.cpp")]
    if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(s) for s in srcs):
        build.build_asan(verbose=False)
    script = tmp_path / "asan_probe.py"
    script.write_text(SCRIPT)
    env = dict(os.environ, LD_PRELOAD=f"{asan}:{ubsan}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1:exitcode=23",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([sys.executable, str(script), lib], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "ASAN_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
