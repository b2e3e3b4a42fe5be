"""SURVEY §5 (race detection / sanitizers): the host side of the C ABI under
AddressSanitizer, on the CPU.

csrc/Makefile `asan` builds libsel_asan.so with ASan on the host code only
(-Xarch_host -fsanitize=address; the device code is not sanitised and never
runs here).  tests/asan_host_calls.py then drives every host-side entry point
that needs no GPU — argument validation error paths, workspace / plan /
geometry / dispatch-decision functions over a sweep of shapes, the host-filled
resampling tap table, kernel names written into short buffers — in a child
interpreter with the clang ASan runtime preloaded.  Any ASan report aborts the
child.  (It found two integer divisions by zero in workspace sizing for
invalid shapes, fixed in round 4.)"""
import glob
import os
import subprocess
import sys

from conftest import REPO

CSRC = os.path.join(REPO, "dl-speech-enhancement_amd", "csrc")
LIB = os.path.join(REPO, "dl-speech-enhancement_amd", "sel", "libsel_asan.so")


def _asan_runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    assert hits, "clang ASan runtime not found under /opt/rocm/lib/llvm"
    return hits[-1]


def test_host_abi_under_address_sanitizer():
    # incremental: build() has normally built it already
    subprocess.check_call(["make", "-C", CSRC, f"-j{min(8, os.cpu_count() or 4)}", "asan"],
                          stdout=subprocess.DEVNULL, timeout=900)
    env = dict(os.environ, LD_PRELOAD=_asan_runtime(), ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "asan_host_calls.py"), LIB], env=env,
                       capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0 and "AddressSanitizer" not in out, out[-4000:]
    assert out.strip().splitlines()[-1].startswith("ok "), out[-2000:]
