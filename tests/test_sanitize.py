"""Host-side sanitizer run ("host ASan/UBSan build of the C++ CPU path").

`make -C ska-pst-dsp-model_amd SANITIZE=1` builds lib/libpfb_hip_san.so: the same library
with AddressSanitizer + UndefinedBehaviorSanitizer on its host code (argument checks, plan
descriptors and host tables, stream bookkeeping, error channel; the device code is built
as usual).  This test runs the C-ABI CPU tests (tests/test_abi.py, tests/test_abi_args.py)
in a child process with that library and the shared ASan runtime preloaded; any ASan
report or UBSan runtime error aborts the child (halt_on_error / -fno-sanitize-recover).
The log of a run is kept under profiles/ (r05_host_asan_ubsan.log)."""
import glob
import os
import subprocess
import sys

import pytest

from conftest import REPO

SAN_LIB = os.path.join(REPO, "ska-pst-dsp-model_amd", "lib", "libpfb_hip_san.so")


def _asan_runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


def run_sanitized(log_path=None):
    rt = _asan_runtime()
    env = dict(os.environ)
    env.update(LD_PRELOAD=rt, PFB_HIP_LIB=SAN_LIB,
               # the interpreter's own allocations are not the library's: no leak report
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    cmd = [sys.executable, "-m", "pytest", "-q", "-p", "no:cacheprovider",
           os.path.join(REPO, "tests", "test_abi.py"), os.path.join(REPO, "tests", "test_abi_args.py")]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    if log_path:
        with open(log_path, "w") as f:
            f.write(f"$ LD_PRELOAD={rt} PFB_HIP_LIB={SAN_LIB} {' '.join(cmd)}\n{out}\nexit {r.returncode}\n")
    return r.returncode, out


@pytest.mark.skipif(not os.path.exists(SAN_LIB) or _asan_runtime() is None,
                    reason="sanitizer build not present (make -C ska-pst-dsp-model_amd SANITIZE=1)")
def test_abi_under_asan_ubsan():
    with open(SAN_LIB, "rb") as f:  # the library really is instrumented
        blob = f.read()
    assert b"__asan_report_load" in blob and b"__ubsan_handle_" in blob
    rc, out = run_sanitized()
    assert "AddressSanitizer" not in out, out[-4000:]
    assert "runtime error" not in out, out[-4000:]
    assert rc == 0, out[-4000:]
    assert " passed" in out


if __name__ == "__main__":
    rc, _ = run_sanitized(os.path.join(REPO, "profiles", "r05_host_asan_ubsan.log"))
    sys.exit(rc)
