"""Host sanitizer leg (SURVEY.md §5 "race detection / sanitizers"): the C-ABI argument
validation of the HIP library and the oracle's C restatement run under AddressSanitizer +
UndefinedBehaviorSanitizer on the CPU.

Both are rebuilt with host-only instrumentation (csrc/Makefile `asan`: -Xarch_host
-fsanitize=...; the gfx950 device code is unchanged; oracle/Makefile `asan`), then a child
pytest -- the clang ASan runtime preloaded, the sanitized libraries selected through
LGCNHS_LIB_PATH / ORACLE_LIB_PATH -- runs tests/test_native_abi.py's validation and export
checks and the oracle-vs-golden tests. Any sanitizer report aborts the child
(-fno-sanitize-recover=all, halt_on_error) and fails this test. No GPU is touched."""
import glob
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd")


def _asan_runtime():
    hits = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return hits[-1] if hits else None


@pytest.mark.timeout(900)
def test_abi_validation_and_oracle_under_asan_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not in this image")
    subprocess.run(["make", "-C", os.path.join(PKG, "csrc"), "-j8", "asan"], check=True,
                   capture_output=True)
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "asan"], check=True,
                   capture_output=True)
    env = dict(os.environ)
    env.update({
        "LD_PRELOAD": rt,
        # (leaks: the Python interpreter's own allocations are not ours to judge)
        "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0:exitcode=23",
        "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1",
        "LGCNHS_LIB_PATH": os.path.join(PKG, "lib", "asan", "liblgcnhs.so"),
        "ORACLE_LIB_PATH": os.path.join(REPO, "oracle", "build", "asan", "liboracle.so"),
        "ORACLE_THREADS": "4",
    })
    tests = ["tests/test_native_abi.py::test_argument_validation_without_gpu",
             "tests/test_native_abi.py::test_library_exports_every_symbol",
             "tests/test_oracle_golden.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        "-m", "not gpu", *tests], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=850)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert " passed" in out
