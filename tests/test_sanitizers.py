"""Host sanitizers over the native CPU code.

The dataset index builders (``csrc/data_helpers.cpp``, reference
``megatron/data/helpers.cpp``) and the MinHash/LSH de-duplication kernels
(``csrc/dedup.cpp``, with its std::thread pool) are rebuilt as embedded
modules of a sanitizer-instrumented executable (``csrc/sanitize_main.cpp``)
and driven through every entry point by ``scripts/sanitize_driver.py``:

* ASan + UBSan (``-fno-sanitize-recover``): any heap overflow, use after free
  or undefined behaviour aborts the run;
* TSan: the MinHash worker pool must be race-free.

The sanitized results must equal the normal in-tree extensions' results.
GPU kernels are not covered: GPU ASan/XNACK is not available on this pool.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "scripts", "sanitize_driver.py")


@pytest.fixture(scope="module")
def reference(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("ref") / "ref.npz")
    r = subprocess.run([sys.executable, DRIVER, out, "package"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, PYTHONPATH=ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    return dict(np.load(out))


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_native_helpers_under_sanitizer(kind, reference, tmp_path):
    from epfl_megatron_amd.build import build_sanitized
    exe = build_sanitized(kind, str(tmp_path))
    out = str(tmp_path / "san.npz")
    env = dict(os.environ, PYTHONPATH=ROOT,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:report_signal_unsafe=0")
    r = subprocess.run([exe, DRIVER, out, "embedded"], cwd=ROOT, capture_output=True, text=True,
                       timeout=600, env=env)
    report = r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, report
    got = dict(np.load(out))
    assert got.keys() == reference.keys()
    for k in reference:
        np.testing.assert_array_equal(got[k], reference[k], err_msg=k)
