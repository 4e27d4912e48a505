"""CPU: the library's host C under AddressSanitizer + UndefinedBehaviorSanitizer.

csrc/codes.c (code tables, sampled codes, the OSG table image / packed table,
the threaded synthetic IF generator), csrc/sdr_host.c (GPS-SDR PRN spectra,
sine / twiddle / post-DFT tables, GN3S products) and csrc/osg_legacy.c (the
REG_read / REG_write register shim) are compiled with -fsanitize=address,
undefined (abort on the first report) together with tests/sanitize/
san_driver.c; the shim's four tracking-context calls go to a host stand-in
(tests/sanitize/track_stub.c).  GPU code is not sanitized (not available on
the MI355X pool, and host-only here).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gnss-sdr.ru_amd", "csrc")


def test_host_c_under_asan_ubsan(tmp_path):
    exe = tmp_path / "san"
    srcs = [os.path.join(ROOT, "tests", "sanitize", f) for f in ("san_driver.c", "track_stub.c")]
    srcs += [os.path.join(CSRC, f) for f in ("codes.c", "sdr_host.c", "osg_legacy.c", "common.c")]
    cmd = ["gcc", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
           *srcs, "-o", str(exe), "-lm", "-lpthread"]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + b.stderr[-2000:])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                UBSAN_OPTIONS="print_stacktrace=1"))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "sanitized host run OK" in r.stdout
