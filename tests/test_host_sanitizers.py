"""Host code of the native runtime under the sanitizers (SURVEY.md §5.2 race detection /
sanitizers).  GPU AddressSanitizer and xnack+ code objects are not available on the MI355X
pool, so the sanitizers cover the host side: CRC32C (checkpoint / event formats) and the
multi-threaded row gather of the data loader under ASan + UBSan and under ThreadSanitizer,
and the launch-shape validation of the conv kernels (host code of conv_fwd.hip, built by
hipcc with ``-Xarch_host -fsanitize=...``) swept over valid and invalid shapes."""
import hashlib
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "unet_distributed_amd", "csrc")
SRC = [os.path.join(CSRC, "tests", "host_checks.cpp"), os.path.join(CSRC, "runtime", "host_io.cpp")]
OUT = os.path.join(ROOT, "build", "host_checks")


def _build_and_run(name, cmd_prefix, extra_src=(), flags=()):
    srcs = list(SRC) + list(extra_src)
    h = hashlib.sha256(" ".join(cmd_prefix + list(flags)).encode())
    for f in srcs + [os.path.join(CSRC, "kernels", n) for n in sorted(os.listdir(os.path.join(CSRC, "kernels")))]:
        h.update(open(f, "rb").read())
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, "%s-%s" % (name, h.hexdigest()[:16]))
    if not os.path.exists(exe):
        r = subprocess.run(cmd_prefix + list(flags) + srcs + ["-o", exe + ".tmp"], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        os.replace(exe + ".tmp", exe)
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host checks passed" in r.stdout


GXX = shutil.which("g++")


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_host_runtime_asan_ubsan():
    _build_and_run("asan", [GXX, "-std=c++17", "-O1", "-g", "-msse4.2", "-pthread",
                            "-fsanitize=address,undefined", "-fno-sanitize-recover=all"])


@pytest.mark.skipif(GXX is None, reason="g++ not available")
def test_host_runtime_tsan():
    _build_and_run("tsan", [GXX, "-std=c++17", "-O1", "-g", "-msse4.2", "-pthread", "-fsanitize=thread"])


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_conv_shape_validation_asan_ubsan():
    """~1.5 minutes on the first run (hipcc also compiles the gfx950 device code, which this
    host-side check never launches: unoptimised and without debug info -- at -O1 -g it took
    ~8 minutes); cached."""
    _build_and_run("shapes", ["/opt/rocm/bin/hipcc", "-std=c++17", "-O1", "-g", "--offload-arch=gfx950",
                              "-Xarch_device", "-g0", "-Xarch_device", "-O0",
                              "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                              "-DUNET_WITH_SHAPE_CHECKS", "-msse4.2", "-pthread",
                              "-I" + os.path.join(CSRC, "runtime"), "-I" + os.path.join(CSRC, "kernels")],
                   extra_src=[os.path.join(CSRC, "kernels", "conv_fwd.hip"),
                              os.path.join(CSRC, "tests", "win_stubs.cpp")])
