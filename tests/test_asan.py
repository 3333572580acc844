"""Host sanitizer build: the HIP-free host C of the
product (picture_enc.c, picture_tools.c, vp8_host.c, vp8l_host.c), the
oracle and the own decoder built with -fsanitize=address,undefined
(`make -C libwebp_amd/csrc asan`) and driven over random inputs by
tests/asan/host_check.c; any sanitizer report fails the test."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_code_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "asan"], cwd=os.path.join(ROOT, "libwebp_amd", "csrc"))
    # the environment is passed through unchanged apart from the sanitizer
    # options (a preloaded library ahead of the ASan runtime is tolerated)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "build", "asan", "host_check")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_check: ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
