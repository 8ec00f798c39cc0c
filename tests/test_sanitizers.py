"""Host AddressSanitizer + UndefinedBehaviorSanitizer runs ("Host
ASan/UBSan on the CPU oracle"): the C oracle over the parity tests' edge
cases (empty / 1-point / 1025- and 2100-point rays, duplicate cells, cells
beyond the 1e9 sentinel, BoundsError inputs, every Julia-sum block
boundary) and the chain's host-side logic (chain_logic.h, the code both
chain engines run: Philox draws, det_log / det_exp, AS241 at the extremes of
the uniform, proposals at the cell bounds, all three priors' acceptance).
Built by `make -C oracle sanitize` (gcc / the ROCm clang++ for the host only)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], capture_output=True, text=True)
    if r.returncode != 0:
        if "fsanitize" in r.stderr or "asan" in r.stderr.lower():
            pytest.skip("no sanitizer runtime: " + r.stderr[-300:])
        raise AssertionError(r.stderr)
    return os.path.join(ORACLE, "_san")


@pytest.mark.parametrize("prog", ["san_oracle", "san_chain_logic"])
def test_clean_under_asan_ubsan(built, prog):
    env = dict(os.environ)
    # the container preloads a library of its own; ASan only needs to come first among ours
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0:detect_leaks=1:halt_on_error=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1"
    r = subprocess.run([os.path.join(built, prog)], capture_output=True, text=True, env=env, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-3000:]
    assert prog + ": ok" in r.stdout
