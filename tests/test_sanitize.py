"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the CPU
restatement (oracle/arima_oracle.c) and the fit kernel's optimizer state machine on the CPU (cg_lane.hpp via
tests/sim/cglane_sim.cpp) fit a spread of orders, lengths (T = 0..16, 40, 300) and edge inputs (NaN, constant,
1e150-scaled) in one ASan/UBSan executable (tests/sanitize/). Any sanitizer report aborts the run; the driver also
requires the state machine to reproduce the restatement's fits bit for bit. CPU only (no GPU sanitizers here)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")


def test_oracle_and_state_machine_are_sanitizer_clean():
    subprocess.check_call(["make", "-s", "-C", SAN])
    # verify_asan_link_order=0: the ASan runtime is linked statically, whatever else the environment preloads
    env = dict(os.environ, ASAN_OPTIONS="verify_asan_link_order=0:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(SAN, "_build", "san_driver")], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-6000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert " 0 mismatches" in r.stdout, r.stdout
