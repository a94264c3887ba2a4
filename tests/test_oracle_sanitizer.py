"""The C restatement of the sampler (oracle/sampler_ref.c, the checker of every GPU sampling test)
under AddressSanitizer + UndefinedBehaviorSanitizer: odd and tiny vocabularies, bf16 and f32,
strided rows, greedy and every filter. Test infrastructure checking test infrastructure."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sampler_ref_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True, capture_output=True)
    exe = os.path.join(ROOT, "oracle", "_build", "sampler_ref_sanitize")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
