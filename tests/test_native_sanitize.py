"""Host sanitizers over the native runtime (SURVEY.md §5 "race detection / sanitizers"): the schedule
generator + validator and the threaded synthetic-data fill are compiled with AddressSanitizer +
UndefinedBehaviorSanitizer, and the threaded fill again with ThreadSanitizer, then run on the CPU
(tests/native/runtime_sanitize.cpp). GPU-side sanitizers are not available on the MI355X pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "simple_distributed_machine_learning_amd", "csrc", "runtime")
COMMON = os.path.join(ROOT, "simple_distributed_machine_learning_amd", "csrc", "common")
DRIVER = os.path.join(ROOT, "tests", "native", "runtime_sanitize.cpp")
CXX = shutil.which("g++")


def _build_and_run(tmp_path, name, flags):
    exe = str(tmp_path / name)
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-I{RT}", f"-I{COMMON}", DRIVER,
           os.path.join(RT, "schedule.cpp"), "-o", exe, "-pthread"] + flags
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if b.returncode != 0 and "cannot find" in b.stderr and "san" in b.stderr:
        pytest.skip(f"sanitizer runtime not installed: {b.stderr.strip()[:200]}")
    assert b.returncode == 0, b.stderr
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout, r.stdout
    return r.stdout


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_runtime_under_asan_ubsan(tmp_path):
    out = _build_and_run(tmp_path, "rt_asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])
    n = int(out.split("runtime sanitize:")[1].split("programs")[0])
    assert n > 1000


@pytest.mark.skipif(CXX is None, reason="no g++")
def test_threaded_synthetic_fill_under_tsan(tmp_path):
    _build_and_run(tmp_path, "rt_tsan", ["-fsanitize=thread", "-DSDML_SYNTH_ONLY"])
