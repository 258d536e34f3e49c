"""Race / memory checking of the native runtime cores (SURVEY §5 "race detection").

The reference runs its C++ unit tests under TSAN / ASAN builds (bazel `--config=tsan` /
`--config=asan`, reference `.bazelrc` and `ci/ci.sh`), which covers plasma and the raylet
scheduler. Here the same two native cores are built from source with the host sanitizers and
driven by dedicated stress programs:

* ``csrc/tests/store_stress.cc`` — 6 threads on ONE shared-memory store mapping doing
  create/seal/get/release/delete, batched wait, sealed-notification polling and explicit
  spilling, with restore-on-get under memory pressure; built with ThreadSanitizer and with
  AddressSanitizer + UBSan. Payload bytes are verified on every get; the heap self-check and
  zero-bytes-in-use are asserted at the end.
* ``csrc/tests/sched_fuzz.cc`` — randomised submit / object-ready / dispatch / release / cancel
  and placement-group create / place / remove sequences against the scheduler core with
  resource-conservation invariants; built with AddressSanitizer + UBSan.

Host code only (no GPU code is instrumented). Skipped when the compiler lacks the runtime.
"""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
CXX = shutil.which("g++")

pytestmark = pytest.mark.skipif(CXX is None, reason="g++ not available")


def _build(tmp_path, name, srcs, san):
    out = str(tmp_path / name)
    cmd = [CXX, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", f"-fsanitize={san}",
           f"-I{CSRC}", *[os.path.join(CSRC, s) for s in srcs], "-o", out, "-lpthread", "-lrt"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        if "cannot find" in r.stderr and "san" in r.stderr:
            pytest.skip(f"{san} runtime not installed")
        raise AssertionError(r.stderr[-4000:])
    return out


def _run(cmd, env_extra):
    env = dict(os.environ, **env_extra)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    report = r.stdout + r.stderr
    return r.returncode, report


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_object_store_concurrent_lifecycle(tmp_path, san):
    exe = _build(tmp_path, "store_stress", ["tests/store_stress.cc", "store/shm_store.cc"], san)
    spill = tmp_path / "spill"
    spill.mkdir()
    rc, report = _run([exe, str(spill), "6", "3000"],
                      {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1",
                       "ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                       "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
    assert "WARNING: ThreadSanitizer" not in report, report[-6000:]
    assert "ERROR: AddressSanitizer" not in report, report[-6000:]
    assert "runtime error:" not in report, report[-6000:]
    assert rc == 0 and "STRESS OK" in report, report[-6000:]
    # the run really exercised spill + restore under contention
    line = next(ln for ln in report.splitlines() if ln.startswith("spilled="))
    stats = dict(kv.split("=") for kv in line.split())
    assert int(stats["spilled"]) > 0 and int(stats["restored"]) > 0, report
    # clients SIGKILLed holding the store mutex mid-update (4 crash points): recovered every time
    crash = next(ln for ln in report.splitlines() if ln.startswith("crash phase:"))
    cs = dict(kv.split("=") for kv in crash.split(":", 1)[1].split())
    assert int(cs["recoveries"]) >= 4 and int(cs["bad"]) == 0, crash


def test_scheduler_fuzz_resource_conservation(tmp_path):
    exe = _build(tmp_path, "sched_fuzz", ["tests/sched_fuzz.cc", "sched/scheduler.cc"], "address,undefined")
    for seed in (1, 2, 3):
        rc, report = _run([exe, "8000", str(seed)],
                          {"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=1",
                           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"})
        assert "ERROR: AddressSanitizer" not in report, report[-6000:]
        assert "runtime error:" not in report, report[-6000:]
        assert rc == 0 and "FUZZ OK" in report, (seed, report[-6000:])
