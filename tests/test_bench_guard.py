"""bench.py's watchdog for the sharded leg (CPU): a leg that hangs or raises
at N > 1 must not cost the bench line — give_up runs and ends the process
with a non-zero status; a timer firing as the leg returns
yields exactly one outcome."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = """
import os, sys, time
sys.path.insert(0, {root!r})
import bench
def give_up(why):
    print("GAVE UP:", why, flush=True)
    os._exit(bench.SHARDED_LEG_FAILED)
mode = sys.argv[1]
if mode == "hang":
    bench.guarded(lambda: time.sleep(30), 0.5, give_up, "leg")
elif mode == "raise":
    bench.guarded(lambda: 1 / 0, 30, give_up, "leg")
elif mode == "race":
    # the leg returns right as the watchdog fires: one line, never two
    print("RESULT:", bench.guarded(lambda: time.sleep(0.2) or 42, 0.2, give_up, "leg"), flush=True)
    time.sleep(0.5)   # a late timer would print here
else:
    print("RESULT:", bench.guarded(lambda: 42, 30, give_up, "leg"), flush=True)
"""


def run(mode):
    return subprocess.run([sys.executable, "-c", PROG.format(root=ROOT), mode], capture_output=True, text=True,
                          timeout=20)


def test_guard_hang_gives_up_quickly():
    r = run("hang")
    assert r.returncode == 3 and "GAVE UP: leg did not finish within 0 s" in r.stdout, r.stdout + r.stderr


def test_guard_exception_gives_up():
    r = run("raise")
    assert r.returncode == 3 and "GAVE UP: leg failed: ZeroDivisionError" in r.stdout, r.stdout + r.stderr


def test_guard_passes_result_through():
    r = run("ok")
    assert r.returncode == 0 and "RESULT: 42" in r.stdout, r.stdout + r.stderr


def test_guard_race_has_one_outcome():
    for _ in range(6):
        r = run("race")
        lines = [x for x in r.stdout.splitlines() if x.startswith(("RESULT", "GAVE UP"))]
        assert len(lines) == 1, r.stdout + r.stderr
        assert (r.returncode, lines[0][:6]) in ((0, "RESULT"), (3, "GAVE U")), r.stdout + r.stderr
