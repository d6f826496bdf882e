"""CPU: bench.py's N>1 watchdog fires on a hang (no progress line for the
idle limit) or past the section's total limit, and not while progress lines
keep coming (a hung section must end the job non-zero, a slow
one must not)."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _run(idle, total, beat_for, beat_every=0.05):
    fired = []
    done = threading.Event()

    def fire(reason):
        fired.append((time.time(), reason))
        done.set()
    t0 = time.time()
    wd = bench.Watchdog(idle, total, fire)
    while time.time() - t0 < beat_for:
        bench.progress("beat")
        time.sleep(beat_every)
    done.wait(5)
    wd.cancel()
    return t0, fired


def test_fires_when_progress_stops():
    t0, fired = _run(0.4, 60, beat_for=1.0)
    assert fired and "no progress" in fired[0][1]
    assert fired[0][0] - t0 >= 1.0  # not while the beats came


def test_fires_past_total_limit_despite_progress():
    t0, fired = _run(5, 0.8, beat_for=1.5)
    assert fired and "exceeded" in fired[0][1]


def test_cancel_stops_it():
    fired = []
    wd = bench.Watchdog(0.2, 60, lambda r: fired.append(r))
    wd.cancel()
    time.sleep(0.5)
    assert not fired


def test_watchdog_line_survives_concurrent_updates():
    """The line is built on the watchdog thread while the main thread keeps
    adding results: every attempt yields parseable JSON with the error set
    (the race a bare dict(partial) lost once)."""
    import json
    partial = {"variants": {}}
    stop = threading.Event()

    def writer():
        i = 0
        while not stop.is_set():
            partial["variants"]["v%d" % (i % 500)] = {"ms_p50": i, "samples": list(range(i % 50))}
            partial["k%d" % (i % 300)] = i
            i += 1
    t = threading.Thread(target=writer)
    t.start()
    try:
        for _ in range(200):
            line = json.loads(bench.watchdog_line({"metric": "m", "value": 1.0}, partial, "no progress",
                                                  lambda x: {"value": None}))
            assert line["value"] == 1.0 and "watchdog" in line["xgmi_allreduce"]["error"]
    finally:
        stop.set()
        t.join()


def test_watchdog_line_falls_back_when_unreadable():
    import json

    # a snapshot that can never be serialised (a set is not JSON)
    line = json.loads(bench.watchdog_line({"metric": "m", "value": 2.0, "per_gpu_efficiency": {}},
                                          {"a": {1, 2}}, "stuck", lambda x: {}, tries=2))
    assert line["value"] == 2.0 and "unreadable" in line["xgmi_allreduce"]["error"]
    assert "per_gpu_efficiency" not in line
