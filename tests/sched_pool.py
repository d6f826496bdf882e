"""Batched rank processes for the golden-schedule GPU tests — test
infrastructure.

Spawning P rank processes per test case (each importing torch) dominated the
GPU suite's time.  Every process-rank test case
registers its job at collection time; cases that need the same rank count P
and the same environment (the knobs are read per process) form ONE group,
run by ONE set of P tests/sched_worker.py processes on the first request, one
job after another with a fresh context each.  Each test then checks its own
job's outputs and modes, so every case keeps its own test id and verdict.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "sched_worker.py")

_groups = {}   # (P, env items) -> [job, ...]
_results = {}  # (P, env items) -> {job key: Result}


class Result:
    def __init__(self, outs=None, modes=None, err=None):
        self.outs = outs    # [rank] -> array [runs, n]
        self.modes = modes  # [rank] -> [mode dict per run]
        self.err = err


def _key(P, env):
    return (int(P), tuple(sorted(env.items())))


def _job_key(job):
    return (job["case"], job["runs"])


def register(case, env, runs):
    """Declare a job (at collection time, from a test's parameter list)."""
    P = int(case.split("/")[3][1:])
    jobs = _groups.setdefault(_key(P, env), [])
    job = {"case": case, "runs": int(runs)}
    if all(_job_key(j) != _job_key(job) for j in jobs):
        jobs.append(job)


def result(case, env, runs):
    """The job's Result (running its whole group the first time)."""
    P = int(case.split("/")[3][1:])
    key = _key(P, env)
    register(case, env, runs)
    if key not in _results or (case, int(runs)) not in _results[key]:
        _results.setdefault(key, {}).update(_run_group(P, dict(env), _groups[key]))
    return _results[key][(case, int(runs))]


def _run_group(P, env, jobs):
    out = {}
    with tempfile.TemporaryDirectory() as d:
        jf = os.path.join(d, "jobs.json")
        with open(jf, "w") as f:
            json.dump(jobs, f)
        e = dict(os.environ, **env)
        logs = [open(os.path.join(d, f"log{r}.txt"), "w") for r in range(P)]
        procs = [subprocess.Popen([sys.executable, WORKER, str(r), str(P), d, jf], env=e, stdout=logs[r],
                                  stderr=subprocess.STDOUT) for r in range(P)]
        deadline = 120 + 40 * len(jobs)
        rcs = []
        try:
            for p in procs:
                rcs.append(p.wait(timeout=deadline))
        except subprocess.TimeoutExpired:
            for p in procs:
                p.kill()
            for p in procs:
                p.wait()
            rcs = [p.returncode for p in procs]
        for f in logs:
            f.close()
        tails = {r: open(os.path.join(d, f"log{r}.txt")).read()[-2000:] for r in range(P)}
        for j, job in enumerate(jobs):
            errs = []
            for r in range(P):
                ef = os.path.join(d, f"e{r}_{j}.txt")
                if os.path.exists(ef):
                    errs.append(f"rank {r}: " + open(ef).read()[-1500:])
                elif not os.path.exists(os.path.join(d, f"o{r}_{j}.npy")):
                    errs.append(f"rank {r}: no output (worker exit {rcs[r]}): {tails[r]}")
            if errs:
                out[_job_key(job)] = Result(err="\n".join(errs))
                continue
            outs = [np.load(os.path.join(d, f"o{r}_{j}.npy")) for r in range(P)]
            modes = [json.load(open(os.path.join(d, f"m{r}_{j}.json"))) for r in range(P)]
            out[_job_key(job)] = Result(outs=outs, modes=modes)
    return out
