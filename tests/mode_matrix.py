"""The execution-mode matrix of the plan executor — TEST
INFRASTRUCTURE.

After round 6 the executor has ONE plan-selecting knob (GLOO_AMD_MESH) and
the launch-mode selectors (GLOO_AMD_GRAPH, GLOO_AMD_INTERP,
GLOO_AMD_INTERP_SLICE_BYTES, GLOO_AMD_FUSE_BYTES, GLOO_AMD_INTERP_MAX_SLICES:
each picks a mode the library also picks by itself by message size, so the
small golden fixtures can reach every mode).  Everything else is fixed or
follows the rank layout.  The axes a run's behaviour depends on:

  route       mesh (derived mesh plan) | reference (the reference's exchange)
  signal      device (stream-ordered signal / wait kernels; any rank layout
              but ranks of one process sharing a GPU) | host (host waits:
              ranks of one process sharing a GPU)
  launch      interp (one-workgroup interpreter) | sliced (interpreter, one
              workgroup per slice) | graph (hipGraph replay) | eager
  completion  own (the algorithm's own stream; run() returns on the
              device-published done word) | caller (a stream the caller
              passes; run() returns without waiting)
  arena       device (fine-grained HBM inboxes) | host (pinned host inboxes,
              the HOST workspace)

Structural exclusions (executor.cc): host signalling has no interpreter and
no graph (both need device-side waits), so it is eager only; a HOST-workspace
arena is never sliced (proposeSlices).  Every other combination is a cell,
and tests/test_mode_matrix_gpu.py runs each cell once on a golden case of the
reference, asserting the mode the executor reports.
"""
import itertools

ROUTES = ("mesh", "reference")
SIGNALS = ("device", "host")
LAUNCHES = ("interp", "sliced", "graph", "eager")
COMPLETIONS = ("own", "caller")
ARENAS = ("device", "host")

# one golden case per route (tests/golden/sched_golden.npz), chosen so that
# every launch mode is reachable: the mesh ring-chunked plan at P = 3 slices
# at 1 KiB per slice, the reference HD route only at P = 2 (its exchange is
# sliceable there, plan_sim.sliceable)
CASES = {"mesh": ("ring_chunked/sum/f32/P3/k1/n10007", "1024"),
         "reference": ("halving_doubling/sum/f32/P2/k1/n1000", "256")}


def possible(route, signal, launch, completion, arena):
    if signal == "host" and launch != "eager":
        return False
    if arena == "host" and launch == "sliced":
        return False
    return True


def cells():
    out = []
    for c in itertools.product(ROUTES, SIGNALS, LAUNCHES, COMPLETIONS, ARENAS):
        if possible(*c):
            out.append(dict(zip(("route", "signal", "launch", "completion", "arena"), c)))
    return out


def cell_id(c):
    return "-".join(c[k] for k in ("route", "signal", "launch", "completion", "arena"))


def env_of(c):
    """The environment that selects the cell's route and launch mode."""
    case, slice_bytes = CASES[c["route"]]
    e = {"GLOO_AMD_MESH": "1" if c["route"] == "mesh" else "0"}
    if c["launch"] == "sliced":
        e["GLOO_AMD_INTERP_SLICE_BYTES"] = slice_bytes
    elif c["launch"] == "graph":
        e.update(GLOO_AMD_INTERP="0", GLOO_AMD_GRAPH="1")
    elif c["launch"] == "eager":
        e.update(GLOO_AMD_INTERP="0", GLOO_AMD_GRAPH="0")
    return e


def check_mode(c, modes):
    """`modes`: a rank's mode() after each of its runs.  The executor must
    report the cell it was asked for."""
    last = modes[-1]
    assert last["device_signal"] == (c["signal"] == "device"), (c, last)
    assert last["host_arena"] == (c["arena"] == "host"), (c, last)
    if c["arena"] == "device":
        assert last["fine_arena"], (c, last)
    assert last["own_stream"] == (c["completion"] == "own"), (c, last)
    if c["launch"] == "interp":
        assert all(m["interp"] and m["interp_slices"] == 1 for m in modes), (c, modes)
    elif c["launch"] == "sliced":
        assert all(m["interp"] and m["interp_slices"] > 1 for m in modes), (c, modes)
    elif c["launch"] == "graph":
        assert not modes[0]["graph"] and all(m["graph"] for m in modes[1:]), (c, modes)
    else:
        assert not any(m["graph"] or m["interp"] for m in modes), (c, modes)
