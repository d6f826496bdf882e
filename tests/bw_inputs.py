"""Deterministic inputs for the bandwidth-regime parity cases (TEST
INFRASTRUCTURE).

The reference's own outputs at BASELINE sizes (config 3: 256 MiB per rank,
config 4 / 5 at bandwidth sizes) are too large to commit, so
tests/golden/bw_golden.json keeps, per case, the seed these inputs are drawn
from, a SHA-256 digest of every rank's reference output and a few sampled
values.  oracle/gen_golden.py (`bw`) draws the inputs here, runs the reference
(oracle/_ref) on them and records the digests; the GPU tests draw the SAME
inputs on the box (numpy's PCG64 stream is platform-independent) and compare
the HIP executor's output digests.
"""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "bw_golden.json")


def f32_to_bf16(f):
    """Round-to-nearest-even float32 -> bfloat16 bits (c10::BFloat16 for
    finite values; the inputs here are finite)."""
    u = np.ascontiguousarray(f, dtype=np.float32).view(np.uint32)
    return ((u + (((u >> 16) & 1) + 0x7FFF)) >> 16).astype(np.uint16)


def make_input(dtype, op, n, seed, rank):
    """Rank `rank`'s input of a case: N(0, 1) values (U(0.5, 2) for PRODUCT,
    so products of 8 ranks stay finite), stored as `dtype` (16-bit floats as
    raw bits, round to nearest even)."""
    rng = np.random.default_rng([seed, rank])
    if op == "product":
        f = rng.random(n, dtype=np.float32) * np.float32(1.5) + np.float32(0.5)
    else:
        f = rng.standard_normal(n, dtype=np.float32)
    if dtype == "f32":
        return f
    if dtype == "f16":
        return f.astype(np.float16).view(np.uint16)
    if dtype == "bf16":
        return f32_to_bf16(f)
    raise ValueError(dtype)


def even_recv(P, n):
    """recvElems as gloo/test/reduce_scatter_test.cc:86-92 builds them."""
    out, rem, chunk = [], n, (n + P - 1) // P
    for _ in range(P):
        out.append(min(chunk, rem))
        rem = rem - chunk if rem > chunk else 0
    return out


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).view(np.uint8).tobytes()).hexdigest()


def sample_index(n, k=64, seed=99):
    """Fixed sample positions (for a readable diff when a digest differs)."""
    rng = np.random.default_rng(seed)
    return np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, k)])).astype(np.int64)


def load():
    with open(GOLDEN) as f:
        return json.load(f)
