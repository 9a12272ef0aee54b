#!/usr/bin/env python3
"""Generate tests/golden/ fixtures from the compiled, UNMODIFIED reference.

Run in the build container (needs /root/reference and MPICH at /opt/conda):

    make -C oracle all && python tests/golden/make_golden.py

Two kinds of case, both produced by oracle/_ref/psort_ref (see
oracle/ref_harness.cc for how it drives psort.cc without modifying it):

* "psort": `mpirun -np P psort_ref N` = the reference main() with its sort call
  routed to parallel_bitonic_sort (psort.cc:167) -- generator, block layout,
  stdout lines and check_sort exactly as shipped.  Per-rank blocks are dumped
  before and after the sort.
* "keys": the reference's parallel_bitonic_sort on a given key set (u32
  SplitMix64 keys, and u64 duplicate-heavy/skewed keys carried as
  order-preserving doubles).
* algo "quick": the same two kinds with the reference's OWN parallel_quick_sort
  (psort.cc:377, the binary as shipped); per-rank output sizes are
  data-dependent and recorded.

Stored: a JSON manifest (sizes, error counts, stdout, SHA-256 of inputs and of
the rank-ordered outputs, head/tail keys) plus raw little-endian arrays for the
small cases.  Fixtures are data only; no reference source is stored.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402  (only for the SplitMix64 inputs)

REF = O.REF_BIN
PS = [1, 2, 4, 8]
PSORT_NS = [13, 100, 1024, 1031, 65537, 1000003, 1000005]
FULL_LIMIT = 1031  # keep whole arrays for N <= this


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def hexkeys(a):
    return [format(int(x), "016x") for x in np.ascontiguousarray(a).view(np.uint64)]


def run(cmd, env=None):
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd}: {r.returncode}\n{r.stdout}\n{r.stderr}")
    return r.stdout


def psort_case(n, p, algo="bitonic"):
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, PSORT_DUMP_DIR=d, PSORT_ALGO=algo)
        out = run([O.MPIRUN, "-np", str(p), REF, str(n)], env=env)
        ins = [np.fromfile(f"{d}/in_{r}_of_{p}.f64") for r in range(p)]
        outs = [np.fromfile(f"{d}/out_{r}_of_{p}.f64") for r in range(p)]
    lines = out.strip().splitlines()
    errors = int(lines[-1].split()[0])
    stable = [l for l in lines if "required" not in l and "sort time" not in l]
    x, y = np.concatenate(ins), np.concatenate(outs)
    case = {
        "mode": "psort", "algo": algo, "n": n, "p": p,
        "sizes": [int(b.size) for b in outs],
        "errors": errors, "stdout_stable": stable,
        "in_sha256": sha(x), "out_sha256": sha(y),
        "in_head": hexkeys(x[:8]), "out_head": hexkeys(y[:8]), "out_tail": hexkeys(y[-8:]),
    }
    if n <= FULL_LIMIT:
        x.tofile(os.path.join(HERE, f"psort_in_N{n}.f64"))
        tag = "" if algo == "bitonic" else algo + "_"
        y.tofile(os.path.join(HERE, f"psort_{tag}out_N{n}_P{p}.f64"))
    return case


def keys_case(name, keys, p, dtype, store_full, algo="bitonic"):
    with tempfile.TemporaryDirectory() as d:
        kf, of = f"{d}/keys.bin", f"{d}/out.bin"
        keys.tofile(kf)
        out = run([O.MPIRUN, "-np", str(p), REF, "--dtype", dtype, "--keys", kf, "--out", of,
                   "--algo", algo])
        y = np.fromfile(of, dtype=keys.dtype)
    errors = int([l for l in out.splitlines() if "errors in sorting" in l][0].split()[0])
    info = json.loads([l for l in out.splitlines() if l.startswith("{")][0])
    case = {
        "mode": "keys", "algo": algo, "name": name, "dtype": dtype, "n": int(keys.size), "p": p,
        "errors": errors, "sizes": info["sizes"], "in_sha256": sha(keys), "out_sha256": sha(y),
    }
    if store_full:
        tag = "" if algo == "bitonic" else algo + "_"
        y.tofile(os.path.join(HERE, f"keys_{tag}{name}_P{p}.out"))
    return case


def mixed_u64(n, seed):
    """Config-5 style mix, restricted to keys the reference can carry as
    ordered doubles (<= 0x7FF0000000000000): duplicate-heavy alphabet, skewed
    ODD_DIST bit patterns, uniform, zeros and the largest carried key."""
    rng = np.random.default_rng(seed)
    top = np.uint64(0x7FF0000000000000)
    n_alpha, n_skew, n_uni, n_zero = int(n * .4), int(n * .3), int(n * .2), int(n * .05)
    alpha = rng.integers(0, int(top), size=1024, dtype=np.uint64)
    parts = [alpha[rng.integers(0, 1024, size=n_alpha)],
             O.generate_f64(n_skew).view(np.uint64),
             rng.integers(0, int(top), size=n_uni, dtype=np.uint64),
             np.zeros(n_zero, dtype=np.uint64)]
    rest = n - sum(x.size for x in parts)
    parts.append(np.full(rest, top, dtype=np.uint64))
    keys = np.concatenate(parts)
    rng.shuffle(keys)
    return keys


def main():
    if not os.path.exists(REF):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    cases = []
    for n in PSORT_NS:
        for p in PS:
            c = psort_case(n, p)
            print(f"psort N={n} P={p} errors={c['errors']}", flush=True)
            cases.append(c)
    for n in [1000, 4099, 65541, 1000007]:
        keys = O.splitmix(0x5EED0001, n, np.uint32)
        for p in PS:
            c = keys_case(f"u32_n{n}", keys, p, "u32", store_full=n <= 4099)
            print(f"keys u32 N={n} P={p} errors={c['errors']}", flush=True)
            cases.append(c)
    for n in [5003, 20011]:
        keys = mixed_u64(n, 0x5EED0005 + n)
        keys.tofile(os.path.join(HERE, f"keys_u64mix_n{n}.in"))
        for p in PS:
            c = keys_case(f"u64mix_n{n}", keys, p, "u64", store_full=True)
            print(f"keys u64 N={n} P={p} errors={c['errors']}", flush=True)
            cases.append(c)
    # the shipped sort: parallel_quick_sort
    for n in [13, 100, 1024, 1031, 65537, 1000003]:
        for p in PS:
            c = psort_case(n, p, "quick")
            print(f"psort quick N={n} P={p} sizes={c['sizes']} errors={c['errors']}", flush=True)
            cases.append(c)
    for n in [1000, 4099, 65541]:
        keys = O.splitmix(0x5EED0001, n, np.uint32)
        for p in PS:
            c = keys_case(f"u32_n{n}", keys, p, "u32", store_full=n <= 4099, algo="quick")
            print(f"keys quick u32 N={n} P={p} sizes={c['sizes']}", flush=True)
            cases.append(c)
    for n in [5003, 20011]:
        keys = mixed_u64(n, 0x5EED0005 + n)
        for p in PS:
            c = keys_case(f"u64mix_n{n}", keys, p, "u64", store_full=True, algo="quick")
            print(f"keys quick u64 N={n} P={p} sizes={c['sizes']}", flush=True)
            cases.append(c)
    meta = {
        "generator": "tests/golden/make_golden.py",
        "reference": "Parallel-Sorting/src/psort.cc (unmodified; parallel_bitonic_sort and "
                     "parallel_quick_sort via oracle/_ref)",
        "mpi": "MPICH 3.3.2 (/opt/conda), g++ 11, -g -O1",
        "cases": cases,
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(cases)} cases written")


if __name__ == "__main__":
    main()
