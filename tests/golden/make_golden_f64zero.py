#!/usr/bin/env python3
"""Golden fixtures for f64 keys that mix -0.0 and +0.0 (and tiny +-1e-300),
from the compiled, UNMODIFIED reference (oracle/_ref/psort_ref, see
make_golden.py): its parallel_bitonic_sort (psort.cc:167-201) on the same
4002 doubles at P = 1, 2, 4, 8.

    make -C oracle all && python tests/golden/make_golden_f64zero.py

-0.0 == +0.0 as doubles, so std::sort (psort.cc:175) and the keep-min/max
merges (psort.cc:116-164) leave the two zeros in an implementation-defined
order; the fixtures record what the reference actually writes, so the GPU test
can pin every position whose value is not zero bit for bit, every position by
value, and measure (not assume) where the zero signs differ.

Writes tests/golden/f64zero.in (raw LE doubles), f64zero_P{p}.out and
f64zero.json (sizes, error counts, SHA-256, the sign pattern statistics).
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
import oracle_lib as O  # noqa: E402


def keys():
    rng = np.random.default_rng(3)
    x = np.concatenate([np.zeros(500), -np.zeros(500), rng.standard_normal(3000), [1e-300, -1e-300]])
    rng.shuffle(x)
    return x


def main():
    x = keys()
    x.tofile(os.path.join(HERE, "f64zero.in"))
    cases = []
    for p in (1, 2, 4, 8):
        with tempfile.TemporaryDirectory() as d:
            x.tofile(f"{d}/k")
            r = subprocess.run([O.MPIRUN, "-np", str(p), O.REF_BIN, "--dtype", "f64", "--keys", f"{d}/k",
                                "--out", f"{d}/o"], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                raise RuntimeError(r.stderr)
            y = np.fromfile(f"{d}/o")
        y.tofile(os.path.join(HERE, f"f64zero_P{p}.out"))
        errors = int([l for l in r.stdout.splitlines() if "errors in sorting" in l][0].split()[0])
        info = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
        z = np.signbit(y[y == 0])
        cases.append({"p": p, "n": int(x.size), "sizes": info["sizes"], "errors": errors,
                      "out_sha256": hashlib.sha256(y.tobytes()).hexdigest(),
                      "zeros": int(z.size), "negative_zeros": int(z.sum()),
                      "zero_sign_changes": int(np.count_nonzero(np.diff(z.astype(np.int8))))})
        print(cases[-1], flush=True)
    with open(os.path.join(HERE, "f64zero.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_f64zero.py",
                   "reference": "Parallel-Sorting/src/psort.cc (unmodified) parallel_bitonic_sort via oracle/_ref",
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
