#!/usr/bin/env python3
"""Golden fixtures for the BASELINE-sized configs (tests/golden/large.json).

Run in the build container (needs /root/reference built into oracle/_ref and
MPICH at /opt/conda; ~30 GiB of RAM, ~10 minutes):

    make -C oracle all && python tests/golden/make_golden_large.py

Configs (BASELINE.json / SURVEY.md 8(d)):
* 3 / 4: 2^28 u32 (SplitMix64 seed 0x5EED0002) and 2^30 u32 (seed 0x5EED0003).
  N % P == 0 at P = 1, 2, 4, 8, so the reference's parallel_bitonic_sort output
  is the globally sorted sequence at every P: one SHA-256 per size,
  from the oracle's sort, PINNED by running the compiled reference itself
  (`mpirun -np P psort_ref --dtype u32 --gen-splitmix SEED --n N --out F`) at
  P = 8 for both sizes and P = 2, 4 at 2^28, whose outputs must hash the same.
* 5: u64, N = 2^29 - 3 (N % 8 = 5: the reference's defective uneven-block
  output) and N = 2^29 - 7 (N % 8 = 1), P = 8, the orc_u64mix mix (seed
  0x5EED0005).  Two variants each:
    - "ref":  sentinel 0x7FF0000000000000, every key carried by the reference
      as an ordered double -> the compiled reference's output SHA and error
      count, cross-checked against the oracle's P-rank restatement;
    - "full": all-ones sentinel (NaN as a double: the reference cannot carry
      it) -> the oracle's P-rank restatement (oracle.c, itself pinned by the
      "ref" variant and tests/golden/golden.json).
Only hashes, sizes and error counts are stored (data, no reference source).
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402

MIX_SEED = 0x5EED0005
TMP = os.environ.get("GOLDEN_TMP", "/tmp")


def sha_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 26), b""):
            h.update(blk)
    return h.hexdigest()


def sha(a):
    h = hashlib.sha256()
    v = np.ascontiguousarray(a).view(np.uint8)
    for i in range(0, v.size, 1 << 28):
        h.update(v[i:i + (1 << 28)])
    return h.hexdigest()


def mix(n, top, threads=8):
    """orc_u64mix over threads (ctypes releases the GIL)."""
    out = np.empty(n, dtype=np.uint64)
    step = (n + threads - 1) // threads

    def part(t):
        g0 = t * step
        cnt = max(0, min(n, g0 + step) - g0)
        if cnt:
            out[g0:g0 + cnt] = O.u64mix(MIX_SEED, n, top, g0, cnt)
    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(part, range(threads)))
    return out


def run_ref(args, timeout=3600):
    r = subprocess.run([O.MPIRUN, *args], capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"{args}: rc {r.returncode}\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    errors = int([l for l in r.stdout.splitlines() if "errors in sorting" in l][0].split()[0])
    info = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    return errors, info


def u32_case(logn, seed, ref_ps):
    n = 1 << logn
    t = time.time()
    x = O.splitmix(seed, n, np.uint32)
    in_sha = sha(x)
    y = O.local_sort(x)
    del x
    out_sha = sha(y)
    head, tail = [int(v) for v in y[:4]], [int(v) for v in y[-4:]]
    del y
    print(f"u32 2^{logn}: oracle sorted sha {out_sha[:16]} ({time.time() - t:.0f}s)", flush=True)
    refs = []
    for p in ref_ps:
        with tempfile.TemporaryDirectory(dir=TMP) as d:
            of = os.path.join(d, "out.bin")
            t = time.time()
            errors, info = run_ref(["-np", str(p), O.REF_BIN, "--dtype", "u32", "--gen-splitmix", hex(seed),
                                    "--n", str(n), "--out", of])
            rsha = sha_file(of)
        print(f"  reference P={p}: sha {rsha[:16]} errors {errors} sort {info['sort_s']:.1f}s "
              f"({time.time() - t:.0f}s)", flush=True)
        if rsha != out_sha or errors != 0:
            raise SystemExit(f"reference P={p} differs from the oracle at 2^{logn}")
        refs.append({"p": p, "out_sha256": rsha, "errors": errors, "sort_s": info["sort_s"]})
    return {"config": 3 if logn == 28 else 4, "dtype": "u32", "n": n, "seed": seed,
            "generator": "splitmix top 32 bits (orc_splitmix_u32 / misort_fill_splitmix)",
            "in_sha256": in_sha, "out_sha256": out_sha, "errors": 0, "ps": [1, 2, 4, 8],
            "out_head": head, "out_tail": tail,
            "pinned_by_reference": refs}


def u64_case(n, variant, p=8):
    top = O.REF_TOP if variant == "ref" else O.ALL_ONES
    t = time.time()
    x = mix(n, top)
    in_sha = sha(x)
    y = O.parallel_bitonic_sort(x, p)
    out_sha, errors = sha(y), O.check_sort(y, p)
    sizes = [int(s) for s in O.block_sizes(n, p)]
    print(f"u64mix {variant} N={n} P={p}: oracle sha {out_sha[:16]} errors {errors} "
          f"({time.time() - t:.0f}s)", flush=True)
    del y
    case = {"config": 5, "dtype": "u64", "variant": variant, "n": n, "p": p, "seed": MIX_SEED,
            "top": hex(top), "generator": "orc_u64mix", "sizes": sizes,
            "in_sha256": in_sha, "out_sha256": out_sha, "errors": errors}
    if variant == "ref":
        with tempfile.TemporaryDirectory(dir=TMP) as d:
            kf, of = os.path.join(d, "keys.bin"), os.path.join(d, "out.bin")
            x.tofile(kf)
            del x
            t = time.time()
            rerr, info = run_ref(["-np", str(p), O.REF_BIN, "--dtype", "u64", "--keys", kf, "--out", of])
            rsha = sha_file(of)
        print(f"  reference P={p}: sha {rsha[:16]} errors {rerr} ({time.time() - t:.0f}s)", flush=True)
        if rsha != out_sha or rerr != errors or info["sizes"] != sizes:
            raise SystemExit(f"reference differs from the oracle: u64mix N={n}")
        case["pinned_by_reference"] = [{"p": p, "out_sha256": rsha, "errors": rerr, "sort_s": info["sort_s"]}]
    return case


def main():
    if not os.path.exists(O.REF_BIN):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "all"], check=True)
    cases = [u32_case(28, 0x5EED0002, [2, 4, 8]), u32_case(30, 0x5EED0003, [8])]
    for n in [(1 << 29) - 3, (1 << 29) - 7]:
        for variant in ["ref", "full"]:
            cases.append(u64_case(n, variant))
    meta = {"generator": "tests/golden/make_golden_large.py",
            "reference": "Parallel-Sorting/src/psort.cc (unmodified) via oracle/_ref/psort_ref, MPICH 3.3.2",
            "cases": cases}
    with open(os.path.join(HERE, "large.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(cases)} large cases written")


if __name__ == "__main__":
    main()
