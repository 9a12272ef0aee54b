#!/usr/bin/env python3
"""Exchange codec on sorted runs of the sizes a compare-split stage sends
(N/P/2 keys at P = 2, 4, 8 for 2^30 keys): encode/decode time, coded size,
round-trip check.  python tools/codec_probe.py > gpurun_out/codec.jsonl"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parallel-computing-mpi_amd"))
import torch  # noqa: E402
import misort  # noqa: E402

ctx = misort.Context(0)
for dt, kb in (("u32", 4), ("u64", 8)):
    for logk in (26, 27, 28):
        k = 1 << logk
        if dt == "u64" and logk == 28:
            continue
        t = torch.int32 if kb == 4 else torch.int64
        full = torch.empty(2 * k, dtype=t, device="cuda")
        ctx.fill_splitmix(full, 0x5EED0003)  # the block a rank holds: 2k keys, k of them cross
        srt = torch.empty_like(full)
        ctx.local_sort(full, srt)
        run = srt[k // 2: k // 2 + k].contiguous()  # a sorted run of k keys
        dec = torch.empty_like(run)
        enc_ms, dec_ms, nbytes = ctx.codec_probe(run, dec)
        ok = bool(torch.equal(run, dec))
        raw = k * kb
        print(json.dumps({"dtype": dt, "keys": k, "raw_MiB": raw / 2**20, "coded_MiB": nbytes / 2**20,
                          "ratio": raw / nbytes, "encode_ms": enc_ms, "decode_ms": dec_ms,
                          "xgmi_raw_ms_at_64GBs": raw / 64e9 * 1e3, "xgmi_coded_ms_at_64GBs": nbytes / 64e9 * 1e3,
                          "roundtrip_ok": ok}), flush=True)
        assert ok
ctx.close()
