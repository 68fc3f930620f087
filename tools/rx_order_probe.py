#!/usr/bin/env python3
"""Diagnostic: is the fused-Rx time sensitive to what ran / was allocated before it in the process?"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "oracle", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402
from bench_configs import events_ms  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
n, L = 1 << 20, 1500


def make():
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pk, n * L, SEED, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    fl = torch.zeros(n, dtype=torch.uint8, device=dev)
    netcsum.tx_finalize_ipv4(pk, n, fl, stride=L, pkt_len=L, stream=st)
    torch.cuda.synchronize()
    return pk, fl


def rx(pk, fl, tag):
    ms = events_ms(lambda: netcsum.rx_validate_ipv4(pk, n, fl, stride=L, pkt_len=L, stream=st), st)
    out = torch.empty(n, dtype=torch.int16, device=dev)
    ms2 = events_ms(lambda: netcsum.batch_strided(pk, L, L, None, 0, 0, n, out, 0, stream=st), st)
    print(json.dumps({"tag": tag, "rx_ms": round(ms, 4), "seg_ms": round(ms2, 4),
                      "ptr_mod_2M": pk.data_ptr() % (1 << 21), "kernel": netcsum.last_launch()}), flush=True)


pk, fl = make()
rx(pk, fl, "fresh")
rx(pk, fl, "fresh-again")
big = torch.empty(4741264103 + 256, dtype=torch.uint8, device=dev)
netcsum.fill(big, 4741264103, SEED, 0)
torch.cuda.synchronize()
rx(pk, fl, "after-big-alloc")
del big, pk, fl
torch.cuda.empty_cache()
pk, fl = make()
rx(pk, fl, "realloc-after-big")
pk2 = pk[1:]
rx(pk2, fl, "odd-base")
