#!/usr/bin/env python3
"""Run ONE packet-batch configuration N times (for rocprofv3 --pmc passes; GPU box only): fused Rx
validation or Tx finalize over 1 M x 1500-B IPv4/TCP datagrams, strided.
Usage: python tools/run_pkt_variant.py <rx|tx> [reps] [nt=0|1] [tile=N]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "uc-tcp-ip_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED  # noqa: E402

KEYS = {"nt": netcsum.TUNE_NT_LOADS, "tile": netcsum.TUNE_TILE,
        "group": netcsum.TUNE_GROUP_LANES}


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    n, L = 1 << 20, 1500
    pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(pk, n * L, SEED, 0)
    v = pk[: n * L].view(n, L)
    v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    netcsum.tx_finalize_ipv4(pk, n, flags, stride=L, pkt_len=L)
    for kv in sys.argv[3:]:
        k, val = kv.split("=")
        netcsum.tune(KEYS[k], int(val))
    for _ in range(reps):
        if name == "rx":
            netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L)
        else:
            netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L)
    torch.cuda.synchronize()
    print(name, sys.argv[3:])


if __name__ == "__main__":
    main()
