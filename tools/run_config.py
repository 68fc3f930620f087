#!/usr/bin/env python3
"""Run ONE BASELINE config's default launch N times (for rocprofv3 kernel-trace / --pmc passes; GPU
box only). Usage: python tools/run_config.py <c2|c3|c4|c5|rx|tx|tx2> [reps]
  c2  1 M x 1500 B + 12-B pseudo, DataCalc       c3  16 M x 20-B IPv4 headers, HdrCalc
  c4  1 M packed UDP 40-9000 B + pseudo          c5  16 M x 1500 B + pseudo (one GPU's shard)
  rx / tx  fused Rx / Tx finalize, 1 M x 1500-B IPv4/TCP, strided; tx2 = two-pass Tx
  rx6 / rxmix  fused Rx of the same datagrams as IPv6/TCP / alternating IPv4 and IPv6 (bench_configs)
  crc  CRC-32 CalcCpl of 1 M x 1500-B frames, strided (the library's default CRC form)
Prints the launch description and the mean ms per launch (HIP events), and the algorithmic bytes."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("uc-tcp-ip_amd", "", "tools"):
    sys.path.insert(0, os.path.join(REPO, sub))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import netcsum  # noqa: E402
from bench import SEED, c2_pseudo_headers  # noqa: E402


def main():
    name = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    if name in ("c2", "c5"):
        n, L = (1 << 20) if name == "c2" else (1 << 24), 1500
        seg = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(seg, n * L, SEED, 0)
        ph = torch.from_numpy(c2_pseudo_headers(0, n, L, 12)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_strided(seg, L, L, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
        algo = n * (L + 12 + 2)
    elif name == "c3":
        n, L = 1 << 24, 20
        hdr = torch.empty(n * L, dtype=torch.uint8, device=dev)
        netcsum.fill(hdr, n * L, SEED, 0)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_strided(hdr, L, L, None, 0, 0, n, out, 2, stream=st)  # noqa: E731
        algo = n * (L + 2)
    elif name == "crc":
        n, L = 1 << 20, 1500
        fr = torch.empty(n * L + 64, dtype=torch.uint8, device=dev)
        netcsum.fill(fr, n * L, SEED, 0)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        fn = lambda: netcsum.crc32_strided(fr, L, L, n, out, 1, stream=st)  # noqa: E731
        algo = n * (L + 4)
    elif name == "c4":
        n = 1 << 20
        lens = np.random.default_rng(7).integers(40, 9001, size=n).astype(np.uint16)
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        total = int(off[-1]) + int(lens[-1])
        base = torch.empty(total + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(base, total, SEED, 0)
        off_d = torch.from_numpy(off.view(np.int64)).to(dev)
        len_d = torch.from_numpy(lens.view(np.int16)).to(dev)
        ph = torch.from_numpy(np.random.default_rng(1).integers(0, 256, size=12 * n, dtype=np.uint8)).to(dev)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        fn = lambda: netcsum.batch_varlen(base, off_d, len_d, ph, 12, 12, n, out, 0, stream=st)  # noqa: E731
        algo = total + 12 * n + 2 * n
    else:
        n, L = 1 << 20, 1500
        pk = torch.empty(n * L + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(pk, n * L, SEED, 0)
        v = pk[: n * L].view(n, L)
        v[:, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8,
                                  device=dev)
        flags = torch.zeros(n, dtype=torch.uint8, device=dev)
        if name == "tx2":
            netcsum.tune(netcsum.TUNE_TX_PASSES, 2)
        if name in ("rx6", "rxmix"):
            v[:, 0:8] = torch.tensor([0x60, 0, 0, 0, (L - 40) >> 8, (L - 40) & 0xFF, 6, 64], dtype=torch.uint8,
                                     device=dev)
            if name == "rxmix":
                v[0::2, 0:12] = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0],
                                             dtype=torch.uint8, device=dev)
                v[0::2, 12:20] = 0x0A
            netcsum.tx_finalize_ip(pk, n, flags, stride=L, pkt_len=L, stream=st)
            fn = lambda: netcsum.rx_validate_ip(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
            if name == "rx6":
                fn = lambda: netcsum.rx_validate_ipv6(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
            algo = n * (L + 1)
        elif name == "rx":
            fn = lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=L, pkt_len=L, stream=st)  # noqa: E731
            algo = n * (L + 1)
        else:
            fn = lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=L, pkt_len=L, stream=st)  # noqa: E731
            algo = n * (L + 4)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / reps
    print(f"{name} {netcsum.last_launch()} ms={ms:.4f} algo_bytes={algo} GBps={algo / ms / 1e6:.1f}", flush=True)


if __name__ == "__main__":
    main()
