#!/usr/bin/env python3
"""Tx finalize of 1 M x 1500-B datagrams: 2-B field stores against whole 32-B sector write-back
(NETCSUM_TUNE_TX_SECTOR 1 / 2), one and two passes (NETCSUM_TUNE_TX_PASSES), IPv4 packed (stride
1500), the reference's template buffers (stride 1520, IP header at +14), IPv6 and mixed rings; two
interleaved passes. Every form's bytes are compared with the default form's (same input each time).

  python tools/tx_sector_probe.py > gpurun_out/TAG_tx_sector_probe.jsonl

Experiment record: NETCSUM_TUNE_TX_SECTOR existed only in the experiment builds of commits 9306138
(32-B sectors) and 9841321 (64-B sectors, one-pass capture by LDS-DMA = box r4e; the r4c build — the
two-pass 4-lane scatter loading its sectors, one-pass reload — and the r4d build — one-pass capture in
VGPRs — differ from it only in the one-pass path); every form was slower than
the 2-B field stores (profiles/r3s_tx_sector32_probe.jsonl, r3s_tx_sector64_probe.jsonl) and the
option was removed from the product. Run it against one of those builds.
"""
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


def ring(dev, n, S, lead, L, ver):
    """n datagrams of L bytes at stride S (+lead): IPv4/TCP, IPv6/TCP, or alternating."""
    b = torch.empty(n * S + 256, dtype=torch.uint8, device=dev)
    netcsum.fill(b, n * S, SEED, 0)
    v = b[: n * S].view(n, S)[:, lead:]
    h4 = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    pl = L - 40
    h6 = torch.tensor([0x60, 0, 0, 0, pl >> 8, pl & 0xFF, 6, 64], dtype=torch.uint8, device=dev)
    if ver == 4:
        v[:, :12] = h4
    elif ver == 6:
        v[:, :8] = h6
    else:
        v[0::2, :12] = h4
        v[1::2, :8] = h6
    return b


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 1 << 20, 1500
    cases = [("v4_packed", 1500, 0, 4), ("v4_template1520", 1520, 14, 4), ("v6_packed", 1500, 0, 6),
             ("mixed_packed", 1500, 0, 0)]
    fns = {4: netcsum.tx_finalize_ipv4, 6: netcsum.tx_finalize_ipv6, 0: netcsum.tx_finalize_ip}
    for rep in range(2):
        for name, S, lead, ver in cases:
            src = ring(dev, n, S, lead, L, ver)
            ref = None
            for passes in (2, 1):
                for sector in (1, 2):
                    netcsum.tune(netcsum.TUNE_TX_PASSES, passes)
                    netcsum.tune(netcsum.TUNE_TX_SECTOR, sector)
                    work = src.clone()
                    fn = fns[ver]
                    ms = events_ms(lambda: fn(work[lead:], n, None, stride=S, pkt_len=L, stream=st), st)
                    desc = netcsum.last_launch()
                    # bytes: one call on a fresh copy of the source
                    work.copy_(src)
                    fn(work[lead:], n, None, stride=S, pkt_len=L, stream=st)
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = work.clone()
                        same = True
                    else:
                        same = bool(torch.equal(work, ref))
                    print(json.dumps({"pass": rep, "case": name, "stride": S, "lead": lead, "tx_passes": passes,
                                      "tx_sector": sector, "ms": round(ms, 4),
                                      "GBps_algorithmic": round(n * (L + 4) / ms / 1e6, 1),
                                      "bytes_equal_default": same, "kernel": desc}), flush=True)
                    del work
            del src, ref
            torch.cuda.empty_cache()
    netcsum.tune(netcsum.TUNE_TX_PASSES, 0)
    netcsum.tune(netcsum.TUNE_TX_SECTOR, 0)


if __name__ == "__main__":
    main()
