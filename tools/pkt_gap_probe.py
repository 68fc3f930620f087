#!/usr/bin/env python3
"""Rx / Tx of 1 M IPv4/TCP datagrams (1500 B) in strided buffers: stride 1500 (packed) up to 1564
(the run-stream kernel's widest gap), the datagram at offset `lead` of each slot, `present` = the
slot's bytes from the datagram on. Isolates what a gap between datagrams costs the run-stream
kernel (the reference's template NET_BUF layout is stride 1520, lead 14). Two interleaved passes."""
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


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    n, L = 1 << 20, 1500
    hdr = torch.tensor([0x45, 0, L >> 8, L & 0xFF, 0, 0, 0x40, 0, 64, 6, 0, 0], dtype=torch.uint8, device=dev)
    flags = torch.zeros(n, dtype=torch.uint8, device=dev)
    cases = [(1500, 0, 1500), (1504, 0, 1500), (1504, 0, 1504), (1520, 0, 1500), (1520, 14, 1506),
             (1520, 16, 1504), (1536, 0, 1536), (1564, 0, 1500)]
    bufs = {}
    for S, lead, present in cases:
        b = torch.empty(n * S + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(b, n * S, SEED, 0)
        b[: n * S].view(n, S)[:, lead:lead + 12] = hdr
        netcsum.tx_finalize_ipv4(b[lead:], n, None, stride=S, pkt_len=present, stream=st)
        bufs[(S, lead, present)] = b
    torch.cuda.synchronize()
    for rep in range(2):
        for key, b in bufs.items():
            S, lead, present = key
            pk = b[lead:]
            rx = events_ms(lambda: netcsum.rx_validate_ipv4(pk, n, flags, stride=S, pkt_len=present, stream=st), st)
            ok = bool(((flags & 0x07) == 0x07).all().item())
            krx = netcsum.last_launch()
            tx = events_ms(lambda: netcsum.tx_finalize_ipv4(pk, n, None, stride=S, pkt_len=present, stream=st), st)
            print(json.dumps({"pass": rep, "stride": S, "lead": lead, "present": present, "rx_ms": round(rx, 4),
                              "tx_ms": round(tx, 4), "rx_all_valid": ok, "kernel_rx": krx}), flush=True)


if __name__ == "__main__":
    main()
