#!/usr/bin/env python3
"""Rx / Tx of 1 M IPv4/TCP 1500-B datagrams in NET_BUF-shaped buffers: the default kernel choice
against the lane-group kernel (TUNE_KERNEL 2), two interleaved passes:

  (1520, 14, 1506)  the reference's template large buffers (net_dev_cfg.c:146-149)
  (2048, 64, 1984)  2-KiB buffers, IPv4 header at +64, the rest of the buffer declared present
  (2048, 64, 1500)  the same with only the datagram declared present (run-stream only with mode 2)
  (1500, 0, 1500)   packed, for reference

Prints one JSON line per (pass, layout, kernel). profiles/r3j_netbuf_kernel_probe.jsonl; an
experiment build that skipped the chunks after each datagram's end in slots >= 1 KiB is in
profiles/r3k_netbuf_slack_skip_probe.jsonl (not kept: 2048-B slots Tx -9 %, Rx -2 %, packed Rx +6 %)."""
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
    bufs = {}
    for S, lead in ((1500, 0), (1520, 14), (2048, 64)):
        b = torch.empty(n * S + 256, dtype=torch.uint8, device=dev)
        netcsum.fill(b, n * S, SEED, 0)
        b[: n * S].view(n, S)[:, lead:lead + 12] = hdr
        netcsum.tx_finalize_ipv4(b[lead:], n, None, stride=S, pkt_len=L, stream=st)
        bufs[S] = b
    torch.cuda.synchronize()
    for rep in range(2):
        for S, lead, present in ((1500, 0, 1500), (1520, 14, 1506), (2048, 64, 1984), (2048, 64, 1500)):
            nb = bufs[S][lead:]
            for kern in (0, 2):
                netcsum.tune(netcsum.TUNE_KERNEL, kern)
                rx = events_ms(lambda: netcsum.rx_validate_ipv4(nb, n, flags, stride=S, pkt_len=present, stream=st),
                               st)
                k_rx = netcsum.last_launch()
                ok = bool(((flags & 0x07) == 0x07).all().item())
                tx = events_ms(lambda: netcsum.tx_finalize_ipv4(nb, n, None, stride=S, pkt_len=present, stream=st),
                               st)
                print(json.dumps({"pass": rep, "stride": S, "lead": lead, "present": present, "tune_kernel": kern,
                                  "rx_ms": round(rx, 4), "tx_ms": round(tx, 4), "rx_all_valid": ok,
                                  "rx_GBps_algorithmic": round(n * (L + 1) / rx / 1e6, 1),
                                  "tx_GBps_algorithmic": round(n * (L + 4) / tx / 1e6, 1),
                                  "kernel_rx": k_rx, "kernel_tx": netcsum.last_launch()}), flush=True)
            netcsum.tune(netcsum.TUNE_KERNEL, 0)


if __name__ == "__main__":
    main()
